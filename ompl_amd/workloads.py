"""Synthetic inputs of the BASELINE.json configurations.

reference_states() draws from the reference's own streams (ompl_amd.sampling: RNG::setSeed, then
one allocStateSampler() per array in order, RandomNumbers.cpp:53-279, StateSpace.cpp:800-806,
:1118-1128) — what the bench and the golden fixtures use.  The numpy samplers below restate the
same distributions with numpy's generator, for tests whose inputs only need to be arbitrary
(parity is defined on identical inputs, which the tests feed to both sides):
  uniform R^n in bounds          RealVectorStateSampler::sampleUniform (RealVectorStateSpace.cpp:45-53)
  uniform SO3, Shoemake          RNG::quaternion (util/src/RandomNumbers.cpp:263-279)
  SE3 = uniform R^3 x SO3        CompoundStateSampler::sampleUniform (base/src/StateSampler.cpp:47-52)
Environments:
  createHornEnvironment(d, eps)  demos/KinematicChain.h:279-315
  sphere field                   32 spheres, r = 0.1, centres from RNG(7)
"""
from __future__ import annotations

import math

import numpy as np


def uniform_rv(rng: np.random.Generator, n: int, dim: int, low=0.0, high=1.0) -> np.ndarray:
    return rng.uniform(low, high, size=(n, dim))


def uniform_quat(rng: np.random.Generator, n: int) -> np.ndarray:
    x0 = rng.random(n)
    r1, r2 = np.sqrt(1.0 - x0), np.sqrt(x0)
    t1 = 2.0 * math.pi * rng.random(n)
    t2 = 2.0 * math.pi * rng.random(n)
    return np.column_stack([np.sin(t1) * r1, np.cos(t1) * r1, np.sin(t2) * r2, np.cos(t2) * r2])


def uniform_se3(rng: np.random.Generator, n: int, low=0.0, high=1.0) -> np.ndarray:
    return np.ascontiguousarray(np.column_stack([rng.uniform(low, high, size=(n, 3)), uniform_quat(rng, n)]))


def uniform_chain(rng: np.random.Generator, n: int, links: int) -> np.ndarray:
    return rng.uniform(-math.pi, math.pi, size=(n, links))


def horn_environment(d: int, eps: float) -> np.ndarray:
    """createHornEnvironment (demos/KinematicChain.h:279-315), segments (x0,y0,x1,y1)."""
    env = []
    w = 1.0 / float(d)
    x, y, theta = w, -eps, 0.0
    scale = w * (1.0 + math.pi * eps)
    for _ in range(d - 1):
        theta += math.pi / float(d)
        xN = x + math.cos(theta) * scale
        yN = y + math.sin(theta) * scale
        env.append((x, y, xN, yN))
        x, y = xN, yN
    theta, x, y = 0.0, w, eps
    scale = w * (1.0 - math.pi * eps)
    for _ in range(d - 1):
        theta += math.pi / d
        xN = x + math.cos(theta) * scale
        yN = y + math.sin(theta) * scale
        env.append((x, y, xN, yN))
        x, y = xN, yN
    return np.array(env, dtype=np.float64)


def sphere_field(count: int = 32, radius: float = 0.1, seed: int = 7, low=0.0, high=1.0):
    """count sphere centres = 3 * count successive RNG(seed).uniformReal(low, high) draws."""
    from . import sampling

    c = sampling.rng_uniform(seed, 3 * count, low, high).reshape(count, 3)
    return np.ascontiguousarray(c), np.full(count, radius)


def reference_states(space, counts, seed: int = 42):
    """RNG::setSeed(seed); then for each n in counts: sampler = space.allocStateSampler(),
    n x sampler.sampleUniform().  Returns one array per count."""
    from . import sampling

    sampling.set_seed(seed)
    out = []
    for n in counts:
        out.append(sampling.StateSampler(space).sample_uniform(int(n)))
    return out


def reference_valid_states(space, n: int, is_valid, seed: int = 42, chunk: int = 1_000_000, sampler=None):
    """The first n valid states of one sampler's uniform stream — what the reference's
    UniformValidStateSampler yields in order (rejection, ValidStateSampler attempts), since an
    invalid draw is simply followed by the next one.  Pass `sampler` to continue a stream."""
    from . import sampling

    if sampler is None:
        sampling.set_seed(seed)
        sampler = sampling.StateSampler(space)
    parts, have = [], 0
    while have < n:
        x = sampler.sample_uniform(chunk)
        x = x[np.asarray(is_valid(x), dtype=bool)]
        parts.append(x[: n - have])
        have += len(parts[-1])
    return np.ascontiguousarray(np.concatenate(parts)), sampler


def rrt_star_k(n: int, d: int) -> int:
    """k_rrt * log(n+1), k_rrt = 1.1 * 2^(d+1) e (1 + 1/d)  (RRTstar.cpp:609, :1147-1159)."""
    k_rrt = 1.1 * (2.0 ** (d + 1) * math.e * (1.0 + 1.0 / d))
    return int(math.ceil(k_rrt * math.log(n + 1)))


def prm_star_k(n: int, d: int) -> int:
    """ceil((e + e/d) log n)  (ConnectionStrategy.h:141-149)."""
    return int(math.ceil((math.e + math.e / d) * math.log(n)))


def unit_ball_measure(d: int) -> float:
    """Volume of the unit d-ball (util/src/GeometricEquations.cpp:55-60)."""
    return math.pi ** (d / 2.0) / math.gamma(d / 2.0 + 1.0)


def bitstar_radius(n: int, d: int, measure: float, rewire: float = 1.1) -> float:
    """BIT* radius r = rewire * r_RGG,min * (ln n / n)^(1/d), r_RGG,min = (2 (1 + 1/d) measure / zeta_d)^(1/d)
    (ImplicitGraph.cpp:1372-1381, :1389-1400).  SE(3) over [0,1]^3: d = 6, measure = 1 * pi^2
    (SO3StateSpace.cpp:171-175) -> 0.1528 at n = 1e7."""
    r_rgg = (2.0 * (1.0 + 1.0 / d) * (measure / unit_ball_measure(d))) ** (1.0 / d)
    return rewire * r_rgg * (math.log(n) / n) ** (1.0 / d)
