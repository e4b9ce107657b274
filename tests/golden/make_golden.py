"""Generate the committed golden fixtures in tests/golden/ (run in the build container,
where /root/reference exists):

    python tests/golden/make_golden.py

Inputs are drawn from the reference's RNG streams (RNG::setSeed(42) / (7), one
allocStateSampler() per array: ompl_amd.workloads.reference_states, checked bit for bit
against the oracle's restatement in tests/test_rng.py).

nn_*.npz     : inputs + nearestK / nearestR results of the REFERENCE's own
               NearestNeighborsLinear.h (compiled unmodified into oracle/_ref/ by
               oracle/Makefile), with the oracle's restated metric as distance.
motion_*.npz : inputs + validity bits / nd / first-invalid / isValid-call counts of the
               oracle restatement of DiscreteMotionValidator (the reference motion
               validator cannot be compiled here: it needs Boost).
               Regression pins: "parity pinned by restatement".
circles2d.npz: the reference test resources tests/resources/circle_obstacles.txt and
               circle_queries.txt as arrays (data files of the reference's tests).
"""
from __future__ import annotations

import math
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))

import pyoracle as O  # noqa: E402
from ompl_amd import sampling as S  # noqa: E402
from ompl_amd import workloads as W  # noqa: E402
from ompl_amd.checkers import (Circles2DChecker, HypercubeChecker, KinematicChainChecker,  # noqa: E402
                               SpheresChecker)
from ompl_amd.spaces import (KinematicChainSpace, RealVectorStateSpace, SE3StateSpace,  # noqa: E402
                             SO3StateSpace)

REF = "/root/reference"


def spaces():
    return {
        "r6": RealVectorStateSpace(6),
        "se3": SE3StateSpace(),
        "so3": SO3StateSpace(),
        "chain12": KinematicChainSpace(12, 1.0 / 12),
    }


def make_nn():
    assert O.ref is not None, "oracle/_ref/libref_linear.so missing: run `make -C oracle` first"
    for name, sp in spaces().items():
        data, q = W.reference_states(sp, (3000, 64), seed=42)  # setSeed(42): data sampler, query sampler
        q[0] = data[17]  # a query that is stored: reference returns it first at d=0
        out = {"data": data, "queries": q}
        for k in (1, 10, 41):
            ids, d, cnt = O.ref_knn(sp, data, q, k)
            out[f"knn{k}_ids"], out[f"knn{k}_dist"], out[f"knn{k}_cnt"] = ids, d, cnt
        r = float(np.median(out["knn10_dist"][:, 9]))  # about ten hits per query
        off, ids = O.ref_radius(sp, data, q, r)
        out.update({"radius": np.array(r), "radius_off": off, "radius_ids": ids})
        np.savez_compressed(os.path.join(HERE, f"nn_{name}.npz"), **out)
        print(f"nn_{name}.npz: radius {r:.4f}, {int(off[-1])} hits")


def circles_data():
    obs, qs = [], []
    with open(os.path.join(REF, "tests/resources/circle_obstacles.txt")) as f:
        for line in f.readlines()[2:]:
            p = line.split()
            if len(p) >= 4:
                obs.append([float(p[1]), float(p[2]), float(p[3])])
    with open(os.path.join(REF, "tests/resources/circle_queries.txt")) as f:
        rows = [line.split() for line in f if line.strip()]
    for i in range(0, len(rows) - 1, 2):
        qs.append([float(rows[i][2]), float(rows[i][3]), float(rows[i + 1][2]), float(rows[i + 1][3])])
    return np.array(obs), np.array(qs)


def _perturb(local_seed, shape, scale):
    """Symmetric perturbations in [-scale, scale) from RNG(local_seed).uniformReal."""
    n = int(np.prod(shape))
    return (S.rng_uniform(local_seed, n, -scale, scale)).reshape(shape)


def make_motion():
    cases = {}
    # SE3 + hypercube on the translation (HypercubeBenchmark predicate, 3 dims)
    sp = SE3StateSpace()
    a, b, a2, b2 = W.reference_states(sp, (2000, 2000, 2000, 2000), seed=7)
    # bias half of the endpoints into the valid passage so both outcomes occur
    a[:1000, :3] = np.clip(a[:1000, :3] * 0.1, 0, 1)
    b[:1000, :3] = np.clip(a[:1000, :3] + _perturb(71, (1000, 3), 0.08), 0, 1)
    cases["se3_hypercube"] = (sp, HypercubeChecker(3, 0.1), a, b)
    c, r = W.sphere_field(32, 0.1, 7)
    cases["se3_spheres"] = (sp, SpheresChecker(c, r), a2, b2)
    # R6 hypercube at the demo's resolution 0.001 (HypercubeBenchmark.cpp:97)
    sp6 = RealVectorStateSpace(6)
    sp6.setLongestValidSegmentFraction(0.001)
    (a3,) = W.reference_states(RealVectorStateSpace(6, 0.0, 0.12), (2000,), seed=7)
    b3 = np.clip(a3 + _perturb(72, (2000, 6), 0.08), 0, 1)
    cases["r6_hypercube"] = (sp6, HypercubeChecker(6, 0.1), a3, b3)
    # kinematic chain, horn environment (KinematicChainBenchmark.cpp:48-49)
    spc = KinematicChainSpace(12, 1.0 / 12)
    env = W.horn_environment(12, math.log(12.0) / 12.0)
    ck = KinematicChainChecker(env)
    a4, _ = W.reference_valid_states(spc, 1000, lambda x: O.is_valid(spc, ck, x), seed=7, chunk=20000)  # s1 valid
    b4 = np.mod(a4 + _perturb(73, (1000, 12), 0.25) + math.pi, 2 * math.pi) - math.pi
    cases["chain12_horn"] = (spc, ck, a4, b4)
    # circles 2-D: reference obstacles, resolution 0.002 (2DcirclesSetup.h:79-90)
    obs, qs = circles_data()
    np.savez_compressed(os.path.join(HERE, "circles2d.npz"), obstacles=obs, queries=qs)
    spr = RealVectorStateSpace(2, 0.0, 100.0)
    spr.setLongestValidSegmentFraction(0.002)
    ra, rb = W.reference_states(spr, (2000, 2000), seed=7)
    a5 = np.concatenate([qs[:, 0:2], ra])
    b5 = np.concatenate([qs[:, 2:4], rb])
    cases["r2_circles"] = (spr, Circles2DChecker(obs), a5, b5)
    for name, (sp_, ck, s1, s2) in cases.items():
        valid, nd, fi, checks = O.check_motions(sp_, ck, s1, s2)
        sv = O.is_valid(sp_, ck, s2)
        np.savez_compressed(os.path.join(HERE, f"motion_{name}.npz"), s1=s1, s2=s2, valid=valid, nd=nd,
                            first_invalid=fi, checks=np.array(checks), s2_valid=sv)
        print(f"motion_{name}.npz: {valid.mean():.3f} valid, mean nd {nd.mean():.1f}, {checks} isValid calls")


if __name__ == "__main__":
    make_nn()
    make_motion()
