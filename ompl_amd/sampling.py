"""The reference's input streams: RNG seed generator + uniform state samplers (C ABI,
ompl_amd/csrc/sampler.cpp), mirroring the reference's calls:

  set_seed(42)                      ompl::RNG::setSeed(42)          util/src/RandomNumbers.cpp:213-216
  s = StateSampler(space)           space->allocStateSampler()      base/src/StateSpace.cpp:800-806, :1118-1128
  s.sample_uniform(n)               n x sampler->sampleUniform(st)  base/src/StateSampler.cpp:47-52

Every StateSampler draws its RNG seeds from the process-wide seed generator at construction
(SE3: compound + R^3 + SO3 = 3 seeds), so the order of construction after set_seed decides
the streams, exactly as in the reference.
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from . import abi
from .spaces import KinematicChainSpace, RealVectorStateSpace, SE3StateSpace, StateSpace


def set_seed(seed: int) -> None:
    abi.lib.ompl_gpu_rng_set_seed(int(seed))


def get_seed() -> int:
    return int(abi.lib.ompl_gpu_rng_get_seed())


def next_seed() -> int:
    """The seed an RNG() constructed now would take (drawn from the generator), for mirroring an
    RNG that lives outside this library (a planner's rng_, GNAT's pivot selector)."""
    return int(abi.lib.ompl_gpu_rng_next_seed())


def seeds_drawn() -> int:
    """Seeds the process-wide generator has handed out (RNG() constructions)."""
    return int(abi.lib.ompl_gpu_rng_seeds_drawn())


class StateSampler(abi.Handle):
    """allocStateSampler() of `space`; bounds of the R^n part from the space descriptor."""

    _destroy_fn = "ompl_gpu_sampler_destroy"

    def __init__(self, space: StateSpace):
        self.space = space
        s = space.to_abi()
        lo = hi = None
        if isinstance(space, (RealVectorStateSpace, SE3StateSpace, KinematicChainSpace)):
            lo = np.ascontiguousarray(space.low, dtype=np.float64)
            hi = np.ascontiguousarray(space.high, dtype=np.float64)
        h = C.c_void_p()
        abi.check(abi.lib.ompl_gpu_sampler_create(C.byref(h), C.byref(s), abi.dptr(lo) if lo is not None else None,
                                                  abi.dptr(hi) if hi is not None else None))
        self._own(h)

    def sample_uniform(self, n: int) -> np.ndarray:
        out = np.empty((int(n), self.space.dim), dtype=np.float64)
        abi.check(abi.lib.ompl_gpu_sampler_sample_uniform(self._h, int(n), abi.dptr(out)))
        return out

    def local_seeds(self) -> list:
        seeds = (C.c_uint32 * 3)()
        cnt = C.c_int(0)
        abi.check(abi.lib.ompl_gpu_sampler_local_seeds(self._h, seeds, C.byref(cnt)))
        return [int(seeds[i]) for i in range(cnt.value)]


def rng_uniform(local_seed: int, n: int, low: float = 0.0, high: float = 1.0) -> np.ndarray:
    """n x RNG(local_seed).uniformReal(low, high): an RNG with an explicit local seed
    (RandomNumbers.cpp:225-228) draws nothing from the seed generator."""
    out = np.empty(int(n), dtype=np.float64)
    abi.check(abi.lib.ompl_gpu_rng_uniform_real(int(local_seed), int(n), float(low), float(high), abi.dptr(out)))
    return out
