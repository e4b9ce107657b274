"""The reference's input streams: ompl::RNG's seed generator and the uniform
state samplers, restated twice — in the product (ompl_amd/csrc/sampler.cpp, used for the bench
and fixture inputs) and in the oracle (oracle/rng.cpp) — and pinned by the C++ standard's
known answers for the two engines the reference uses (RandomNumbers.cpp:53-113, RandomNumbers.h:190-192)."""
import math

import numpy as np
import pytest

import pyoracle as O
from ompl_amd import sampling as S
from ompl_amd.spaces import KinematicChainSpace, RealVectorStateSpace, SE3StateSpace, SO3StateSpace


def test_engine_known_answers():
    # [rand.predef]: 10000th invocation of a default-constructed engine
    assert O.lib.oracle_mt19937_10000th() == 4123659995
    assert O.lib.oracle_ranlux24_base_10000th() == 7937952


def test_seed_stream_matches_oracle():
    S.set_seed(42)
    want = O.seed_stream(42, 7)
    d0 = S.seeds_drawn()
    se3 = S.StateSampler(SE3StateSpace())        # compound + R^3 + SO3
    rv = S.StateSampler(RealVectorStateSpace(6))  # one
    so3 = S.StateSampler(SO3StateSpace())        # one
    ch = S.StateSampler(KinematicChainSpace(12, 1 / 12))
    assert S.seeds_drawn() - d0 == 6
    got = se3.local_seeds() + rv.local_seeds() + so3.local_seeds() + ch.local_seeds()
    assert got == [int(x) for x in want[:6]]
    assert all(1 <= s <= 1_000_000_000 for s in got)


@pytest.mark.parametrize("name", ["se3", "r6", "so3", "chain12", "se3_box"])
def test_samples_match_oracle_bitwise(name):
    sp = {"se3": SE3StateSpace(), "r6": RealVectorStateSpace(6), "so3": SO3StateSpace(),
          "chain12": KinematicChainSpace(12, 1 / 12), "se3_box": SE3StateSpace(-1.0, 1.0)}[name]
    S.set_seed(42)
    s = S.StateSampler(sp)
    x = s.sample_uniform(5000)
    ref = O.sample_uniform(sp, s.local_seeds(), 5000)
    np.testing.assert_array_equal(x, ref)
    lo, hi = (np.array(sp.low), np.array(sp.high)) if hasattr(sp, "low") else (None, None)
    if lo is not None:
        nrn = len(lo)
        assert (x[:, :nrn] >= lo).all() and (x[:, :nrn] < hi).all()
    if name in ("se3", "so3", "se3_box"):
        q = x[:, -4:]
        np.testing.assert_allclose(np.linalg.norm(q, axis=1), 1.0, atol=1e-12)


def test_streams_are_deterministic_and_ordered():
    S.set_seed(42)
    a = S.StateSampler(SE3StateSpace()).sample_uniform(100)
    b = S.StateSampler(SE3StateSpace()).sample_uniform(100)
    S.set_seed(42)
    a2 = S.StateSampler(SE3StateSpace()).sample_uniform(100)
    np.testing.assert_array_equal(a, a2)
    assert not np.array_equal(a, b)  # the second sampler draws the next seeds


def test_explicit_local_seed():
    d0 = S.seeds_drawn()
    x = S.rng_uniform(7, 96)
    assert S.seeds_drawn() == d0  # RNG(localSeed) draws no seed
    ref = O.sample_uniform(RealVectorStateSpace(1), [7], 96)
    np.testing.assert_array_equal(x, ref[:, 0])
    assert math.isclose(float(np.mean(x)), 0.5, abs_tol=0.1)
