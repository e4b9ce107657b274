"""GPU parity tests of the motion-validation path (through the C ABI): validity bits,
segment counts, first-invalid samples and isValid-call counts must be identical to the
oracle restatement of DiscreteMotionValidator and to the golden fixtures."""
import math

import numpy as np
import pytest

import pyoracle as O
from ompl_amd import DiscreteMotionValidatorGPU
from ompl_amd import workloads as W
from ompl_amd.checkers import (AllValidChecker, Circles2DChecker, HypercubeChecker, KinematicChainChecker,
                               SpheresChecker)
from ompl_amd.spaces import KinematicChainSpace, RealVectorStateSpace, SE3StateSpace

pytestmark = pytest.mark.gpu


def _case(name, golden):
    if name == "se3_hypercube":
        return SE3StateSpace(), HypercubeChecker(3, 0.1)
    if name == "se3_spheres":
        c, r = W.sphere_field(32, 0.1, 7)
        return SE3StateSpace(), SpheresChecker(c, r)
    if name == "r6_hypercube":
        sp = RealVectorStateSpace(6)
        sp.setLongestValidSegmentFraction(0.001)
        return sp, HypercubeChecker(6, 0.1)
    if name == "chain12_horn":
        return KinematicChainSpace(12, 1.0 / 12), KinematicChainChecker(W.horn_environment(12, math.log(12.0) / 12.0))
    sp = RealVectorStateSpace(2, 0.0, 100.0)
    sp.setLongestValidSegmentFraction(0.002)
    return sp, Circles2DChecker(golden("circles2d.npz")["obstacles"])


@pytest.mark.parametrize("name", ["se3_hypercube", "se3_spheres", "r6_hypercube", "chain12_horn", "r2_circles"])
def test_motion_golden(gpu, golden, name):
    g = golden(f"motion_{name}.npz")
    sp, ck = _case(name, golden)
    mv = DiscreteMotionValidatorGPU(sp, ck, gpu)
    valid, nd, fi = mv.checkMotions(g["s1"], g["s2"], want_nd=True, want_first_invalid=True)
    np.testing.assert_array_equal(nd, g["nd"])
    np.testing.assert_array_equal(valid, g["valid"])
    np.testing.assert_array_equal(fi, g["first_invalid"])
    assert mv.getValidMotionCount() == int(g["valid"].sum())
    assert mv.getInvalidMotionCount() == int((~g["valid"]).sum())
    assert mv.stateChecks() == int(g["checks"])  # same isValid() work as the FIFO bisection
    np.testing.assert_array_equal(mv.isValid(g["s2"]), g["s2_valid"])
    mv.resetMotionCounter()
    assert mv.getValidMotionCount() == 0 and mv.getInvalidMotionCount() == 0


def test_motion_random_vs_oracle(gpu):
    rng = np.random.default_rng(21)
    sp = SE3StateSpace()
    c, r = W.sphere_field(32, 0.1, 7)
    ck = SpheresChecker(c, r)
    a, b = W.uniform_se3(rng, 100000), W.uniform_se3(rng, 100000)
    mv = DiscreteMotionValidatorGPU(sp, ck, gpu)
    valid, nd, fi = mv.checkMotions(a, b, want_nd=True, want_first_invalid=True)
    ov, ond, ofi, checks = O.check_motions(sp, ck, a, b)
    np.testing.assert_array_equal(nd, ond)
    np.testing.assert_array_equal(valid, ov)
    np.testing.assert_array_equal(fi, ofi)
    assert mv.stateChecks() == checks


def test_motion_edge_cases(gpu):
    sp = SE3StateSpace()
    mv = DiscreteMotionValidatorGPU(sp, AllValidChecker(), gpu)
    rng = np.random.default_rng(3)
    a = W.uniform_se3(rng, 10)
    v, nd = mv.checkMotions(a, a, want_nd=True)           # s1 == s2: nd = 0, s2 checked only
    assert v.all() and (nd == 0).all()
    assert mv.checkMotion(a[0], a[1]) is True
    ok, t = mv.checkMotion(a[0], a[1], lastValid=True)
    assert ok and t is None
    hc = DiscreteMotionValidatorGPU(sp, HypercubeChecker(3, 0.1), gpu)
    s1 = np.array([0.05, 0.05, 0.05, 0, 0, 0, 1.0])
    s2 = np.array([0.5, 0.5, 0.5, 0, 0, 0, 1.0])        # s2 invalid
    ok, t = hc.checkMotion(s1, s2, lastValid=True)
    _, ond, ofi, _ = O.check_motions(sp, HypercubeChecker(3, 0.1), s1[None], s2[None])
    assert not ok and t == (ofi[0] - 1) / ond[0]
    assert hc.checkMotions(np.zeros((0, 7)), np.zeros((0, 7))).shape == (0,)


def test_state_validity_random(gpu):
    rng = np.random.default_rng(4)
    sp = KinematicChainSpace(12, 1.0 / 12)
    ck = KinematicChainChecker(W.horn_environment(12, math.log(12.0) / 12.0))
    x = W.uniform_chain(rng, 50000, 12)
    mv = DiscreteMotionValidatorGPU(sp, ck, gpu)
    np.testing.assert_array_equal(mv.isValid(x), O.is_valid(sp, ck, x))


@pytest.mark.parametrize("name", ["se3", "so3", "r6", "chain12"])
@pytest.mark.parametrize("count,endpoints", [(0, True), (0, False), (1, True), (7, False), (12, True)])
def test_get_motion_states(gpu, name, count, endpoints):
    """SpaceInformation::getMotionStates (SpaceInformation.cpp:201-275, alloc = true) on the
    device against the oracle: same number of states, endpoints copied, interior samples at
    j / (count + 1), bit-identical in every space (SO3 / SE3 slerp: glibc's own acos and sin on
    the device)."""
    from ompl_amd.spaces import SO3StateSpace
    rng = np.random.default_rng(91)
    sp = {"se3": SE3StateSpace, "so3": SO3StateSpace, "r6": lambda: RealVectorStateSpace(6),
          "chain12": lambda: KinematicChainSpace(12, 1.0 / 12)}[name]()
    sample = {"se3": lambda n: W.uniform_se3(rng, n), "so3": lambda n: W.uniform_quat(rng, n),
              "r6": lambda n: W.uniform_rv(rng, n, 6), "chain12": lambda n: W.uniform_chain(rng, n, 12)}[name]
    a, b = sample(300), sample(300)
    a[:3] = b[:3]  # zero-length motions
    mv = DiscreteMotionValidatorGPU(sp, AllValidChecker(), gpu)
    got = mv.getMotionStates(a, b, count, endpoints)
    want = O.motion_states(sp, a, b, count, endpoints)
    assert got.shape == want.shape == (300, count + (2 if endpoints else 0), sp.dim)
    np.testing.assert_array_equal(got, want)
    if endpoints:
        np.testing.assert_array_equal(got[:, 0], a)
        np.testing.assert_array_equal(got[:, -1], b)


def test_motion_states_count_limit(gpu):
    """count near UINT32_MAX: the states-per-motion arithmetic must not wrap (the call is
    rejected with OMPL_GPU_ERR_INVALID_ARG instead of returning OK with nothing written)."""
    import ctypes as C

    from ompl_amd import abi
    sp = RealVectorStateSpace(2)
    mv = DiscreteMotionValidatorGPU(sp, AllValidChecker(), gpu)
    a = np.zeros((1, 2))
    out = np.zeros(8)
    for count in (0xFFFFFFFE, 0xFFFFFFFF):
        st = abi.lib.ompl_gpu_mv_motion_states(mv._h, abi.dptr(a), abi.dptr(a), 1, count, 1, abi.dptr(out))
        assert st == abi.ERR_INVALID_ARG


@pytest.mark.parametrize("name", ["se3_hypercube", "se3_spheres", "r6_hypercube", "chain12_horn", "r2_circles"])
def test_motion_golden_bench_path(gpu, golden, name):
    """The planner / bench call (no nd, no first-invalid): the lane-per-sample kernel (fixed widths:
    a wave's samples laid end to end; the KinematicChain's thread-per-edge walk) gives the golden
    validity bits and the FIFO bisection's isValid-call count (DiscreteMotionValidator.cpp:93-145)."""
    g = golden(f"motion_{name}.npz")
    sp, ck = _case(name, golden)
    mv = DiscreteMotionValidatorGPU(sp, ck, gpu)
    np.testing.assert_array_equal(mv.checkMotions(g["s1"], g["s2"]), g["valid"])
    assert mv.stateChecks() == int(g["checks"])
    mv2 = DiscreteMotionValidatorGPU(sp, ck, gpu)
    valid, nd = mv2.checkMotions(g["s1"], g["s2"], want_nd=True)
    np.testing.assert_array_equal(valid, g["valid"])
    np.testing.assert_array_equal(nd, g["nd"])
    assert mv2.stateChecks() == int(g["checks"])


def test_chain_motion_random_vs_oracle(gpu):
    """KinematicChain motions (PRM*'s, about half invalid) on the bench path (no nd / lastValid): bits
    and the isValid count equal the oracle's FIFO bisection; long edges (up to 41 segments) included."""
    rng = np.random.default_rng(23)
    sp = KinematicChainSpace(12, 1.0 / 12)
    ck = KinematicChainChecker(W.horn_environment(12, math.log(12.0) / 12.0))
    a = W.uniform_chain(rng, 60000, 12)
    b = a + rng.normal(scale=0.05, size=a.shape) * rng.integers(1, 20, size=(len(a), 1))
    b = np.mod(b + np.pi, 2 * np.pi) - np.pi
    ok = O.is_valid(sp, ck, a)
    a, b = a[ok], b[ok]
    mv = DiscreteMotionValidatorGPU(sp, ck, gpu)
    valid = mv.checkMotions(a, b)
    ov, ond, _, checks = O.check_motions(sp, ck, a, b)
    np.testing.assert_array_equal(valid, ov)
    assert mv.stateChecks() == checks
    assert 0.2 < ov.mean() < 0.9 and ond.max() >= 32


def test_sphere_screen_knife_edge(gpu):
    """Interior samples within ~1e-9 .. 1e-5 (relative) of a sphere surface: the packed fp32 sphere
    screen must hand every ambiguous sample to the fp64 test, so bits and counts equal the oracle's."""
    rng = np.random.default_rng(24)
    sp = SE3StateSpace()
    c, r = W.sphere_field(32, 0.1, 7)
    ck = SpheresChecker(c, r)
    n = 40000
    k = rng.integers(0, len(c), n)
    u = rng.normal(size=(n, 3))
    u /= np.linalg.norm(u, axis=1, keepdims=True)
    delta = rng.choice([-1e-5, -1e-7, -1e-9, 0.0, 1e-9, 1e-7, 1e-5], n)
    m = c[k] + u * (r[k] * (1 + delta))[:, None]           # a point at the surface (+- delta)
    tng = np.cross(u, rng.normal(size=(n, 3)))
    tng /= np.linalg.norm(tng, axis=1, keepdims=True)
    half = (0.02 + 0.08 * rng.random(n))[:, None] * tng
    q = W.uniform_se3(rng, n)[:, 3:]
    s1 = np.hstack([m - half, q])
    s2 = np.hstack([m + half, q])                           # the t = 1/2 sample sits on m
    mv = DiscreteMotionValidatorGPU(sp, ck, gpu)
    valid = mv.checkMotions(s1, s2)
    ov, ond, ofi, checks = O.check_motions(sp, ck, s1, s2)
    np.testing.assert_array_equal(valid, ov)
    assert mv.stateChecks() == checks
    v2, nd, fi = DiscreteMotionValidatorGPU(sp, ck, gpu).checkMotions(s1, s2, want_nd=True, want_first_invalid=True)
    np.testing.assert_array_equal(v2, ov)
    np.testing.assert_array_equal(nd, ond)
    np.testing.assert_array_equal(fi, ofi)
