"""PRM* roadmap construction on the device, causal batches: milestone i
connects to its k_i = ceil((e + e/d) ln(i + 1)) nearest among every earlier vertex
(PRM.cpp:562-596, ConnectionStrategy.h:145-149) and each edge is checked with checkMotion.
The device answers a batch at once — the stored part by the batched kNN, the in-batch part by
a causal scan — and must equal the oracle's sequential loop vertex by vertex: same neighbours
in the same (distance, id) order, same edge validity."""
import math

import numpy as np
import pytest

import pyoracle as O
from ompl_amd import DiscreteMotionValidatorGPU, NearestNeighborsGPU
from ompl_amd import workloads as W
from ompl_amd.checkers import KinematicChainChecker, SpheresChecker, AllValidChecker
from ompl_amd.spaces import KinematicChainSpace, RealVectorStateSpace, SE3StateSpace

pytestmark = pytest.mark.gpu


def _run(sp, ck, states, batches, gpu):
    kc = math.e + math.e / sp.getDimension()  # PRM.cpp:195-198: KStarStrategy(..., si_->getStateDimension())
    k_cap = max(1, int(math.ceil(kc * math.log(len(states)))))
    nn = NearestNeighborsGPU(sp, gpu)
    mv = DiscreteMotionValidatorGPU(sp, ck, gpu)
    got_n, got_c, got_v, edges = [], [], [], 0
    at = 0
    for b in batches:
        n, c, v, e = nn.prm_add_milestones(mv, states[at:at + b], kc, k_cap)
        got_n.append(n)
        got_c.append(c)
        got_v.append(v)
        edges += e
        at += b
    assert at == len(states) and nn.size() == len(states)
    on, oc, ov = O.prm_causal(sp, ck, states, kc, k_cap)
    gn, gc, gv = np.concatenate(got_n), np.concatenate(got_c), np.concatenate(got_v)
    np.testing.assert_array_equal(gc, oc)
    np.testing.assert_array_equal(gn, on)
    np.testing.assert_array_equal(gv, ov.astype(bool))
    assert edges == int(oc.sum())
    nv, ni = mv.getValidMotionCount(), mv.getInvalidMotionCount()
    assert nv + ni == edges and nv == int(ov.sum())
    return gc


def test_prm_star_se3_spheres(gpu):
    sp = SE3StateSpace()
    c, r = W.sphere_field(32, 0.1, 7)
    ck = SpheresChecker(c, r)
    states, _ = W.reference_valid_states(sp, 3000, lambda x: O.is_valid(sp, ck, x), seed=42, chunk=6000)
    cnt = _run(sp, ck, states, (700, 300, 1000, 1000), gpu)  # the first batch starts from an empty roadmap
    assert cnt[0] == 0 and cnt[-1] == math.ceil((math.e + math.e / 6) * math.log(3000))


def test_prm_star_long_segments(gpu):
    """A first batch of 1,500 milestones on an empty roadmap: milestone j's stored list is empty,
    so every earlier milestone is an in-batch candidate and the longest segment (1,499 entries)
    exceeds the LDS rank sort's 1,024 (kernels.h kRankSortMax) — the two stable radix passes sort
    the segments instead; then a second batch over the stored 1,500."""
    sp = SE3StateSpace()
    c, r = W.sphere_field(32, 0.1, 7)
    ck = SpheresChecker(c, r)
    states, _ = W.reference_valid_states(sp, 2000, lambda x: O.is_valid(sp, ck, x), seed=9, chunk=6000)
    cnt = _run(sp, ck, states, (1500, 500), gpu)
    assert cnt[1499] == math.ceil((math.e + math.e / 6) * math.log(1500))


def test_prm_star_kinematic_chain(gpu):
    sp = KinematicChainSpace(12, 1.0 / 12)  # KinematicChainBenchmark.cpp:48-49
    ck = KinematicChainChecker(W.horn_environment(12, math.log(12.0) / 12.0))
    states, _ = W.reference_valid_states(sp, 1200, lambda x: O.is_valid(sp, ck, x), seed=42, chunk=5000)
    _run(sp, ck, states, (200, 1000), gpu)


def test_prm_star_ties_by_id(gpu):
    """Duplicate grid states: equal distances resolve by insertion id, across the stored / in-batch split."""
    sp = RealVectorStateSpace(2)
    g = np.stack(np.meshgrid(np.arange(0, 1, 0.1), np.arange(0, 1, 0.1)), -1).reshape(-1, 2)
    states = np.concatenate([g, g, g])
    _run(sp, AllValidChecker(), states, (90, 110, 100), gpu)


def test_prm_star_rank_slices(gpu):
    """Two replicas that both insert every milestone but each compute half of every batch's
    neighbours / edges (the multi-GPU decomposition, j0/j1) together equal the full answer, and
    both replicas end with the same roadmap."""
    sp = SE3StateSpace()
    c, r = W.sphere_field(32, 0.1, 7)
    ck = SpheresChecker(c, r)
    states, _ = W.reference_valid_states(sp, 1500, lambda x: O.is_valid(sp, ck, x), seed=5, chunk=4000)
    kc = math.e + math.e / sp.getDimension()
    k_cap = max(1, int(math.ceil(kc * math.log(len(states)))))
    reps = [(NearestNeighborsGPU(sp, gpu), DiscreteMotionValidatorGPU(sp, ck, gpu)) for _ in range(2)]
    got_n, got_c, got_v = [], [], []
    at = 0
    for b in (400, 600, 500):
        x = states[at:at + b]
        h = b // 2
        for rk, (nn, mv) in enumerate(reps):
            j0, j1 = (0, h) if rk == 0 else (h, b)
            n, cc, v, _ = nn.prm_add_milestones(mv, x, kc, k_cap, j0, j1)
            assert n.shape[0] == j1 - j0
            got_n.append(n)
            got_c.append(cc)
            got_v.append(v)
        at += b
    on, oc, ov = O.prm_causal(sp, ck, states, kc, k_cap)
    np.testing.assert_array_equal(np.concatenate(got_c), oc)
    np.testing.assert_array_equal(np.concatenate(got_n), on)
    np.testing.assert_array_equal(np.concatenate(got_v), ov.astype(bool))
    assert reps[0][0].size() == reps[1][0].size() == len(states)


def test_lazy_prm_star_neighbours_and_weights(gpu):
    """LazyPRM::addMilestone (LazyPRM.cpp:285-309): the same causal neighbours, no motion check,
    edge weights = distance(milestone, neighbour) equal to the oracle metric."""
    sp = KinematicChainSpace(12, 1.0 / 12)
    ck = KinematicChainChecker(W.horn_environment(12, math.log(12.0) / 12.0))
    states, _ = W.reference_valid_states(sp, 900, lambda x: O.is_valid(sp, ck, x), seed=11, chunk=5000)
    kc = math.e + math.e / sp.getDimension()
    k_cap = max(1, int(math.ceil(kc * math.log(len(states)))))
    nn = NearestNeighborsGPU(sp, gpu)
    got = [nn.lazyprm_add_milestones(states[a:b], kc, k_cap) for a, b in ((0, 300), (300, 900))]
    gn = np.concatenate([g[0] for g in got])
    gc = np.concatenate([g[1] for g in got])
    gd = np.concatenate([g[2] for g in got])
    on, oc, _ = O.prm_causal(sp, ck, states, kc, k_cap)
    np.testing.assert_array_equal(gc, oc)
    np.testing.assert_array_equal(gn, on)
    for i in range(len(states)):
        for r in range(gc[i]):
            assert gd[i, r] == O.distance(sp, states[i], states[gn[i, r]])
        assert np.all(np.isinf(gd[i, gc[i]:]))
    assert nn.size() == len(states)
