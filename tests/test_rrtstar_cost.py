"""RRT*'s cost logic (ompl_gpu_rrtstar_stage_host / _commit, ompl_amd/csrc/rrtstar_tree.cpp) on
the CPU: the geometric part of every iteration — nearest, steer, checkMotion, the neighbourhood
nearestK(x, ceil(k_rrt ln(size + 1))) over the tree as it stands and both motion bits per
neighbour — comes from the oracle (brute force, oracle validator), staged in batches of
different sizes, and the committed tree must equal the oracle's sequential RRT* loop
(oracle/rrtstar.cpp, RRTstar.cpp:247-542): every sample's nearest / added id / chosen parent,
every vertex's parent, incCost and cost — bit for bit, the arithmetic being the same host fp64.
No GPU: the library's tree functions never touch the device."""
import ctypes as C
import math

import numpy as np
import pytest

import pyoracle as O
from ompl_amd import abi
from ompl_amd import sampling as S
from ompl_amd import workloads as W
from ompl_amd.checkers import HypercubeChecker, SpheresChecker
from ompl_amd.rrtstar import k_rrt
from ompl_amd.spaces import RealVectorStateSpace, SE3StateSpace


def _p(a):
    return C.c_void_p(a.ctypes.data)


class _Tree:
    def __init__(self):
        self.h = C.c_void_p()
        assert abi.lib.ompl_gpu_rrtstar_tree_create(C.byref(self.h)) == 0

    def add(self, parent, inc, cost):
        p, i, c = (np.ascontiguousarray(a, dt) for a, dt in ((parent, np.int64), (inc, float), (cost, float)))
        assert abi.lib.ompl_gpu_rrtstar_tree_add(self.h, len(p), _p(p), _p(i), _p(c)) == 0

    def stage(self, near, added, inc, off, ids, dist, bits):
        arrs = [np.ascontiguousarray(a, dt) for a, dt in ((near, np.uint32), (added, np.uint32), (inc, float),
                                                           (off, np.uint64), (ids, np.uint32), (dist, float),
                                                           (bits, np.uint8))]
        assert abi.lib.ompl_gpu_rrtstar_stage_host(self.h, len(near), *[_p(a) for a in arrs]) == 0

    def commit(self, ns, maxd):
        near, added, chosen = (np.empty(ns, np.int64) for _ in range(3))
        got = C.c_size_t()
        assert abi.lib.ompl_gpu_rrtstar_commit(self.h, maxd, ns, _p(near), _p(added), _p(chosen), C.byref(got)) == 0
        assert got.value == ns
        return near, added, chosen

    def read(self):
        n = C.c_size_t()
        assert abi.lib.ompl_gpu_rrtstar_tree_size(self.h, C.byref(n)) == 0
        n = n.value
        par, inc, cost = np.empty(n, np.int64), np.empty(n), np.empty(n)
        assert abi.lib.ompl_gpu_rrtstar_tree_read(self.h, 0, n, _p(par), _p(inc), _p(cost)) == 0
        return par, inc, cost

    def totals(self):
        t = np.zeros(6, np.uint64)
        assert abi.lib.ompl_gpu_rrtstar_tree_totals(self.h, t.ctypes.data_as(C.POINTER(C.c_uint64))) == 0
        return t

    def close(self):
        abi.lib.ompl_gpu_rrtstar_tree_destroy(self.h)


def _geometric(sp, ck, states, samples, maxd, krrt):
    """the device batch's outputs for samples in order (states grows as samples are added)"""
    near, added, inc, off, ids, dist, bits = [], [], [], [0], [], [], []
    for s in samples:
        n = len(states)
        oi, od, _ = O.knn(sp, np.asarray(states), s[None], 1)
        nm = int(oi[0, 0])
        d = O.distance(sp, states[nm], s)
        x = O.interpolate(sp, states[nm], s, maxd / d) if d > maxd else s.copy()
        near.append(nm)
        ok = bool(O.check_motions(sp, ck, states[nm][None], x[None])[0][0])
        if not ok:
            added.append(0xFFFFFFFF)
            inc.append(0.0)
            off.append(off[-1])
            continue
        inc.append(O.distance(sp, states[nm], x))
        k = int(math.ceil(krrt * math.log(n + 1)))
        ni, nd, cnt = O.knn(sp, np.asarray(states), x[None], k)
        ni, nd = ni[0, :cnt[0]], nd[0, :cnt[0]]
        nb = np.asarray(states)[ni]
        fwd = O.check_motions(sp, ck, nb, np.repeat(x[None], len(ni), 0))[0]
        bwd = O.check_motions(sp, ck, np.repeat(x[None], len(ni), 0), nb)[0]
        ids.extend(ni.tolist())
        dist.extend(nd.tolist())
        bits.extend((fwd.astype(np.uint8) | (bwd.astype(np.uint8) << 1)).tolist())
        off.append(off[-1] + len(ni))
        added.append(n)
        states.append(x)
    return near, added, inc, off, ids, dist, bits


def _run(sp, ck, start_states, parent, inc0, cost0, samples, batches):
    maxd = 0.2 * sp.getMaximumExtent()
    krrt = k_rrt(sp.getDimension())
    tree = _Tree()
    tree.add(parent, inc0, cost0)
    states = [np.asarray(r, float) for r in start_states]
    got = []
    at = 0
    for b in batches:
        g = _geometric(sp, ck, states, samples[at:at + b], maxd, krrt)
        tree.stage(*g)
        got.append(tree.commit(b, maxd))
        at += b
    assert at == len(samples)
    near, added, chosen = (np.concatenate([o[j] for o in got]) for j in range(3))
    ref = O.rrtstar(sp, ck, start_states, parent, inc0, cost0, samples, maxd, krrt)
    radd = ref["added"].astype(np.int64)
    radd[radd == 0xFFFFFFFF] = -1
    np.testing.assert_array_equal(near, ref["nearest"].astype(np.int64))
    np.testing.assert_array_equal(added, radd)
    np.testing.assert_array_equal(chosen, ref["parent_choice"])
    par, inc, cost = tree.read()
    np.testing.assert_array_equal(par, ref["parent"])
    np.testing.assert_array_equal(inc, ref["inc"])
    np.testing.assert_array_equal(cost, ref["cost"])
    t = tree.totals()
    assert int(t[0]) == ref["rewires"] and ref["rewires"] > 0
    assert int(t[1]) == ref["checks"]  # the checkMotion calls the sequential loop makes
    assert int(t[2]) == ref["n_added"] and int(t[4]) == len(samples)
    tree.close()


def test_cost_logic_r3_spheres():
    sp = RealVectorStateSpace(3)
    c, r = W.sphere_field(32, 0.1, 7)
    ck = SpheresChecker(c, r)
    S.set_seed(42)
    x = S.StateSampler(sp).sample_uniform(1400)
    start = x[np.flatnonzero(O.is_valid(sp, ck, x[:50]))[0]]
    _run(sp, ck, start[None], [-1], [0.0], [0.0], x[50:1400], (1, 3, 60, 436, 850))


def test_cost_logic_se3_hypercube_existing_tree():
    """an existing tree (nearest-earlier parents, path-length costs), then samples in batches"""
    sp = SE3StateSpace(0.0, 1.0)
    ck = HypercubeChecker(3, 0.1)
    S.set_seed(7)
    x = S.StateSampler(sp).sample_uniform(60000)
    v = O.check_motions_mt(sp, ck, x, x, 8)
    tree = x[v][:300]
    parent = np.full(len(tree), -1, np.int64)
    inc = np.zeros(len(tree))
    for j in range(1, len(tree)):
        oi, od, _ = O.knn(sp, tree[:j], tree[j][None], 1)
        parent[j], inc[j] = int(oi[0, 0]), od[0, 0]
    cost = np.zeros(len(tree))
    for j in range(1, len(tree)):
        cost[j] = cost[parent[j]] + inc[j]
    samples = np.concatenate([x[~v][:500], x[v][300:600]])[np.random.default_rng(1).permutation(800)]
    _run(sp, ck, tree, parent, inc, cost, samples, (200, 600))


def test_cost_logic_inconsistent_tree():
    """an existing tree whose costs are not parent's cost + incCost (each edge's share scaled by
    0.6-1.4: costs still grow along every path, as any RRT* tree's must — an ancestor cheaper than
    its descendant is what keeps a rewire from closing a cycle), so the commit takes its general
    rewiring loop (costs may rise under updateChildCosts) — against the sequential loop"""
    sp = RealVectorStateSpace(3)
    c, r = W.sphere_field(32, 0.1, 7)
    ck = SpheresChecker(c, r)
    S.set_seed(11)
    x = S.StateSampler(sp).sample_uniform(3000)
    v = O.is_valid(sp, ck, x)
    tree = x[v][:200]
    parent = np.full(len(tree), -1, np.int64)
    inc = np.zeros(len(tree))
    for j in range(1, len(tree)):
        oi, od, _ = O.knn(sp, tree[:j], tree[j][None], 1)
        parent[j], inc[j] = int(oi[0, 0]), od[0, 0]
    f = np.random.default_rng(3).uniform(0.6, 1.4, len(tree))
    cost = np.zeros(len(tree))
    for j in range(1, len(tree)):
        cost[j] = cost[parent[j]] + inc[j] * f[j]  # no longer parent's cost + incCost
    _run(sp, ck, tree, parent, inc, cost, x[v][200:500], (100, 200))


def test_commit_rejects_bad_batches():
    tree = _Tree()
    tree.add([-1], [0.0], [0.0])
    # a neighbour id past the tree
    tree.stage([0], [1], [0.1], [0, 1], [5], [0.1], [3])
    near = np.empty(1, np.int64)
    got = C.c_size_t()
    assert abi.lib.ompl_gpu_rrtstar_commit(tree.h, 1.0, 1, _p(near), None, None, C.byref(got)) == abi.ERR_INVALID_ARG
    # nothing staged
    assert abi.lib.ompl_gpu_rrtstar_commit(tree.h, 1.0, 0, None, None, None, None) == abi.ERR_INVALID_ARG
    # a parent that is not an earlier id
    p = np.array([3], np.int64)
    assert abi.lib.ompl_gpu_rrtstar_tree_add(tree.h, 1, _p(p), None, None) == abi.ERR_INVALID_ARG
    # a start state with a cost other than the identity
    p, cc = np.array([-1], np.int64), np.array([0.5])
    assert abi.lib.ompl_gpu_rrtstar_tree_add(tree.h, 1, _p(p), None, _p(cc)) == abi.ERR_INVALID_ARG
    # an added id that is not new (0 exists), and a neighbour that is not earlier than the added state
    for added, ids in (([0], [0]), ([1], [1])):
        tree.stage([0], added, [0.1], [0, 1], ids, [0.1], [3])
        assert abi.lib.ompl_gpu_rrtstar_commit(tree.h, 1.0, 1, _p(near), None, None, C.byref(got)) == \
            abi.ERR_INVALID_ARG
    # added ids out of order
    tree.stage([0, 0], [2, 1], [0.1, 0.1], [0, 1, 2], [0, 0], [0.1, 0.1], [3, 3])
    near2 = np.empty(2, np.int64)
    assert abi.lib.ompl_gpu_rrtstar_commit(tree.h, 1.0, 2, _p(near2), None, None, C.byref(got)) == abi.ERR_INVALID_ARG
    tree.close()
