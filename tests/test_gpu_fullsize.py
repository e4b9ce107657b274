"""GPU parity at the benchmark configurations' full sizes, on the bench's own inputs (the
reference RNG streams: RNG::setSeed(42), a tree sampler, then a query sampler), plus a device
port of the reference's randomAccessPatternTest (tests/datastructures/nearestneighbors.cpp:208-287).

* cfg3: the 10^6-state SE(3) tree, 10^5 queries through the culled group walk
  at k = 10, 128 of them checked against the oracle's brute force.
* cfg2 (M1): the 10^5-state R^6 store, 10^5 queries through the culled group walk at k = 10,
  128 of them checked against the oracle's brute force (bit-exact distances).
* cfg5 (M4): the 10^7 valid-sample SE(3) set, 10^5 vertices through the radius walk at BIT*'s
  r = 0.1528, 32 CSR segments checked against the oracle's brute force.
"""
import math

import numpy as np
import pytest

import pyoracle as O
from ompl_amd import DiscreteMotionValidatorGPU, NearestNeighborsGPU
from ompl_amd import workloads as W
from ompl_amd.checkers import SpheresChecker
from ompl_amd.spaces import SE3StateSpace
from parity import assert_dist_close, assert_knn_parity, oracle_knn_mt

pytestmark = pytest.mark.gpu


def _oracle_radius_mt(sp, data, queries, r, threads=8):
    from concurrent.futures import ThreadPoolExecutor

    parts = np.array_split(np.arange(len(queries)), min(threads, len(queries)))
    with ThreadPoolExecutor(len(parts)) as ex:
        res = list(ex.map(lambda ix: O.radius(sp, data, queries[ix], r), parts))
    segs = []
    for off, ids, d in res:
        for q in range(len(off) - 1):
            segs.append((ids[int(off[q]):int(off[q + 1])], d[int(off[q]):int(off[q + 1])]))
    return segs


def test_cfg3_reference_tree_k10(gpu):
    import bench

    sp = SE3StateSpace(0.0, 1.0)
    tree, q = bench.reference_inputs(sp, 1_000_000, 100_000, 0)
    nn = NearestNeighborsGPU(sp, gpu)
    nn.add(tree)
    before = nn.cull_stats()[2]
    ids, d, cnt = nn.nearestKBatch(q, 10)
    assert nn.cull_stats()[2] > before, "the batch did not take the culled group walk"
    assert (cnt == 10).all()
    pick = np.concatenate([np.arange(64), np.random.default_rng(3).choice(np.arange(64, len(q)), 64, replace=False)])
    oi, od = oracle_knn_mt(O, sp, tree, q[pick], 16)
    assert_knn_parity(ids[pick], d[pick], oi, od, 10)
    nn.close()


def test_cfg2_reference_store_k10(gpu):
    """cfg2: RealVectorStateSpace(6) over [0,1]^6, the bench's reference-stream
    10^5-state store and 10^5 queries, nearestK(k = 10) through the culled group walk; 128 queries
    (the first 64 and 64 random) against the oracle's brute force: identical ids (ties aside) and
    bit-identical fp64 distances (the R^n metric is exact in the reference's operation order)."""
    import bench
    from ompl_amd.spaces import RealVectorStateSpace

    sp = RealVectorStateSpace(6)
    tree, q = bench.reference_inputs(sp, 100_000, 100_000, 0)
    nn = NearestNeighborsGPU(sp, gpu)
    nn.add(tree)
    before = nn.cull_stats()[2]
    ids, d, cnt = nn.nearestKBatch(q, 10)
    assert nn.cull_stats()[2] > before, "the batch did not take the culled group walk"
    assert (cnt == 10).all()
    pick = np.concatenate([np.arange(64), np.random.default_rng(8).choice(np.arange(64, len(q)), 64, replace=False)])
    oi, od = oracle_knn_mt(O, sp, tree, q[pick], 16)
    np.testing.assert_array_equal(d[pick], od[:, :10])
    assert_knn_parity(ids[pick], d[pick], oi, od, 10)
    assert bool(np.all(np.diff(d, axis=1) >= 0)), "every list sorted ascending"
    nn.close()


def test_cfg5_radius_1e7_valid_samples(gpu):
    import bench

    sp = SE3StateSpace(0.0, 1.0)
    c, rr = W.sphere_field(32, 0.1, 7)
    mv = DiscreteMotionValidatorGPU(sp, SpheresChecker(c, rr), gpu)
    tree, q = bench.reference_inputs(sp, 10_000_000, 100_000, 0, valid=mv.isValid)
    r = W.bitstar_radius(len(tree), 6, math.pi ** 2)
    assert abs(r - 0.1528) < 5e-4
    nn = NearestNeighborsGPU(sp, gpu)
    nn.add(tree)
    off, ids, d = nn.nearestRBatch(q, r)
    assert int(off[-1]) > 10 * len(q)  # ~10.8 neighbours per vertex at this radius
    pick = np.concatenate([np.arange(16), np.random.default_rng(4).choice(np.arange(16, len(q)), 16, replace=False)])
    segs = _oracle_radius_mt(sp, tree, q[pick], r)
    for j, qi in enumerate(pick):
        gi, gd = ids[int(off[qi]):int(off[qi + 1])], d[int(off[qi]):int(off[qi + 1])]
        oi, od = segs[j]
        assert len(gi) == len(oi), f"query {qi}: {len(gi)} vs {len(oi)} neighbours"
        assert np.array_equal(gi.astype(np.int64), oi.astype(np.int64)), f"query {qi}: ids differ"
        assert_dist_close(gd, od)
    nn.close()
    mv.close()


def test_random_access_pattern(gpu):
    """randomAccessPatternTest (nearestneighbors.cpp:208-287) on SE(3) [0,1]^3: m = 200 rounds of
    n = 10 adds, n queries each with nearestK(k uniform in [1, maxk = 30]) and nearestR(r uniform in
    [0, 3]) compared with the Linear structure (here the oracle's brute force over the live
    states: equal sizes, per-rank distances within eps = 1e-6 as the reference checks — and
    identical ids, which it does not), then every stored state removed with probability 0.5
    (size and list checked).  Each round also answers its queries as one batch of 64, so the
    culled walk sees the same interleaving of adds, removals and index rebuilds."""
    from ompl_amd import sampling as S

    sp = SE3StateSpace(0.0, 1.0)
    S.set_seed(42)
    smp = S.StateSampler(sp)
    rng = np.random.default_rng(2087)
    nn = NearestNeighborsGPU(sp, gpu)
    stored = {}  # id -> state (the live set)
    m, n, maxk = 200, 10, 30
    for _ in range(m):
        new = smp.sample_uniform(n)
        for i, x in zip(nn.add(new), new):
            stored[int(i)] = x
        live = np.array(sorted(stored))
        data = np.array([stored[i] for i in live])
        qs = smp.sample_uniform(n)
        for s in qs:
            k = int(rng.integers(1, maxk + 1))
            ids, d, cnt = nn.nearestKBatch(s, k)
            oi, od, ocnt = O.knn(sp, data, s[None], k)
            assert int(cnt[0]) == int(ocnt[0]) == min(k, len(live))
            kk = int(cnt[0])
            assert np.allclose(d[0, :kk], od[0, :kk], rtol=0, atol=1e-6)
            assert np.array_equal(ids[0, :kk].astype(np.int64), live[oi[0, :kk].astype(np.int64)])
            r = float(rng.uniform(0.0, 3.0))
            off, rid, rd = nn.nearestRBatch(s, r)
            ooff, oid, ord_ = O.radius(sp, data, s[None], r)
            assert int(off[1]) == int(ooff[1])
            assert np.allclose(rd, ord_, rtol=0, atol=1e-6)
            assert np.array_equal(rid.astype(np.int64), live[oid.astype(np.int64)])
        batch = smp.sample_uniform(64)
        k = int(rng.integers(1, maxk + 1))
        ids, d, cnt = nn.nearestKBatch(batch, k)
        kk = min(k, len(live))
        oi, od, ocnt = O.knn(sp, data, batch, min(k + 6, len(live)))  # + 6: the boundary tie class
        assert (cnt == kk).all()
        assert_knn_parity(ids[:, :kk], d[:, :kk], live[oi.astype(np.int64)], od, kk)
        for i in list(stored):
            if rng.uniform() < 0.5:
                sz = nn.size()
                assert nn.remove(i)
                del stored[i]
                assert nn.size() == sz - 1 == len(stored)
        assert sorted(nn.list()) == sorted(stored)
    builds, appends = nn.index_stats()
    assert builds >= 2 and appends >= 1  # removals forced rebuilds; adds went to the tail
    nn.close()


def test_cfg4_chain_culled_scan_1e6(gpu):
    """cfg4: PRM*'s stored-part kNN on the KinematicChain space at the bench's
    size — 10^6 reference-stream states, k = 41 (ConnectionStrategy.h:145-149) — through the
    culled chain scan over the k-d sorted joint-position store; 64 of 8,192 milestones checked
    against the oracle's brute force, then again after a tail append (a PRM* batch's 8,192 new
    milestones) and 500 removals."""
    import bench
    from ompl_amd.spaces import KinematicChainSpace

    sp = KinematicChainSpace(12, 1.0 / 12)
    tree, q = bench.reference_inputs(sp, 1_000_000, 8_192, 0)
    nn = NearestNeighborsGPU(sp, gpu)
    nn.add(tree)
    before = nn.cull_stats()[2]
    ids, d, cnt = nn.nearestKBatch(q, 41)
    assert nn.cull_stats()[2] > before, "the batch did not take the culled chain scan"
    assert (cnt == 41).all()
    pick = np.random.default_rng(5).choice(len(q), 64, replace=False)
    oi, od = oracle_knn_mt(O, sp, tree, q[pick], 41)
    np.testing.assert_array_equal(d[pick], od)  # the chain metric is bit-exact (fp64, reference order)
    np.testing.assert_array_equal(ids[pick].astype(np.int64), oi.astype(np.int64))
    # a PRM* batch later: the milestones join the store (tail tiles), some states go away
    nn.add(q)
    gone = np.random.default_rng(6).choice(len(tree), 500, replace=False)
    for i in gone:
        nn.remove(int(i))
    q2 = bench.reference_inputs(sp, 0, 2 * 8_192, 0)[1][8_192:]
    ids2, d2, _ = nn.nearestKBatch(q2, 41)
    keep = np.ones(len(tree) + len(q), dtype=bool)
    keep[gone] = False
    store = np.concatenate([tree, q])
    live_ids = np.flatnonzero(keep)
    pick2 = np.random.default_rng(7).choice(len(q2), 64, replace=False)
    oi2, od2 = oracle_knn_mt(O, sp, store[live_ids], q2[pick2], 41)
    np.testing.assert_array_equal(d2[pick2], od2)
    np.testing.assert_array_equal(ids2[pick2].astype(np.int64), live_ids[oi2.astype(np.int64)])
    nn.close()


# ---- every query at full size: the culled paths against the exact fp64 scan -------------------
# The oracle checks above sample queries (the CPU brute force over 10^6-10^7 states is slow); here
# every query of the bench batch is compared with the library's exact fp64 brute-force scan
# (set_exact: no fp32 screen, no culling — itself pinned against the oracle by test_gpu_nn.py on
# every space), bit for bit: ids and distances.
def _culled_vs_exact(sp, tree, q, k, gpu):
    nn = NearestNeighborsGPU(sp, gpu)
    nn.add(tree)
    ids, d, cnt = nn.nearestKBatch(q, k)
    nn.set_exact(True)
    ei, ed, ecnt = nn.nearestKBatch(q, k)
    nn.close()
    np.testing.assert_array_equal(cnt, ecnt)
    np.testing.assert_array_equal(d, ed)
    np.testing.assert_array_equal(ids, ei)


def test_cfg3_every_query_vs_exact_scan(gpu):
    import bench

    sp = SE3StateSpace(0.0, 1.0)
    tree, q = bench.reference_inputs(sp, 1_000_000, 100_000, 0)
    _culled_vs_exact(sp, tree, q, 10, gpu)


def test_cfg2_every_query_vs_exact_scan(gpu):
    import bench
    from ompl_amd.spaces import RealVectorStateSpace

    sp = RealVectorStateSpace(6)
    tree, q = bench.reference_inputs(sp, 100_000, 100_000, 0)
    _culled_vs_exact(sp, tree, q, 10, gpu)


def test_cfg4_every_milestone_vs_exact_scan(gpu):
    import bench
    from ompl_amd.spaces import KinematicChainSpace

    sp = KinematicChainSpace(12, 1.0 / 12)
    tree, q = bench.reference_inputs(sp, 1_000_000, 8_192, 0)
    _culled_vs_exact(sp, tree, q, 41, gpu)


def test_cfg5k_every_vertex_vs_exact_scan(gpu):
    """BIT*'s kNN mode at its k = 57 on the 10^7 valid-sample set, 10^4 vertices."""
    import bench

    sp = SE3StateSpace(0.0, 1.0)
    c, rr = W.sphere_field(32, 0.1, 7)
    mv = DiscreteMotionValidatorGPU(sp, SpheresChecker(c, rr), gpu)
    tree, q = bench.reference_inputs(sp, 10_000_000, 10_000, 0, valid=mv.isValid)
    mv.close()
    _culled_vs_exact(sp, tree, q, 57, gpu)


def test_cfg5_every_vertex_radius_vs_exact_scan(gpu):
    """BIT*'s radius mode (r = 0.1528) on the 10^7 valid-sample set, 2 x 10^4 vertices: the slab
    walk's CSR equals the exact fp64 scan's, offsets, ids and distances."""
    import bench

    sp = SE3StateSpace(0.0, 1.0)
    c, rr = W.sphere_field(32, 0.1, 7)
    mv = DiscreteMotionValidatorGPU(sp, SpheresChecker(c, rr), gpu)
    tree, q = bench.reference_inputs(sp, 10_000_000, 20_000, 0, valid=mv.isValid)
    mv.close()
    r = W.bitstar_radius(len(tree), 6, math.pi ** 2)
    nn = NearestNeighborsGPU(sp, gpu)
    nn.add(tree)
    off, ids, d = nn.nearestRBatch(q, r)
    nn.set_exact(True)
    eoff, eids, ed = nn.nearestRBatch(q, r)
    nn.close()
    np.testing.assert_array_equal(off, eoff)
    np.testing.assert_array_equal(ids, eids)
    np.testing.assert_array_equal(d, ed)
