"""GPU parity at the benchmark configurations' full sizes, on one bench step of each workload
(bench.Runner: the reference RNG streams, RNG::setSeed(42), a tree sampler, then a query sampler),
checked against the CPU oracle for EVERY query and EVERY edge of the step — the GNAT restatement
(oracle/gnat.cpp, itself checked exact against brute force in test_oracle.py, as the reference's
tests/datastructures/nearestneighbors.cpp:147-184 checks GNAT against Linear) and the oracle
DiscreteMotionValidator (oracle/oracle.cpp, DiscreteMotionValidator.cpp:93-145).  No test here
compares the library with itself.

* cfg3: 10^6-state SE(3) tree, 10^5 samples: every nearestK(k = 10) list, every
  steered state (RRT.cpp:137-146) and every checkMotion bit / segment count.
* cfg2 (M1): 10^5-state R^6 store, 10^5 queries, k = 10, bit-exact distances.
* cfg4 (M3): PRM* on the 10^6-vertex KinematicChain roadmap, two causal 8,192-milestone batches
  (the bench's step: 8 causal 1,024-row chunks, concurrent per-milestone cursors; the second batch
  sees the first in the store's tail): every milestone's stored neighbours against GNAT, 96
  milestones per batch in full against the sequential loop's list over roadmap + earlier
  milestones (PRM.cpp:562-596, ConnectionStrategy.h:145-149), every edge's validity bit.
* cfg5 (M4): 10^7 valid SE(3) samples, 10^5 vertices: every nearestR(r = 0.1528) segment and
  every edge bit; BIT*'s kNN mode (k = 57) for every vertex and every edge bit.
Also the device port of the reference's randomAccessPatternTest
(tests/datastructures/nearestneighbors.cpp:208-287).
"""
import argparse
import math

import numpy as np
import pytest

import pyoracle as O
from ompl_amd import NearestNeighborsGPU
from ompl_amd.spaces import SE3StateSpace
from parity import CPU_THREADS, assert_dist_close, assert_knn_parity_rows

pytestmark = pytest.mark.gpu


def _run_steps(workload, steps=1, bitstar_knn=False, queries=None):
    """one bench.Runner of `workload` at its bench defaults; `steps` steps, each step's device
    outputs copied to the host"""
    import torch

    import bench

    t, q, k = bench.DEFAULTS[workload]
    a = argparse.Namespace(workload=workload, tree=t, queries=queries or q, k=k, exact=False,
                           partition="replicated", warmup=0, steps=steps, bitstar_knn=bitstar_knn)
    dev = torch.device("cuda", 0)
    stream = torch.cuda.Stream(dev)
    run = bench.Runner(a, torch, dev, 0, 0, stream)
    run.stream = stream
    outs = []
    for _ in range(steps):
        run.step()
        torch.cuda.synchronize(dev)
        o = {"m": run.m}
        for name in ("ids", "dd", "s_from", "s_to", "valid", "off", "cnt", "evalid"):
            if hasattr(run, name):
                o[name] = getattr(run, name).cpu().numpy()
        outs.append(o)
    return run, outs


def _gnat(sp, data):
    g = O.Gnat(sp)
    g.add(data, bulk=True)
    return g


def _check_edges(sp, ck, s1, s2, valid):
    """every edge's checkMotion bit against the oracle validator on the same endpoints"""
    ov = O.check_motions_mt(sp, ck, s1, s2, CPU_THREADS)
    bad = np.flatnonzero(ov != valid.astype(bool))
    assert len(bad) == 0, f"{len(bad)} of {len(s1)} edges differ from the oracle (first {bad[:8]})"
    return float(ov.mean())


# ---- cfg3 --------------------------------------------------------------------------------------
@pytest.fixture(scope="module")
def cfg3(gpu):
    run, (o,) = _run_steps("cfg3")
    out = dict(sp=run.sp, ck=run.ck, tree=run.tree, q=run.q_host, maxd=run.maxd, **o)
    run.close()
    return out


def test_cfg3_every_query_vs_gnat(cfg3):
    """all 10^5 nearestK(k = 10) lists of the headline step against GNAT (k + 4 exposes the k-th
    rank's tie class)"""
    c = cfg3
    g = _gnat(c["sp"], c["tree"])
    oi, od, oc = g.knn(c["q"], 14, CPU_THREADS)
    assert (oc == 14).all()
    assert_knn_parity_rows(c["ids"], c["dd"], oi, od, 10)


def test_cfg3_every_edge_vs_oracle(cfg3):
    """the step's 10^5 motions: from = the nearest stored state; to = the sample, or
    interpolate(nearest, sample, maxDistance / d) when d > maxDistance (RRT.cpp:141-146), equal to
    the oracle's interpolation bit for bit (translation and slerped rotation); every validity bit and
    validSegmentCount equal to the oracle validator's on the same endpoints"""
    c = cfg3
    sp, nq = c["sp"], len(c["q"])
    near = c["ids"][:, 0].astype(np.int64)
    np.testing.assert_array_equal(c["s_from"][:nq], c["tree"][near])
    d = c["dd"][:, 0]
    far = np.flatnonzero(d > c["maxd"])
    want = c["q"].copy()
    for i in far:
        want[i] = O.interpolate(sp, c["tree"][near[i]], c["q"][i], c["maxd"] / d[i])
    got = c["s_to"][:nq]
    np.testing.assert_array_equal(got, want)
    ov, ond, _, _ = O.check_motions(sp, c["ck"], c["s_from"][:nq], got)
    np.testing.assert_array_equal(c["valid"][:nq].astype(bool), ov)
    _check_edges(sp, c["ck"], c["s_from"][:nq], got, c["valid"][:nq])


# ---- cfg2 --------------------------------------------------------------------------------------
def test_cfg2_every_query_vs_gnat(gpu):
    """all 10^5 nearestK(k = 10) lists of the R^6 step against GNAT, bit-exact distances (the R^n
    metric is exact in the reference's operation order)"""
    run, (o,) = _run_steps("cfg2")
    g = _gnat(run.sp, run.tree)
    oi, od, _ = g.knn(run.q_host, 14, CPU_THREADS)
    np.testing.assert_array_equal(o["dd"], od[:, :10])
    assert_knn_parity_rows(o["ids"], o["dd"], oi, od, 10)
    assert bool(np.all(np.diff(o["dd"], axis=1) >= 0))
    run.close()


# ---- cfg4: PRM* causal batches at the bench's size ---------------------------------------------
@pytest.fixture(scope="module")
def cfg4(gpu):
    run, outs = _run_steps("cfg4", steps=2)
    assert len(run.milestones) == 2 and all(len(b) == 8192 for b in run.milestones)
    out = dict(sp=run.sp, ck=run.ck, kc=run.kc, roadmap=run.tree, batches=run.milestones, outs=outs,
               k_cap=run.k)
    run.close()
    out["gnat"] = _gnat(out["sp"], out["roadmap"])
    return out


def _cfg4_batch(c, b):
    """batch b (0 or 1) of the cfg4 run against the sequential PRM* loop"""
    sp, n0 = c["sp"], len(c["roadmap"])
    x = c["batches"][b]
    m = len(x)
    earlier = np.concatenate([c["batches"][i] for i in range(b)] + [np.empty((0, sp.dim))])
    base = n0 + len(earlier)  # id of the batch's first milestone
    o = c["outs"][b]
    nbr, cnt, val = o["ids"].view(np.uint32).astype(np.int64), o["cnt"].astype(np.int64), o["evalid"].astype(bool)
    kj = np.array([int(math.ceil(c["kc"] * math.log(base + j + 1))) for j in range(m)])
    np.testing.assert_array_equal(cnt, np.minimum(kj, base + np.arange(m)))
    # every milestone: the stored roadmap entries of its list are GNAT's first entries, in order
    kg = int(kj.max())
    gi, gd, _ = c["gnat"].knn(x, kg, CPU_THREADS)
    allst = np.concatenate([c["roadmap"], earlier, x])
    for j in range(m):
        row = nbr[j, :cnt[j]]
        st = row[row < n0]
        np.testing.assert_array_equal(st, gi[j, :len(st)].astype(np.int64), err_msg=f"milestone {base + j}")
    # sampled milestones in full: roadmap (GNAT) + every earlier milestone (brute force), merged by
    # (distance, id), first k_j — includes the causal chunk boundaries (1,024-row chunks)
    pick = sorted(set([0, 1, 2, 63, 64, 1023, 1024, 1025, 2047, 2048, 4095, 4096, 6143, 8190, 8191])
                  | set(np.random.default_rng(50 + b).choice(m, 81, replace=False).tolist()))
    for j in pick:
        prev = np.concatenate([earlier, x[:j]])
        ci, cd = gi[j].astype(np.int64), gd[j]
        if len(prev):
            pi, pd, pc = O.knn(sp, prev, x[j][None], int(kj[j]))
            ci = np.concatenate([ci, pi[0, :pc[0]].astype(np.int64) + n0])
            cd = np.concatenate([cd, pd[0, :pc[0]]])
        order = np.lexsort((ci, cd))[: kj[j]]
        want = ci[order]
        np.testing.assert_array_equal(nbr[j, :cnt[j]], want, err_msg=f"milestone {base + j}")
        # the distances behind that order, from the oracle metric
        dd = np.array([O.distance(sp, allst[i], x[j]) for i in want])
        np.testing.assert_array_equal(dd, cd[order])
    # every edge: checkMotion(state[neighbour], state[milestone]) (PRM.cpp:582)
    live = np.arange(nbr.shape[1])[None, :] < cnt[:, None]
    s1 = allst[nbr[live]]
    s2 = np.repeat(x, cnt, axis=0)
    frac = _check_edges(sp, c["ck"], s1, s2, val[live])
    assert 0.0 < frac < 1.0
    return int(live.sum())


def test_cfg4_prm_batch_1_vs_sequential_loop(cfg4):
    """the first 8,192-milestone batch over the 10^6-vertex roadmap (8 causal chunks)"""
    assert _cfg4_batch(cfg4, 0) > 8192 * 30


def test_cfg4_prm_batch_2_tail_vs_sequential_loop(cfg4):
    """the second batch: the first batch's milestones are stored in the culled store's tail"""
    assert _cfg4_batch(cfg4, 1) > 8192 * 30


def test_cfg4_chain_store_after_removals(cfg4, gpu):
    """the culled chain scan after a tail append and 500 removals, 64 milestones against the
    oracle's brute force over the live states (bit-exact chain distances)"""
    from parity import oracle_knn_mt

    c = cfg4
    sp = c["sp"]
    nn = NearestNeighborsGPU(sp, gpu)
    nn.add(c["roadmap"])
    nn.add(c["batches"][0])
    gone = np.random.default_rng(6).choice(len(c["roadmap"]), 500, replace=False)
    for i in gone:
        nn.remove(int(i))
    q2 = c["batches"][1]
    before = nn.cull_stats()[2]
    ids2, d2, _ = nn.nearestKBatch(q2, 41)
    assert nn.cull_stats()[2] > before, "the batch did not take the culled chain scan"
    keep = np.ones(len(c["roadmap"]) + len(c["batches"][0]), dtype=bool)
    keep[gone] = False
    store = np.concatenate([c["roadmap"], c["batches"][0]])
    live_ids = np.flatnonzero(keep)
    pick2 = np.random.default_rng(7).choice(len(q2), 64, replace=False)
    oi2, od2 = oracle_knn_mt(O, sp, store[live_ids], q2[pick2], 41, CPU_THREADS)
    np.testing.assert_array_equal(d2[pick2], od2)
    np.testing.assert_array_equal(ids2[pick2].astype(np.int64), live_ids[oi2.astype(np.int64)])
    nn.close()


# ---- cfg5: BIT* batches over 10^7 valid samples -------------------------------------------------
def _assert_csr_ties(off, ids, oids, od):
    """equal CSR ids, except that inside a segment ids may trade places when their oracle
    distances are equal (a tie class, ordered by id on the device)"""
    bad = np.flatnonzero(ids != oids)
    if not len(bad):
        return
    seg = np.searchsorted(off.astype(np.int64), bad, side="right") - 1
    for q in np.unique(seg):
        a, b = int(off[q]), int(off[q + 1])
        assert sorted(ids[a:b].tolist()) == sorted(oids[a:b].tolist()), f"segment {q}: different neighbour sets"
        pos = {int(i): a + j for j, i in enumerate(oids[a:b])}
        for p in bad[seg == q]:
            o = pos[int(ids[p])]  # where the oracle has the device's id of position p
            assert od[o] == od[p], f"segment {q}: ids out of order beyond a tie"


@pytest.fixture(scope="module")
def cfg5_gnat(gpu):
    import bench
    from ompl_amd import DiscreteMotionValidatorGPU
    from ompl_amd import workloads as W
    from ompl_amd.checkers import SpheresChecker

    sp = SE3StateSpace(0.0, 1.0)
    c, rr = W.sphere_field(32, 0.1, 7)
    mv = DiscreteMotionValidatorGPU(sp, SpheresChecker(c, rr), gpu)
    key = ("cfg5", 10_000_000, 100_000)
    tree, _ = bench.shared_inputs("cfg5", sp, key[1], key[2], mv.isValid, None, None)
    mv.close()
    return _gnat(sp, tree)


def test_cfg5_radius_every_vertex_vs_gnat(cfg5_gnat):
    """all 10^5 nearestR(r = 0.1528) segments of the BIT* step (offsets, ids, distances) and
    every edge's checkMotion(vertex, sample) bit"""
    run, (o,) = _run_steps("cfg5")
    assert abs(run.radius - 0.1528) < 5e-4
    q = run.q_host
    off, ids, d = o["off"].astype(np.uint64), o["ids"][: o["m"]].astype(np.int64), o["dd"][: o["m"]]
    goff, gids, gd = cfg5_gnat.radius(q, run.radius, CPU_THREADS)
    np.testing.assert_array_equal(off, goff)
    assert int(off[-1]) > 10 * len(q)  # ~10.8 neighbours per vertex at this radius
    assert_dist_close(d, gd)
    _assert_csr_ties(off, ids, gids.astype(np.int64), gd)
    # the step checks the edges in place (ompl_gpu_mv_check_edges_device): (vertex q, sample ids[e])
    s1 = np.repeat(q, np.diff(off).astype(np.int64), axis=0)
    _check_edges(run.sp, run.ck, s1, run.tree[ids], o["valid"][: o["m"]])
    run.close()


def test_cfg5_knn_every_vertex_vs_gnat(cfg5_gnat):
    """BIT*'s kNN mode (k = 57): all 10^5 lists and every edge's checkMotion(vertex, sample) bit"""
    run, (o,) = _run_steps("cfg5", bitstar_knn=True)
    k = run.k
    assert k == 57
    oi, od, _ = cfg5_gnat.knn(run.q_host, k + 4, CPU_THREADS)
    assert_knn_parity_rows(o["ids"], o["dd"], oi, od, k)
    ids = o["ids"].astype(np.int64).reshape(-1)
    s1 = np.repeat(run.q_host, k, axis=0)  # the edges checked in place: (vertex, sample ids[e])
    _check_edges(run.sp, run.ck, s1, run.tree[ids], o["valid"][: o["m"]])
    run.close()


# ---- the reference's randomAccessPatternTest on the device ------------------------------------
def test_random_access_pattern(gpu):
    """randomAccessPatternTest (nearestneighbors.cpp:208-287) on SE(3) [0,1]^3: m = 200 rounds of
    n = 10 adds, n queries each with nearestK(k uniform in [1, maxk = 30]) and nearestR(r uniform in
    [0, 3]) compared with the Linear structure (here the oracle's brute force over the live
    states: equal sizes, per-rank distances within eps = 1e-6 as the reference checks — and
    identical ids, which it does not), then every stored state removed with probability 0.5
    (size and list checked).  Each round also answers its queries as one batch of 64, so the
    culled walk sees the same interleaving of adds, removals and index rebuilds."""
    from ompl_amd import sampling as S
    from parity import assert_knn_parity

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


def test_cfg3_steps_in_flight_identical(gpu):
    """bench's steps in flight (--lanes 2: alternate steps on two streams, each lane its own NN /
    validator handles over the same tree) give every step the same neighbours, steered motions and
    validity bits as the one-stream step — no lane reads another's scratch"""
    import torch

    import bench

    t, q, k = bench.DEFAULTS["cfg3"]
    outs = {}
    for lanes in (1, 2):
        a = argparse.Namespace(workload="cfg3", tree=t, queries=20000, k=k, exact=False, partition="replicated",
                               warmup=0, steps=4, bitstar_knn=False, lanes=lanes)
        dev = torch.device("cuda", 0)
        run = bench.Runner(a, torch, dev, 0, 0, torch.cuda.Stream(dev))
        assert len(run.lanes) == lanes
        res = []
        for _ in range(4):  # back to back, synchronised only at the end
            run.step()
            res.append({n: getattr(run, n) for n in ("ids", "dd", "s_to", "valid")})
        torch.cuda.synchronize(dev)
        outs[lanes] = [{n: v.cpu().numpy() for n, v in r.items()} for r in res]
        run.close()
    for a1, a2 in zip(outs[1], outs[2]):
        for n in a1:
            np.testing.assert_array_equal(a1[n], a2[n])
