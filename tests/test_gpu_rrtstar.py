"""RRT* iterations (RRT*): the device batch (ompl_gpu_rrtstar_batch_device) plus
the host cost logic (ompl_amd/rrtstar.py) against the oracle's sequential RRT* loop
(oracle/rrtstar.cpp, RRTstar.cpp:247-542 with its defaults) on the same samples:

* every sample's nearest state, whether it joined the tree and which parent it chose (delayCC's
  first valid neighbour in cost order, RRTstar.cpp:319-357), and the final tree — every vertex's
  parent and cost after all rewiring (:414-457) and child-cost updates (:633-643) — through the
  pipelined solve_batches (native cost logic on a host thread) and the sequential solve_batch;
* every neighbourhood nearestK(x, ceil(k_rrt ln(size + 1))) (:603-618) of sampled added states
  against the oracle's brute force over the tree as it stood (ids and order);
* both motion bits of every neighbourhood entry against the oracle validator.
Batches start from a single start state, so the first ones are dominated by in-batch nearest
states (the device's fixed point) and k > size; later ones by the stored tree."""
import math

import numpy as np
import pytest

import pyoracle as O
from ompl_amd import sampling as S
from ompl_amd import workloads as W
from ompl_amd.checkers import HypercubeChecker, SpheresChecker
from ompl_amd.rrtstar import RRTstarGPU
from ompl_amd.spaces import RealVectorStateSpace, SE3StateSpace
from parity import assert_dist_close

pytestmark = pytest.mark.gpu


def _run(sp, ck, start, samples, batches, gpu):
    maxd = 0.2 * sp.getMaximumExtent()
    planner = RRTstarGPU(sp, ck, maxd, gpu)
    planner.add_tree(start[None])
    cuts = np.cumsum((0,) + tuple(batches))
    assert cuts[-1] == len(samples)
    # the pipelined form: batch i's cost logic (host thread) overlaps batch i + 1's device work
    out = planner.solve_batches([samples[a:b] for a, b in zip(cuts[:-1], cuts[1:])])
    near, added, chosen = (np.concatenate([o[j] for o in out]) for j in range(3))
    ref = O.rrtstar(sp, ck, start[None], [-1], [0.0], [0.0], samples, maxd, planner.k_rrt)
    radd = ref["added"].astype(np.int64)
    radd[radd == 0xFFFFFFFF] = -1
    np.testing.assert_array_equal(near, ref["nearest"].astype(np.int64))
    np.testing.assert_array_equal(added, radd)
    np.testing.assert_array_equal(chosen, ref["parent_choice"])
    n = planner.n
    assert n == 1 + ref["n_added"] and n == planner.nn.size()
    np.testing.assert_array_equal(planner.parent[:n], ref["parent"])
    # every space bit for bit (SO3: glibc's own acos / sin on the device, so steered rotations and
    # the distances from them are the reference's)
    np.testing.assert_array_equal(planner.cost[:n], ref["cost"])
    np.testing.assert_array_equal(planner.inc[:n], ref["inc"])
    assert ref["rewires"] > 0 and planner.stats["rewires"] == ref["rewires"]
    assert planner.stats["checks_used"] == ref["checks"]
    return planner, ref


def _neighbourhoods_and_bits(planner, sp, ck, samples, gpu):
    """one more batch: its neighbourhoods against brute force over the tree as it stood, and every
    neighbourhood entry's two motion bits against the oracle validator"""
    import torch

    dev = torch.device("cuda", gpu)
    s = torch.as_tensor(samples).to(dev)
    ns = len(samples)
    near = torch.empty(ns, dtype=torch.int32, device=dev)
    added = torch.empty(ns, dtype=torch.int32, device=dev)
    inc = torch.empty(ns, dtype=torch.float64, device=dev)
    n0 = planner.nn.size()
    res = planner.batch_device(s.data_ptr(), ns, near.data_ptr(), added.data_ptr(), inc.data_ptr())
    E = int(res.total)
    off = planner._host(res.offsets, ns + 1, torch.int64)
    ids = planner._host(res.ids, E, torch.int32).view(np.uint32).astype(np.int64)
    dist = planner._host(res.dist, E, torch.float64)
    bits = planner._host(res.bits, E, torch.uint8)
    add = added.cpu().numpy().view(np.uint32).astype(np.int64)
    tree = planner.nn.states()
    assert len(tree) == n0 + int(res.added)
    seg = np.repeat(np.arange(ns), np.diff(off))
    x = np.empty((ns, sp.dim))
    ok = add != 0xFFFFFFFF
    x[ok] = tree[add[ok]]
    # the bits: checkMotion(nbh, x) and checkMotion(x, nbh)
    fwd = O.check_motions_mt(sp, ck, tree[ids], x[seg], 16)
    bwd = O.check_motions_mt(sp, ck, x[seg], tree[ids], 16)
    np.testing.assert_array_equal((bits & 1) != 0, fwd)
    np.testing.assert_array_equal((bits & 2) != 0, bwd)
    assert 0 < fwd.mean() and fwd.sum() != E
    # the neighbourhoods of up to 24 added states: brute force over ids < the state's own id
    for i in np.flatnonzero(ok)[:: max(1, int(ok.sum()) // 24)]:
        xi = int(add[i])
        k = int(math.ceil(planner.k_rrt * math.log(xi + 1)))
        oi, od, oc = O.knn(sp, tree[:xi], tree[xi][None], k)
        got = ids[off[i]:off[i + 1]]
        assert len(got) == int(oc[0])
        np.testing.assert_array_equal(got, oi[0, :oc[0]].astype(np.int64))
        assert_dist_close(dist[off[i]:off[i + 1]], od[0, :oc[0]])
    return res


def test_rrtstar_r3_spheres(gpu):
    """R^3 in [0,1]^3 with the 32-sphere field: everything bit-exact (no transcendental metric)"""
    sp = RealVectorStateSpace(3)
    c, r = W.sphere_field(32, 0.1, 7)
    ck = SpheresChecker(c, r)
    S.set_seed(42)
    smp = S.StateSampler(sp)
    x = smp.sample_uniform(6000)
    start = x[np.flatnonzero(O.is_valid(sp, ck, x[:50]))[0]]
    samples = x[50:4050]
    planner, ref = _run(sp, ck, start, samples, (1, 3, 60, 436, 1500, 2000), gpu)
    assert planner.stats["rounds"] >= 2  # the first batches depend on their own states
    res = _neighbourhoods_and_bits(planner, sp, ck, x[4050:6000], gpu)
    assert res.total > 0
    planner.close()


def test_rrtstar_se3_spheres(gpu):
    """SE(3) in [0,1]^3 with the sphere field, k_rrt = 446.5 (k from 1 to ~4,000 over the run)"""
    sp = SE3StateSpace(0.0, 1.0)
    c, r = W.sphere_field(32, 0.1, 7)
    ck = SpheresChecker(c, r)
    S.set_seed(42)
    smp = S.StateSampler(sp)
    x = smp.sample_uniform(7000)
    start = x[np.flatnonzero(O.is_valid(sp, ck, x[:50]))[0]]
    samples = x[50:6050]
    planner, ref = _run(sp, ck, start, samples, (1, 15, 484, 2500, 3000), gpu)
    _neighbourhoods_and_bits(planner, sp, ck, x[6050:7000], gpu)
    planner.close()


def test_rrtstar_se3_hypercube_existing_tree(gpu):
    """configs[2]'s checker (the HypercubeBenchmark passage on the translation) from a given tree:
    2,000 valid states whose parents / costs are a nearest-earlier chain, then 3,000 samples"""
    sp = SE3StateSpace(0.0, 1.0)
    ck = HypercubeChecker(3, 0.1)
    S.set_seed(7)
    smp = S.StateSampler(sp)
    x = smp.sample_uniform(150000)
    v = O.check_motions_mt(sp, ck, x, x, 16)  # isValid of each (a motion of length 0)
    assert v.sum() >= 2600
    tree = x[v][:2000]
    parent = np.full(len(tree), -1, np.int64)
    inc = np.zeros(len(tree))
    for j in range(1, len(tree)):
        oi, od, _ = O.knn(sp, tree[:j], tree[j][None], 1)
        parent[j], inc[j] = int(oi[0, 0]), od[0, 0]
    cost = np.zeros(len(tree))
    for j in range(1, len(tree)):
        cost[j] = cost[parent[j]] + inc[j]
    samples = x[~v][:2400]
    samples = np.concatenate([samples, x[v][2000:2600]])[np.random.default_rng(1).permutation(3000)]
    maxd = 0.2 * sp.getMaximumExtent()
    planner = RRTstarGPU(sp, ck, maxd, gpu)
    planner.add_tree(tree, parent, inc, cost)
    out = [planner.solve_batch(samples[a:a + 1000]) for a in range(0, 3000, 1000)]
    near, added, chosen = (np.concatenate([o[j] for o in out]) for j in range(3))
    ref = O.rrtstar(sp, ck, tree, parent, inc, cost, samples, maxd, planner.k_rrt)
    radd = ref["added"].astype(np.int64)
    radd[radd == 0xFFFFFFFF] = -1
    np.testing.assert_array_equal(near, ref["nearest"].astype(np.int64))
    np.testing.assert_array_equal(added, radd)
    np.testing.assert_array_equal(chosen, ref["parent_choice"])
    n = planner.n
    np.testing.assert_array_equal(planner.parent[:n], ref["parent"])
    np.testing.assert_array_equal(planner.cost[:n], ref["cost"])
    np.testing.assert_array_equal(planner.inc[:n], ref["inc"])
    assert ref["n_added"] > 50
    planner.close()


def test_rrtstar_bench_size_vs_sequential(gpu):
    """configs[2] RRT* at the size bench.py measures it (`workloads.rrt_star`): the bench's own
    10^6-state tree (bench._rrtstar_tree: the first 10^6 valid states of the reference stream, an
    RRT-like parent chain) and two 10^4-sample batches of the bench's sample stream, so k reaches
    ceil(k_rrt ln(n + 1)) = 6,169, the in-batch fixed point and the causal in-batch neighbour merge
    run at full size, and the second batch sees the first one's states in the index's tail.  Against
    the oracle's sequential RRT* (oracle/rrtstar.cpp over the GNAT restatement, RRTstar.cpp:247-542,
    603-618) on the same tree and samples: every sample's nearest, added id and chosen parent, the
    rewire and checkMotion counts, and the final parent / incCost / cost of every vertex."""
    import torch

    import bench
    from ompl_amd import DiscreteMotionValidatorGPU

    sp, ck = SE3StateSpace(0.0, 1.0), HypercubeChecker(3, 0.1)
    maxd = 0.2 * sp.getMaximumExtent()
    mv0 = DiscreteMotionValidatorGPU(sp, ck, gpu)
    tree, parent, inc, cost, qs = bench._rrtstar_tree(torch, sp, mv0, 1_000_000, gpu)
    mv0.close()
    ns = 10_000
    samples = qs.sample_uniform(2 * ns)
    planner = RRTstarGPU(sp, ck, maxd, gpu)
    planner.add_tree(tree, parent, inc, cost)
    out = planner.solve_batches([samples[:ns], samples[ns:]])
    near, added, chosen = (np.concatenate([o[j] for o in out]) for j in range(3))
    ref = O.rrtstar(sp, ck, tree, parent, inc, cost, samples, maxd, planner.k_rrt, use_gnat=True)
    assert ref["processed"] == 2 * ns
    radd = ref["added"].astype(np.int64)
    radd[radd == 0xFFFFFFFF] = -1
    np.testing.assert_array_equal(near, ref["nearest"].astype(np.int64))
    np.testing.assert_array_equal(added, radd)
    np.testing.assert_array_equal(chosen, ref["parent_choice"])
    n = planner.n
    assert n == len(tree) + ref["n_added"] and ref["n_added"] > 100
    st = planner.stats
    assert st["rewires"] == ref["rewires"] and st["checks_used"] == ref["checks"]
    # neighbourhoods at the benchmark's k: ceil(446.5 ln(10^6 + 1)) = 6,169 entries per added state
    k_full = int(math.ceil(planner.k_rrt * math.log(len(tree) + 1)))
    assert k_full == 6169 and st["neighbours"] >= k_full * ref["n_added"]
    np.testing.assert_array_equal(planner.parent[:n], ref["parent"])
    np.testing.assert_array_equal(planner.inc[:n], ref["inc"])
    np.testing.assert_array_equal(planner.cost[:n], ref["cost"])
    planner.close()
