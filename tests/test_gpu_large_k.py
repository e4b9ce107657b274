"""GPU parity of the large-k path (k > 32: histogram threshold + candidate sort), the
RRT* neighbourhood size k = ceil(k_rrt log(n+1)) (RRTstar.cpp:603-618)."""
import numpy as np
import pytest

import pyoracle as O
from ompl_amd import NearestNeighborsGPU
from ompl_amd import workloads as W
from ompl_amd.spaces import KinematicChainSpace, RealVectorStateSpace, SE3StateSpace, SO3StateSpace
from parity import assert_knn_parity

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("nq", [3, 150])
def test_large_k_se3_rrtstar(gpu, nq):
    rng = np.random.default_rng(50 + nq)
    sp = SE3StateSpace()
    n = 100_000
    data, q = W.uniform_se3(rng, n), W.uniform_se3(rng, nq)
    k_rrt = W.rrt_star_k(n, 6)  # 5,141 at n = 1e5
    assert k_rrt == 5141
    nn = NearestNeighborsGPU(sp, gpu)
    nn.add(data)
    oi, od, _ = O.knn(sp, data, q, k_rrt + 8)
    for k in (33, 64, 100, 1000, k_rrt):
        ids, d, cnt = nn.nearestKBatch(q, k)
        assert (cnt == k).all()
        assert_knn_parity(ids, d, oi, od, k)


@pytest.mark.parametrize("name", ["r6", "so3", "chain12"])
def test_large_k_other_spaces(gpu, name):
    rng = np.random.default_rng(7)
    if name == "r6":
        sp, data, q = RealVectorStateSpace(6), W.uniform_rv(rng, 50000, 6), W.uniform_rv(rng, 100, 6)
    elif name == "so3":
        sp, data, q = SO3StateSpace(), W.uniform_quat(rng, 50000), W.uniform_quat(rng, 100)
    else:  # KinematicChain R^12 (RRT* on the chain: k in the thousands)
        sp, data, q = KinematicChainSpace(12, 1.0 / 12), W.uniform_chain(rng, 50000, 12), W.uniform_chain(rng, 100, 12)
    nn = NearestNeighborsGPU(sp, gpu)
    nn.add(data)
    oi, od, _ = O.knn(sp, data, q, 508)
    for k in (40, 500):
        ids, d, _ = nn.nearestKBatch(q, k)
        assert_knn_parity(ids, d, oi, od, k)


def test_large_k_more_than_stored(gpu):
    rng = np.random.default_rng(8)
    sp = SE3StateSpace()
    data, q = W.uniform_se3(rng, 300), W.uniform_se3(rng, 70)
    nn = NearestNeighborsGPU(sp, gpu)
    nn.add(data)
    nn.remove(5)
    ids, d, cnt = nn.nearestKBatch(q, 1000)
    assert (cnt == 299).all()
    keep = np.setdiff1d(np.arange(300), [5])
    oi, od, _ = O.knn(sp, data[keep], q, 299)
    assert_knn_parity(ids[:, :299], d[:, :299], keep[oi], od, 299)
    assert np.isinf(d[:, 299:]).all()


def test_large_k_se3_rrtstar_1e6(gpu):
    """M2(iii): RRT*'s k at the headline tree size, k = ceil(446.5 ln(n + 1)) = 6,169 at n = 10^6
    (RRTstar.cpp:603-618), on the reference RNG streams, a few queries."""
    sp = SE3StateSpace()
    data, q = W.reference_states(sp, [1_000_000, 4], seed=42)
    k_rrt = W.rrt_star_k(1_000_000, 6)
    assert k_rrt == 6169
    nn = NearestNeighborsGPU(sp, gpu)
    nn.add(data)
    ids, d, cnt = nn.nearestKBatch(q, k_rrt)
    assert (cnt == k_rrt).all()
    oi, od, _ = O.knn(sp, data, q, k_rrt + 8)
    assert_knn_parity(ids, d, oi, od, k_rrt)


def test_large_k_heavy_ties_take_the_exact_fallback(gpu):
    """50 distinct states, each stored 200 times in a row: whole chunks of the store are exact
    ties, so the fill pass's per-(query, chunk) slabs overflow and the queries are answered by
    the exact fallback kernel — still (distance, id) order, the lowest ids of a tie class first."""
    rng = np.random.default_rng(81)
    sp = SE3StateSpace()
    base = W.uniform_se3(rng, 50)
    data = np.repeat(base, 200, axis=0)
    q = np.concatenate([W.uniform_se3(rng, 40), base[:3]])
    nn = NearestNeighborsGPU(sp, gpu)
    nn.add(data)
    for k in (1000, 4321):
        ids, d, cnt = nn.nearestKBatch(q, k)
        assert (cnt == k).all()
        oi, od, _ = O.knn(sp, data, q, k)
        np.testing.assert_array_equal(ids.astype(np.int64), oi.astype(np.int64))  # ties: ids ascending
        assert_knn_parity(ids, d, oi, od, k)


def test_large_k_spatially_sorted_store(gpu):
    """A store whose id order follows space (states added in a sweep: sorted by x): a query's
    ~k candidates sit in a few contiguous id chunks, so the fill pass's per-(query, chunk) slabs
    overflow.  The overflow goes to the query's pool (ompl_gpu_nn_large_stats: spilled), not to the
    exact fallback, and the answers still equal the oracle's, (distance, id) order included."""
    rng = np.random.default_rng(82)
    sp = SE3StateSpace()
    data = W.uniform_se3(rng, 100_000)
    data = data[np.argsort(data[:, 0], kind="stable")]
    q = W.uniform_se3(rng, 64)
    nn = NearestNeighborsGPU(sp, gpu)
    nn.add(data)
    k = W.rrt_star_k(len(data), 6)
    ids, d, cnt = nn.nearestKBatch(q, k)
    spilled, exact = nn.large_stats()
    assert (cnt == k).all()
    assert spilled > 0, "the sorted store should overflow the per-chunk slabs"
    assert exact == 0, f"{exact} queries took the exact fallback"
    oi, od, _ = O.knn(sp, data, q, k + 8)
    assert_knn_parity(ids, d, oi, od, k)
