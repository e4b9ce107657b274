"""Small-batch kNN over the fp32 rows (ompl_amd/csrc/knn_stream32.hip): RRT's one nearest()
per iteration (RRT.cpp:137, NearestNeighborsGNAT.h:209-233).  The fast mode routes nq < 64,
k <= 16 on SE3 / R^n to the fp32 stream with in-chunk fp64 refinement; its answers must equal
the oracle's exact (distance, id) lists, and the exact fp64 stream's bit for bit."""
import numpy as np
import pytest

import pyoracle as O
from ompl_amd import NearestNeighborsGPU
from ompl_amd import workloads as W
from ompl_amd.spaces import RealVectorStateSpace, SE3StateSpace
from parity import assert_knn_parity

pytestmark = pytest.mark.gpu

SPACES = {
    "r3": (lambda: RealVectorStateSpace(3), lambda rng, n: W.uniform_rv(rng, n, 3)),
    "r6": (lambda: RealVectorStateSpace(6), lambda rng, n: W.uniform_rv(rng, n, 6)),
    "r12": (lambda: RealVectorStateSpace(12), lambda rng, n: W.uniform_rv(rng, n, 12)),
    "se3": (lambda: SE3StateSpace(), lambda rng, n: W.uniform_se3(rng, n)),
}


def _pair(sp, gpu, data):
    fast, exact = NearestNeighborsGPU(sp, gpu), NearestNeighborsGPU(sp, gpu)
    fast.set_mode(0)
    exact.set_mode(1)
    for nn in (fast, exact):
        nn.add(data)
    return fast, exact


@pytest.mark.parametrize("name", list(SPACES))
def test_stream32_vs_oracle(gpu, name):
    mk_sp, sample = SPACES[name]
    rng = np.random.default_rng(321)
    sp = mk_sp()
    data = sample(rng, 150_000)
    data[1000:1010] = data[5]            # exact ties: equal distances, resolved by id
    q = np.concatenate([sample(rng, 5), data[[5, 77_777]]])  # stored states: their own nearest at d = 0
    fast, exact = _pair(sp, gpu, data)
    oi, od, _ = O.knn(sp, data, q, 24)
    for k in (1, 4, 10, 16):
        for sl in (slice(0, 1), slice(0, len(q))):
            ids, d, cnt = fast.nearestKBatch(q[sl], k)
            assert np.all(cnt == k)
            assert_knn_parity(ids, d, oi[sl], od[sl], k)
            ei, ed, _ = exact.nearestKBatch(q[sl], k)
            np.testing.assert_array_equal(ids, ei)
            np.testing.assert_array_equal(d, ed)
    assert fast.nearest(data[77_777]) == 77_777


def test_stream32_tombstones_and_growth(gpu):
    rng = np.random.default_rng(5)
    sp = SE3StateSpace()
    data = W.uniform_se3(rng, 40_000)
    fast, exact = _pair(sp, gpu, data[:30_000])
    for nn in (fast, exact):
        nn.add(data[30_000:])
    q = W.uniform_se3(rng, 3)
    first, _, _ = fast.nearestKBatch(q, 4)
    for nn in (fast, exact):
        for i in set(first[:, :2].reshape(-1).tolist()):
            assert nn.remove(int(i))
    ids, d, _ = fast.nearestKBatch(q, 4)
    ei, ed, _ = exact.nearestKBatch(q, 4)
    np.testing.assert_array_equal(ids, ei)
    np.testing.assert_array_equal(d, ed)
    assert not set(first[:, :2].reshape(-1).tolist()) & set(ids.reshape(-1).tolist())


def test_stream32_fewer_states_than_k(gpu):
    sp = RealVectorStateSpace(6)
    data = W.uniform_rv(np.random.default_rng(9), 5, 6)
    fast, _ = _pair(sp, gpu, data)
    ids, d, cnt = fast.nearestKBatch(data[:2], 10)
    assert np.all(cnt == 5)
    oi, od, _ = O.knn(sp, data, data[:2], 5)
    np.testing.assert_array_equal(ids[:, :5], oi)


def test_stream32_large_store_equals_exact(gpu):
    """10^7-class store (the 2,048-state chunk mapping, n >= 4M): bit-identical to the exact
    fp64 stream on a few single queries (RRT semantics)."""
    rng = np.random.default_rng(77)
    sp = SE3StateSpace()
    data = W.uniform_se3(rng, 4_500_000)
    fast, exact = _pair(sp, gpu, data)
    q = np.concatenate([W.uniform_se3(rng, 3), data[[4_499_999]]])
    for k in (1, 10):
        for i in range(len(q)):
            ids, d, _ = fast.nearestKBatch(q[i:i + 1], k)
            ei, ed, _ = exact.nearestKBatch(q[i:i + 1], k)
            np.testing.assert_array_equal(ids, ei)
            np.testing.assert_array_equal(d, ed)
    assert fast.nearest(data[4_499_999]) == 4_499_999


@pytest.mark.parametrize("copies", [3_000, 70_000])
def test_stream32_split_batch_and_overflow(gpu, copies):
    """The split form (n >= 4M: screen-only stream, candidates per chunk, multi-block refine):
    a batch of queries at k = 1 / 4 / 16 buckets, and a store holding 3,000 copies of one state
    next to the queries, so that whole chunks tie at the same screened distance and overflow
    their candidate lists (the refine kernel rescans them; with 70,000 copies more chunks
    overflow than its list holds, so it rescans every chunk under the threshold): ids and
    distances equal the exact fp64 stream."""
    rng = np.random.default_rng(78)
    sp = SE3StateSpace()
    data = W.uniform_se3(rng, 4_300_000)
    data[1_000_000:1_000_000 + copies] = data[5]
    fast, exact = _pair(sp, gpu, data)
    q = np.concatenate([W.uniform_se3(rng, 5), data[[5]], data[[2_000_000]]])
    q[6, :3] += 1e-7
    for k in (1, 3, 12):
        ids, d, _ = fast.nearestKBatch(q, k)
        ei, ed, _ = exact.nearestKBatch(q, k)
        np.testing.assert_array_equal(ids, ei)
        np.testing.assert_array_equal(d, ed)
    ids, _, _ = fast.nearestKBatch(q[5:6], 12)
    np.testing.assert_array_equal(ids[0], np.concatenate([[5], np.arange(1_000_000, 1_000_011)]))
