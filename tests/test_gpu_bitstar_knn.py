"""GPU parity of the culled group walk at 33 <= k <= 61 (K2 = 64: one list entry per lane).
BIT*'s default neighbourhood is kNN, useKNearest_ = true (bitstar/ImplicitGraph.h:463), with
k = ceil(1.1 (e + e/d) ln n) (bitstar/src/ImplicitGraph.cpp:313-316, 1383-1387): 57 at
n = 10^7 on SE(3) (d = 6); SE(3) PRM* asks k = ceil((e + e/6) ln n) = 44 at 10^6.
The walk must serve these k itself (cull counters move), not the brute-force histogram path."""
import math

import numpy as np
import pytest

import pyoracle as O
from ompl_amd import NearestNeighborsGPU
from ompl_amd import workloads as W
from ompl_amd.spaces import RealVectorStateSpace, SE3StateSpace
from parity import assert_knn_parity, oracle_knn_mt

pytestmark = pytest.mark.gpu


def bitstar_k(n, d):
    return int(math.ceil(1.1 * (math.e + math.e / d) * math.log(n)))


def test_bitstar_k_values():
    assert bitstar_k(10_000_000, 6) == 57
    assert W.prm_star_k(1_000_000, 6) == 44


@pytest.mark.parametrize("name", ["se3", "r6"])
def test_mid_k_walk(gpu, name):
    rng = np.random.default_rng(61)
    if name == "se3":
        sp, data, q = SE3StateSpace(), W.uniform_se3(rng, 200_000), W.uniform_se3(rng, 300)
    else:
        sp, data, q = RealVectorStateSpace(6), W.uniform_rv(rng, 200_000, 6), W.uniform_rv(rng, 300, 6)
    nn = NearestNeighborsGPU(sp, gpu)
    nn.add(data)
    oi, od = oracle_knn_mt(O, sp, data, q, 70)
    for k in (33, 44, 57, 61):
        before = nn.cull_stats()[2]
        ids, d, cnt = nn.nearestKBatch(q, k)
        assert nn.cull_stats()[2] > before, f"k={k} did not take the culled walk"
        assert (cnt == k).all()
        assert_knn_parity(ids, d, oi, od, k)


def test_mid_k_walk_paths_agree(gpu):
    """k = 57 on the culled walk, the exact fp64 scan and the unculled screen: identical."""
    rng = np.random.default_rng(62)
    sp = SE3StateSpace()
    data, q = W.uniform_se3(rng, 50_000), W.uniform_se3(rng, 128)
    nn = NearestNeighborsGPU(sp, gpu)
    nn.add(data)
    a = nn.nearestKBatch(q, 57)
    nn.set_mode(1)
    b = nn.nearestKBatch(q, 57)
    nn.set_mode(2)
    c = nn.nearestKBatch(q, 57)
    for x in (b, c):
        assert np.array_equal(a[0], x[0]) and np.array_equal(a[1], x[1])


def test_mid_k_small_store_and_removals(gpu):
    """k close to the store size, removed states, duplicates: the walk's list is not full."""
    rng = np.random.default_rng(63)
    sp = SE3StateSpace()
    data = W.uniform_se3(rng, 80)
    data = np.concatenate([data, data[:10]])  # exact duplicates: ties broken by id
    q = np.concatenate([W.uniform_se3(rng, 70), data[:5]])
    nn = NearestNeighborsGPU(sp, gpu)
    nn.add(data)
    for r in (3, 17, 50):
        nn.remove(r)
    keep = np.setdiff1d(np.arange(len(data)), [3, 17, 50])
    oi, od, _ = O.knn(sp, data[keep], q, 61)
    ids, d, cnt = nn.nearestKBatch(q, 61)
    assert (cnt == 61).all()
    assert_knn_parity(ids, d, keep[oi], od, 61)


def test_bitstar_knn_1e7_reference_streams(gpu):
    """BIT*'s k = 57 over 10^7 SE(3) samples of the reference RNG streams (RNG::setSeed(42),
    the sample sampler then the vertex sampler), 32 vertices against the oracle's brute force."""
    sp = SE3StateSpace()
    data, q = W.reference_states(sp, [10_000_000, 32], seed=42)
    k = bitstar_k(len(data), 6)
    nn = NearestNeighborsGPU(sp, gpu)
    nn.add(data)
    # the walk runs for >= 64 queries (kStreamMaxQ): pad the batch with more vertices
    qq = np.concatenate([q, W.uniform_se3(np.random.default_rng(5), 96)])
    before = nn.cull_stats()[2]
    ids, d, cnt = nn.nearestKBatch(qq, k)
    assert nn.cull_stats()[2] > before
    oi, od = oracle_knn_mt(O, sp, data, q, k + 6)
    assert (cnt == k).all()
    assert_knn_parity(ids[:32], d[:32], oi, od, k)
