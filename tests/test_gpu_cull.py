"""The culled screen keeps a Morton-sorted copy of the store; it must stay exact across
incremental adds, removals, queries outside the stored bounding box and degenerate
(duplicate-heavy) data."""
import numpy as np
import pytest

import pyoracle as O
from ompl_amd import NearestNeighborsGPU
from ompl_amd import workloads as W
from ompl_amd.spaces import KinematicChainSpace, RealVectorStateSpace, SE3StateSpace
from parity import assert_knn_parity

pytestmark = pytest.mark.gpu


def _check(nn, sp, data_live, ids_live, q, k):
    ids, d, _ = nn.nearestKBatch(q, k)
    oi, od, _ = O.knn(sp, data_live, q, min(k + 8, len(data_live)))
    assert_knn_parity(ids, d, ids_live[oi], od, k)


def test_sorted_store_tracks_adds_and_removes(gpu):
    rng = np.random.default_rng(61)
    sp = SE3StateSpace()
    data = W.uniform_se3(rng, 120000)
    q = W.uniform_se3(rng, 500)
    nn = NearestNeighborsGPU(sp, gpu)
    nn.add(data[:50000])
    _check(nn, sp, data[:50000], np.arange(50000), q, 10)
    nn.add(data[50000:])                        # sorted copy is now stale -> rebuilt
    _check(nn, sp, data, np.arange(120000), q, 10)
    gone = rng.choice(120000, 20000, replace=False)
    for i in gone:
        nn.remove(int(i))
    keep = np.setdiff1d(np.arange(120000), gone)
    _check(nn, sp, data[keep], keep, q, 16)
    screened, _ = nn.stats()
    assert screened == 1500


def test_queries_outside_the_stored_box(gpu):
    rng = np.random.default_rng(62)
    sp = RealVectorStateSpace(6, -1.0, 1.0)
    data = W.uniform_rv(rng, 80000, 6, 0.0, 1.0)
    q = np.concatenate([W.uniform_rv(rng, 200, 6, -1.0, 0.0), W.uniform_rv(rng, 200, 6, 1.0, 3.0)])
    nn = NearestNeighborsGPU(sp, gpu)
    nn.add(data)
    _check(nn, sp, data, np.arange(80000), q, 10)


def test_clustered_and_duplicate_states(gpu):
    rng = np.random.default_rng(63)
    sp = SE3StateSpace()
    base = W.uniform_se3(rng, 300)
    data = np.repeat(base, 40, axis=0) + np.concatenate(
        [rng.normal(0, 1e-4, (12000, 3)), np.zeros((12000, 4))], axis=1)
    data[:, 3:] /= np.linalg.norm(data[:, 3:], axis=1, keepdims=True)
    q = base[rng.choice(300, 100)] + np.concatenate([rng.normal(0, 1e-3, (100, 3)), np.zeros((100, 4))], axis=1)
    nn = NearestNeighborsGPU(sp, gpu)
    nn.add(data)
    _check(nn, sp, data, np.arange(len(data)), q, 16)


def test_se3_quaternion_signs_and_norms(gpu):
    """The group walk stores sign-canonical quaternions and screens the rotation by the chord,
    whose error bound grows with the quaternions' norm excess: stored and query quaternions
    with w < 0 and norms a hair away from 1 keep the culled walk and lose no neighbour; norms
    far from 1 (3 %) make the bound useless, and the exact path answers instead."""
    rng = np.random.default_rng(64)
    sp = SE3StateSpace()
    for spread, culled in ((1e-9, True), (0.03, False)):
        data = W.uniform_se3(rng, 60000)
        data[:, 3:] *= rng.choice([-1.0, 1.0], size=(60000, 1)) * rng.uniform(1 - spread, 1 + spread, (60000, 1))
        q = W.uniform_se3(rng, 700)
        q[:, 3:] *= rng.choice([-1.0, 1.0], size=(700, 1)) * rng.uniform(1 - spread, 1 + spread, (700, 1))
        nn = NearestNeighborsGPU(sp, gpu)
        nn.add(data)
        _check(nn, sp, data, np.arange(len(data)), q, 10)
        scanned, total, qtiles = nn.cull_stats()
        if culled:
            assert 0 < scanned <= total
            assert scanned <= qtiles <= 8 * scanned  # each fetched tile is scanned by 1..G queries
        else:
            assert scanned == 0


def test_group_tail_and_small_batches(gpu):
    """Query counts that leave the last group of the walk partly empty."""
    rng = np.random.default_rng(65)
    sp = RealVectorStateSpace(5, 0.0, 1.0)
    data = W.uniform_rv(rng, 30000, 5)
    nn = NearestNeighborsGPU(sp, gpu)
    nn.add(data)
    for nq in (64, 67, 131, 1001):
        q = W.uniform_rv(rng, nq, 5)
        _check(nn, sp, data, np.arange(len(data)), q, 7)


@pytest.mark.parametrize("links", [4, 8, 12, 16])
def test_chain_culled_scan_16bit_rows(gpu, links):
    """The culled chain scan reads the joint positions as 16-bit fixed point (SortedStore::rows16,
    re-encoded whenever the store changes): exact against the oracle for every link bucket, for
    queries equal to stored states (distance 0, ties with the duplicates), after appends and after
    tombstones (a removed state's code carries the NaN marker and never enters a list)."""
    rng = np.random.default_rng(70 + links)
    sp = KinematicChainSpace(links, 1.0 / links)
    data = W.uniform_chain(rng, 30000, links)
    data[29000:] = data[:1000]                       # duplicates: tie classes resolved by id
    q = np.concatenate([W.uniform_chain(rng, 400, links), data[:100]])
    nn = NearestNeighborsGPU(sp, gpu)
    nn.add(data[:20000])
    _check(nn, sp, data[:20000], np.arange(20000), q, 10)
    nn.add(data[20000:])
    _check(nn, sp, data, np.arange(30000), q, 41)
    gone = rng.choice(30000, 3000, replace=False)
    for i in gone:
        nn.remove(int(i))
    keep = np.setdiff1d(np.arange(30000), gone)
    _check(nn, sp, data[keep], keep, q, 41)
    screened, fallbacks = nn.stats()
    assert screened == 3 * len(q) and fallbacks <= len(q) // 20
