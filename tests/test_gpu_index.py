"""The culled walks' sorted copy is built on the device and kept current incrementally:
states added after a build go to a Morton-ordered tail (no rebuild), removals are tombstoned in
place, and a rebuild happens only when the tail is full or a quarter of the states are gone.
Every answer along the way equals the oracle's (add / remove)."""
import numpy as np
import pytest

import pyoracle as O
from ompl_amd import NearestNeighborsGPU
from ompl_amd import workloads as W
from ompl_amd.spaces import RealVectorStateSpace, SE3StateSpace
from parity import assert_knn_parity

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("space", ["se3", "r6"])
def test_bitstar_style_loop_appends_without_rebuild(gpu, space):
    """BIT*-style: a batch of 100 new samples, then a batched query, repeated
    (ImplicitGraph.cpp:924-1000 addToSamples, then nearestK / nearestR on the grown set)."""
    sp = SE3StateSpace() if space == "se3" else RealVectorStateSpace(6)
    base, extra, q = W.reference_states(sp, (40000, 3000, 300), seed=42)
    nn = NearestNeighborsGPU(sp, gpu)
    nn.add(base)
    have = base
    for it in range(12):
        new = extra[it * 100:(it + 1) * 100]
        nn.add(new)
        have = np.concatenate([have, new])
        ids, d, _ = nn.nearestKBatch(q, 10)
        oi, od, _ = O.knn(sp, have, q, 18)
        assert_knn_parity(ids, d, oi, od, 10)
        if it % 4 == 3:
            off, rid, _ = nn.nearestRBatch(q[:100], 0.3)
            ooff, oid, _ = O.radius(sp, have, q[:100], 0.3)
            np.testing.assert_array_equal(off, ooff)
            np.testing.assert_array_equal(rid.astype(np.int64), oid.astype(np.int64))
    builds, appends = nn.index_stats()
    assert builds == 1 and appends >= 11  # the first query builds (over base + the first batch)


def test_tail_states_are_found_and_removed(gpu):
    """A query sitting on a tail state finds it at d = 0; after remove() it is gone at once."""
    sp = SE3StateSpace()
    base, extra = W.reference_states(sp, (20000, 80), seed=7)  # >= 64 queries: the batched (culled) path
    nn = NearestNeighborsGPU(sp, gpu)
    nn.add(base)
    nn.nearestKBatch(extra, 4)            # builds
    first = int(nn.add(extra)[0])
    ids, d, _ = nn.nearestKBatch(extra, 4)
    np.testing.assert_array_equal(ids[:, 0].astype(np.int64), np.arange(first, first + 80))
    assert (d[:, 0] == 0).all()
    for i in range(0, 80, 2):
        assert nn.remove(first + i)
    for i in range(0, 20000, 97):          # main-tile tombstones too
        assert nn.remove(i)
    ids, d, _ = nn.nearestKBatch(extra, 4)
    keep = np.setdiff1d(np.arange(20080), np.concatenate([first + np.arange(0, 80, 2), np.arange(0, 20000, 97)]))
    allx = np.concatenate([base, extra])
    oi, od, _ = O.knn(sp, allx[keep], extra, 12)
    assert_knn_parity(ids, d, keep[oi], od, 4)
    builds, appends = nn.index_stats()
    assert builds == 1 and appends >= 1


def test_rebuild_when_tail_full_or_many_removed(gpu):
    sp = RealVectorStateSpace(4)
    rng = np.random.default_rng(3)
    data = rng.uniform(0, 1, (30000, 4))
    q = rng.uniform(0, 1, (200, 4))
    nn = NearestNeighborsGPU(sp, gpu)
    nn.add(data[:4000])
    nn.nearestKBatch(q, 8)
    nn.add(data[4000:])                    # far more than the tail region holds: rebuild
    ids, d, _ = nn.nearestKBatch(q, 8)
    oi, od, _ = O.knn(sp, data, q, 16)
    assert_knn_parity(ids, d, oi, od, 8)
    b1, _ = nn.index_stats()
    assert b1 == 2
    gone = np.arange(0, 30000, 2)
    for i in gone:
        nn.remove(int(i))
    ids, d, _ = nn.nearestKBatch(q, 8)
    keep = np.arange(1, 30000, 2)
    oi, od, _ = O.knn(sp, data[keep], q, 16)
    assert_knn_parity(ids, d, keep[oi], od, 8)
    b2, _ = nn.index_stats()
    assert b2 == 3                          # half the states removed: rebuilt


def test_device_rrt_growth_feeds_the_tail(gpu):
    """States appended on the device by the RRT loop are placed in the tail at the next batched
    query (no host copy of the store)."""
    torch = pytest.importorskip("torch")
    from ompl_amd import DiscreteMotionValidatorGPU
    from ompl_amd.checkers import AllValidChecker
    sp = SE3StateSpace()
    tree, samples, q = W.reference_states(sp, (30000, 400, 200), seed=11)
    nn = NearestNeighborsGPU(sp, gpu)
    nn.add(tree)
    nn.nearestKBatch(q, 10)
    mv = DiscreteMotionValidatorGPU(sp, AllValidChecker(), gpu)
    ds = torch.from_numpy(samples).to(f"cuda:{gpu}")
    near = torch.empty(400, dtype=torch.int32, device=ds.device)
    added = torch.empty(400, dtype=torch.int32, device=ds.device)
    nn.rrt_grow_device(mv, ds.data_ptr(), 400, 0.2 * sp.getMaximumExtent(), near.data_ptr(), added.data_ptr())
    allx = nn.states()
    assert len(allx) == 30400
    ids, d, _ = nn.nearestKBatch(q, 10)
    oi, od, _ = O.knn(sp, allx, q, 18)
    assert_knn_parity(ids, d, oi, od, 10)
    builds, appends = nn.index_stats()
    assert builds == 1 and appends >= 1
