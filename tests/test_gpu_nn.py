"""GPU parity tests of the nearest-neighbour path (through the C ABI) against the
oracle and the golden fixtures produced by the reference's NearestNeighborsLinear."""
import math

import numpy as np
import pytest

import pyoracle as O
from ompl_amd import NearestNeighborsGPU, abi
from ompl_amd import workloads as W
from ompl_amd.spaces import KinematicChainSpace, RealVectorStateSpace, SE3StateSpace, SO3StateSpace
from parity import assert_dist_close, assert_knn_parity

pytestmark = pytest.mark.gpu

SPACES = {
    "r6": lambda: RealVectorStateSpace(6),
    "se3": lambda: SE3StateSpace(),
    "so3": lambda: SO3StateSpace(),
    "chain12": lambda: KinematicChainSpace(12, 1.0 / 12),
}


def _sample(name, rng, n):
    return {"r6": lambda: W.uniform_rv(rng, n, 6), "se3": lambda: W.uniform_se3(rng, n),
            "so3": lambda: W.uniform_quat(rng, n), "chain12": lambda: W.uniform_chain(rng, n, 12)}[name]()


@pytest.fixture(params=["fast", "exact", "nocull"])
def path(request):
    """fast = fp32 screen (culled over the Morton-sorted copy for R^n / SE3) + fp64
    certificate, the default for batched queries; exact = the fp64 scan; nocull = the
    chunked fp32 screen.  All must give the same answers."""
    return request.param


def make_nn(sp, gpu, path):
    nn = NearestNeighborsGPU(sp, gpu)
    nn.set_mode({"fast": 0, "exact": 1, "nocull": 2}[path])
    return nn


def _oracle_ext(sp, data, q, k):
    K = min(k + 8, len(data))
    oi, od, _ = O.knn(sp, data, q, max(K, 1))
    return oi, od


@pytest.mark.parametrize("name", list(SPACES))
def test_knn_golden(gpu, path, golden, name):
    g = golden(f"nn_{name}.npz")
    sp = SPACES[name]()
    nn = make_nn(sp, gpu, path)
    nn.add(g["data"])
    assert nn.size() == len(g["data"])
    for k in (1, 10, 41):
        oi, od = _oracle_ext(sp, g["data"], g["queries"], k)
        for sl in (slice(0, 64), slice(0, 7)):  # tiled (nq >= 64) and stream (nq < 64) mappings
            ids, d, cnt = nn.nearestKBatch(g["queries"][sl], k)
            np.testing.assert_array_equal(cnt, g[f"knn{k}_cnt"][sl])
            assert_knn_parity(ids, d, oi[sl], od[sl], k)
            # the golden ids come from the reference's NearestNeighborsLinear: no ties in this data
            np.testing.assert_array_equal(ids.astype(np.int64), g[f"knn{k}_ids"][sl].astype(np.int64))
    assert nn.nearest(g["queries"][0]) == 17  # a stored state is its own nearest, d = 0


@pytest.mark.parametrize("name", list(SPACES))
@pytest.mark.parametrize("nq", [5, 300])
def test_knn_random_vs_oracle(gpu, path, name, nq):
    rng = np.random.default_rng(100 + nq)
    sp = SPACES[name]()
    data, q = _sample(name, rng, 60000), _sample(name, rng, nq)
    nn = make_nn(sp, gpu, path)
    nn.add(data[:25000])
    nn.add(data[25000:])  # growth path: the store is reallocated and copied
    oi, od = _oracle_ext(sp, data, q, 64)  # (distance, id)-sorted: top-k is a prefix
    for k in (1, 4, 10, 16, 33, 64):
        ids, d, cnt = nn.nearestKBatch(q, k)
        assert np.all(cnt == k)
        assert_knn_parity(ids, d, oi, od, k)


def test_knn_bitwise_for_realvector(gpu, path):
    """L2 uses only IEEE-exact operations (sub, mul, add, correctly rounded sqrt): the device
    distances must equal the reference formula bit for bit."""
    rng = np.random.default_rng(5)
    sp = RealVectorStateSpace(6)
    data, q = W.uniform_rv(rng, 20000, 6), W.uniform_rv(rng, 100, 6)
    nn = make_nn(sp, gpu, path)
    nn.add(data)
    ids, d, _ = nn.nearestKBatch(q, 16)
    oi, od, _ = O.knn(sp, data, q, 16)
    np.testing.assert_array_equal(d, od)
    np.testing.assert_array_equal(ids.astype(np.int64), oi.astype(np.int64))


def test_ties_resolved_by_id(gpu, path):
    """Exact distance ties (grid data): results ordered by (distance, id), like the oracle."""
    sp = RealVectorStateSpace(2)
    g = np.stack(np.meshgrid(np.arange(0, 1, 0.1), np.arange(0, 1, 0.1)), -1).reshape(-1, 2)
    data = np.concatenate([g, g])  # every state twice
    q = g[::7] + 0.0
    nn = make_nn(sp, gpu, path)
    nn.add(data)
    for k in (1, 4, 16, 64):
        for sub in (q, q[:3]):
            ids, d, _ = nn.nearestKBatch(sub, k)
            oi, od, _ = O.knn(sp, data, sub, k)
            np.testing.assert_array_equal(d, od)
            np.testing.assert_array_equal(ids.astype(np.int64), oi.astype(np.int64))


def test_k_edge_cases(gpu):
    sp = SE3StateSpace()
    rng = np.random.default_rng(1)
    data = W.uniform_se3(rng, 50)
    nn = NearestNeighborsGPU(sp, gpu)
    with pytest.raises(abi.EmptyError, match="No elements found"):
        nn.nearest(data[0])
    assert nn.nearestK(data[0], 5) == []
    assert nn.nearestR(data[0], 10.0) == []
    nn.add(data)
    assert nn.nearestK(data[0], 0) == []                  # k == 0 -> empty (GNAT.h:226-227)
    res = nn.nearestK(data[3], 64)                        # k > n -> n results, sorted
    assert len(res) == 50 and res[0] == 3
    oi, od, _ = O.knn(sp, data, data[3:4], 50)
    assert res == [int(x) for x in oi[0]]
    assert sorted(nn.nearestR(data[3], float("inf"))) == list(range(50))  # nearestR(inf) = all
    assert nn.nearestR(data[3], float("inf"))[0] == 3
    ids, d, cnt = nn.nearestKBatch(data[3:5], 65)         # large-k path: k > n -> n results
    assert (cnt == 50).all() and list(ids[0, :50]) == [int(x) for x in oi[0]]
    csp = KinematicChainSpace(12, 1 / 12)
    ch = NearestNeighborsGPU(csp, gpu)
    cdata, cq = W.uniform_chain(rng, 100, 12), W.uniform_chain(rng, 2, 12)
    ch.add(cdata)
    ids, d, cnt = ch.nearestKBatch(cq, 65)                 # chain, large-k path
    oi, od, _ = O.knn(csp, cdata, cq, 65)
    assert (cnt == 65).all()
    assert_knn_parity(ids, d, oi, od, 65)


def test_remove_and_clear(gpu, path):
    sp = SE3StateSpace()
    rng = np.random.default_rng(2)
    data, q = W.uniform_se3(rng, 3000), W.uniform_se3(rng, 80)
    nn = make_nn(sp, gpu, path)
    nn.add(data)
    removed = rng.choice(3000, 700, replace=False)
    for i in removed:
        assert nn.remove(int(i))
    assert not nn.remove(int(removed[0]))                  # already removed
    assert nn.size() == 2300 and len(nn.list()) == 2300
    keep = np.setdiff1d(np.arange(3000), removed)
    oi, od, _ = O.knn(sp, data[keep], q, 18)
    ids, d, _ = nn.nearestKBatch(q, 10)
    assert_knn_parity(ids, d, keep[oi], od, 10)
    off, rid, rd = nn.nearestRBatch(q, 0.6)
    assert not np.isin(rid.astype(np.int64), removed).any()
    nn.clear()
    assert nn.size() == 0
    with pytest.raises(abi.EmptyError):
        nn.nearest(q[0])


@pytest.mark.parametrize("name", list(SPACES))
def test_radius_golden(gpu, golden, name):
    g = golden(f"nn_{name}.npz")
    sp = SPACES[name]()
    nn = NearestNeighborsGPU(sp, gpu)
    nn.add(g["data"])
    r = float(g["radius"])
    for sl in (slice(0, 64), slice(0, 9)):
        off, ids, d = nn.nearestRBatch(g["queries"][sl], r)
        ooff, oids, od = O.radius(sp, g["data"], g["queries"][sl], r)
        np.testing.assert_array_equal(off, ooff)
        np.testing.assert_array_equal(ids.astype(np.int64), oids.astype(np.int64))
        assert_dist_close(d, od)
        gofs = g["radius_off"][: sl.stop + 1]
        np.testing.assert_array_equal(off, gofs - gofs[0])


@pytest.mark.parametrize("nq", [3, 200])
def test_radius_random_vs_oracle(gpu, nq):
    rng = np.random.default_rng(7 + nq)
    sp = SE3StateSpace()
    data, q = W.uniform_se3(rng, 50000), W.uniform_se3(rng, nq)
    nn = NearestNeighborsGPU(sp, gpu)
    nn.add(data)
    for r in (0.0, 0.25, 0.5):
        off, ids, d = nn.nearestRBatch(q, r)
        ooff, oids, od = O.radius(sp, data, q, r)
        np.testing.assert_array_equal(off, ooff)
        np.testing.assert_array_equal(ids.astype(np.int64), oids.astype(np.int64))
        assert_dist_close(d, od)


def test_large_tree_properties(gpu, path):
    """1e6 SE(3) tree (the headline size): stream and tiled mappings agree, results are sorted,
    radius and kNN are consistent, and a sample of queries matches the oracle."""
    rng = np.random.default_rng(42)
    sp = SE3StateSpace()
    data, q = W.uniform_se3(rng, 1_000_000), W.uniform_se3(rng, 2000)
    nn = make_nn(sp, gpu, path)
    nn.add(data)
    ids, d, _ = nn.nearestKBatch(q, 10)
    ids_s, d_s, _ = nn.nearestKBatch(q[:40], 10)          # stream mapping
    np.testing.assert_array_equal(ids[:40], ids_s)
    np.testing.assert_array_equal(d[:40], d_s)
    assert np.all(np.diff(d, axis=1) >= 0)
    oi, od = _oracle_ext(sp, data, q[:12], 10)
    assert_knn_parity(ids[:12], d[:12], oi, od, 10)
    r = float(np.median(d[:, 9]))
    off, rid, rd = nn.nearestRBatch(q[:100], r)
    for j in range(100):
        seg = set(rid[off[j]:off[j + 1]].tolist())
        inside = ids[j][d[j] <= r]
        assert set(inside.tolist()) <= seg
    again = nn.nearestKBatch(q, 10)
    np.testing.assert_array_equal(again[0], ids)           # idempotent


def test_device_resident_api(gpu):
    torch = pytest.importorskip("torch")
    rng = np.random.default_rng(8)
    sp = SE3StateSpace()
    data, q = W.uniform_se3(rng, 100000), W.uniform_se3(rng, 1000)
    nn = NearestNeighborsGPU(sp, gpu)
    nn.add(data)
    dq = torch.from_numpy(q).to(f"cuda:{gpu}")
    di = torch.empty((1000, 10), dtype=torch.int32, device=dq.device)
    dd = torch.empty((1000, 10), dtype=torch.float64, device=dq.device)
    nn.knn_device(dq.data_ptr(), 1000, 10, di.data_ptr(), dd.data_ptr())
    nn.sync()
    ids, d, _ = nn.nearestKBatch(q, 10)
    np.testing.assert_array_equal(di.cpu().numpy().astype(np.int64), ids.astype(np.int64))
    np.testing.assert_array_equal(dd.cpu().numpy(), d)
    # RRT extend step (RRT.cpp:137-146)
    maxd = 0.2 * sp.getMaximumExtent()
    fr = torch.empty_like(dq)
    to = torch.empty_like(dq)
    nn.steer_device(dq.data_ptr(), 1000, di.data_ptr(), 10, maxd, fr.data_ptr(), to.data_ptr())
    nn.sync()
    fr, to = fr.cpu().numpy(), to.cpu().numpy()
    np.testing.assert_array_equal(fr, data[ids[:, 0].astype(np.int64)])
    for i in range(0, 1000, 37):
        dd_ = O.distance(sp, fr[i], q[i])
        exp = O.interpolate(sp, fr[i], q[i], maxd / dd_) if dd_ > maxd else q[i]
        np.testing.assert_array_equal(to[i], exp)


def test_chain_features_exact(gpu):
    """KCHAIN: the cumulative cos/sin features are computed on the host with the same libm
    as the reference, so distances are bit-identical."""
    rng = np.random.default_rng(12)
    sp = KinematicChainSpace(12, 1.0 / 12)
    data, q = W.uniform_chain(rng, 20000, 12), W.uniform_chain(rng, 100, 12)
    nn = NearestNeighborsGPU(sp, gpu)
    nn.add(data)
    ids, d, _ = nn.nearestKBatch(q, 10)
    oi, od, _ = O.knn(sp, data, q, 10)
    np.testing.assert_array_equal(d, od)
    np.testing.assert_array_equal(ids.astype(np.int64), oi.astype(np.int64))
    st = nn.states(0, 5)
    np.testing.assert_array_equal(st, data[:5])
    assert math.isfinite(float(st.sum()))


@pytest.mark.parametrize("name", ["se3", "r6", "so3"])
def test_fast_path_is_used_and_certified(gpu, name):
    rng = np.random.default_rng(31)
    sp = SPACES[name]()
    data, q = _sample(name, rng, 200000), _sample(name, rng, 2000)
    nn = NearestNeighborsGPU(sp, gpu)
    nn.add(data)
    ids, d, _ = nn.nearestKBatch(q, 10)
    screened, fallbacks = nn.stats()
    assert screened == 2000 and fallbacks < 200
    oi, od = _oracle_ext(sp, data, q[:50], 10)
    assert_knn_parity(ids[:50], d[:50], oi, od, 10)


def test_fast_path_fallback_when_certificate_fails(gpu):
    """Rotations within 1e-3 rad of each other: the fp32 screen's error bound exceeds the
    distance gaps, certificates fail, and the exact re-run must give the exact answer."""
    rng = np.random.default_rng(32)
    sp = SO3StateSpace()
    v = rng.normal(0, 1e-3, (60000, 3))
    data = np.column_stack([v, np.ones(60000)])
    data /= np.linalg.norm(data, axis=1, keepdims=True)
    q = data[rng.choice(60000, 300, replace=False)] + rng.normal(0, 1e-5, (300, 4))
    q /= np.linalg.norm(q, axis=1, keepdims=True)
    nn = NearestNeighborsGPU(sp, gpu)
    nn.add(data)
    ids, d, _ = nn.nearestKBatch(q, 10)
    screened, fallbacks = nn.stats()
    assert screened == 300 and fallbacks > 0
    oi, od = _oracle_ext(sp, data, q, 10)
    assert_knn_parity(ids, d, oi, od, 10)


def test_bounded_rerun_se3_near_rotations(gpu):
    """SE(3) states whose rotations differ by < 1e-3 rad: the screen's rotation error bound
    (fp32 acos near 1) fails certificates; the bounded exact re-run (one store pass keeping
    d <= the certificate's exact k-th distance) must return the oracle's lists."""
    rng = np.random.default_rng(36)
    sp = SE3StateSpace()
    n = 40000
    v = rng.normal(0, 1e-3, (n, 3))
    quat = np.column_stack([v, np.ones(n)])
    quat /= np.linalg.norm(quat, axis=1, keepdims=True)
    data = np.column_stack([rng.uniform(0, 1, (n, 3)) * 0.02, quat])
    q = data[rng.choice(n, 200, replace=False)].copy()
    q[:, :3] += rng.normal(0, 1e-4, (200, 3))
    nn = NearestNeighborsGPU(sp, gpu)
    nn.add(data)
    ids, d, _ = nn.nearestKBatch(q, 10)
    screened, fallbacks = nn.stats()
    assert screened == 200 and fallbacks > 0
    assert nn.rerun_stats() < fallbacks  # most took the bounded pass
    oi, od = _oracle_ext(sp, data, q, 10)
    assert_knn_parity(ids, d, oi, od, 10)


def test_rerun_beyond_bounded_capacity(gpu):
    """More uncertified queries than the bounded pass takes (512): the persistent re-run launch
    (knn.hip knn_rerun_kernel: bounded pass, rank select, full scans between grid-wide barriers)
    moves the excess to the full-scan list in its second phase and answers it in its third; every
    list must still be the oracle's, and a second batch on the same handle (the barrier counter
    re-zeroed by the batch's first kernel) must be too."""
    rng = np.random.default_rng(38)
    sp = SE3StateSpace()
    n = 30000
    v = rng.normal(0, 1e-3, (n, 3))
    quat = np.column_stack([v, np.ones(n)])
    quat /= np.linalg.norm(quat, axis=1, keepdims=True)
    data = np.column_stack([rng.uniform(0, 1, (n, 3)) * 0.02, quat])
    nn = NearestNeighborsGPU(sp, gpu)
    nn.add(data)
    for rep in range(2):
        q = data[rng.choice(n, 1500, replace=False)].copy()
        q[:, :3] += rng.normal(0, 1e-4, (1500, 3))
        s0, f0 = nn.stats()
        ids, d, _ = nn.nearestKBatch(q, 10)
        s1, f1 = nn.stats()
        assert s1 - s0 == 1500 and f1 - f0 > 512, (rep, f1 - f0)
        oi, od = _oracle_ext(sp, data, q, 10)
        assert_knn_parity(ids, d, oi, od, 10)


def test_bounded_rerun_overflow_takes_full_path(gpu):
    """2,000 identical copies of one state: every query next to it has more than the bounded
    re-run's candidate cap (1,024) at d <= its k-th distance, so the full exact scan answers."""
    rng = np.random.default_rng(37)
    sp = SE3StateSpace()
    base = W.uniform_se3(rng, 30000)
    dup = np.repeat(base[:1], 2000, axis=0)
    data = np.concatenate([base[1:15000], dup, base[15000:]])
    q = np.repeat(base[:1], 8, axis=0)
    q[:, :3] += rng.normal(0, 1e-6, (8, 3))
    q = np.concatenate([q, W.uniform_se3(rng, 120)])
    nn = NearestNeighborsGPU(sp, gpu)
    nn.add(data)
    ids, d, _ = nn.nearestKBatch(q, 10)
    screened, fallbacks = nn.stats()
    assert screened == len(q) and fallbacks >= 8 and nn.rerun_stats() >= 8
    oi, od = _oracle_ext(sp, data, q, 10)
    assert_knn_parity(ids, d, oi, od, 10)
    # the duplicates' tie class is resolved by insertion id, as on the exact path
    np.testing.assert_array_equal(ids[:8].astype(np.int64), np.tile(np.arange(14999, 15009), (8, 1)))


@pytest.mark.parametrize("k", [10, 41])
def test_chain_screen_is_used_and_exact(gpu, k):
    """KinematicChain: the fp32 joint-position screen + fp64 certificate (PRM*'s k = 41,
    ConnectionStrategy.h:147) returns the oracle's neighbours bit for bit."""
    rng = np.random.default_rng(33)
    sp = SPACES["chain12"]()
    data, q = W.uniform_chain(rng, 40000, 12), W.uniform_chain(rng, 300, 12)
    nn = NearestNeighborsGPU(sp, gpu)
    nn.add(data)
    ids, d, cnt = nn.nearestKBatch(q, k)
    screened, fallbacks = nn.stats()
    assert screened == 300 and fallbacks < 30 and (cnt == k).all()
    oi, od, _ = O.knn(sp, data, q[:40], k)
    np.testing.assert_array_equal(d[:40], od)
    np.testing.assert_array_equal(ids[:40].astype(np.int64), oi.astype(np.int64))
    gone = rng.choice(40000, 5000, replace=False)
    for i in gone[:50]:
        nn.remove(int(i))
    ids2, _, _ = nn.nearestKBatch(q, k)
    assert not np.isin(ids2.astype(np.int64), gone[:50]).any()


@pytest.mark.parametrize("scale", [1e20, 1e-25])
def test_extreme_coordinates(gpu, path, scale):
    """Coordinates near fp32 overflow (1e20: squared fp32 distances overflow to inf) or far
    below fp32 precision (1e-25: squares underflow): the screens must not drop neighbours —
    the result equals the reference formula bit for bit (R^n uses only exact IEEE ops)."""
    rng = np.random.default_rng(41)
    sp = RealVectorStateSpace(4)
    data, q = W.uniform_rv(rng, 5000, 4) * scale, W.uniform_rv(rng, 100, 4) * scale
    nn = make_nn(sp, gpu, path)
    nn.add(data)
    for k in (1, 10):
        ids, d, cnt = nn.nearestKBatch(q, k)
        oi, od, _ = O.knn(sp, data, q, k)
        assert (cnt == k).all()
        np.testing.assert_array_equal(d, od)
        np.testing.assert_array_equal(ids.astype(np.int64), oi.astype(np.int64))
    r = float(np.median(od[:, 9]))
    off, rid, rd = nn.nearestRBatch(q, r)
    ooff, oids, _ = O.radius(sp, data, q, r)
    np.testing.assert_array_equal(off, ooff)
    np.testing.assert_array_equal(rid.astype(np.int64), oids.astype(np.int64))
