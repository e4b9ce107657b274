"""GPU parity of the batch paths behind PRM* / BIT* / RRT: the culled radius
walk against the oracle on every path, the device-resident CSR radius API, the edge
endpoints the planners check after a neighbour query, and sequential RRT growth on device
against the oracle's step-by-step RRT loop (RRT.cpp:128-192)."""
import math

import numpy as np
import pytest

import pyoracle as O
from ompl_amd import DiscreteMotionValidatorGPU, NearestNeighborsGPU, abi
from ompl_amd import workloads as W
from ompl_amd.checkers import AllValidChecker, HypercubeChecker, KinematicChainChecker, SpheresChecker
from ompl_amd.spaces import KinematicChainSpace, RealVectorStateSpace, SE3StateSpace
from parity import assert_dist_close

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")


def _nn(sp, gpu, mode):
    nn = NearestNeighborsGPU(sp, gpu)
    nn.set_mode(mode)
    return nn


def _check_radius(nn, sp, data, q, r, keep=None):
    off, ids, d = nn.nearestRBatch(q, r)
    ooff, oids, od = O.radius(sp, data, q, r)
    if keep is not None:
        oids = keep[oids]
    np.testing.assert_array_equal(off, ooff)
    np.testing.assert_array_equal(ids.astype(np.int64), oids.astype(np.int64))
    assert_dist_close(d, od)
    return off


@pytest.mark.parametrize("name", ["se3", "r6"])
@pytest.mark.parametrize("mode", [0, 1])
def test_radius_culled_vs_oracle(gpu, name, mode):
    """mode 0 = culled fp32 walk + fp64 decision, mode 1 = exact fp64 scan: same CSR."""
    rng = np.random.default_rng(81)
    if name == "se3":
        sp, data, q = SE3StateSpace(), W.uniform_se3(rng, 60000), W.uniform_se3(rng, 300)
        radii = (0.0, 0.2, 0.45)
    else:
        sp, data, q = RealVectorStateSpace(6), W.uniform_rv(rng, 60000, 6), W.uniform_rv(rng, 300, 6)
        radii = (0.0, 0.15, 0.3)
    q[:5] = data[100:105]                       # stored states: d = 0 is inside (inclusive <=)
    nn = _nn(sp, gpu, mode)
    nn.add(data)
    for r in radii:
        off = _check_radius(nn, sp, data, q, r)
        if r == 0.0:
            assert (np.diff(off)[:5] >= 1).all()
    # the largest radius again: its longest segment overflowed the one-pass walk's first slab
    # (64 hits) above, so this call runs the single walk with the grown slab
    assert np.diff(off).max() > 64
    paths0 = nn.radius_path_stats()
    _check_radius(nn, sp, data, q, radii[-1])
    if mode == 0:
        one, two = nn.radius_path_stats()
        assert paths0[1] >= 1 and (one, two) == (paths0[0] + 1, paths0[1])  # the grown slab held it
        tiles, pairs = nn.radius_cull_stats()
        assert 0 < tiles <= pairs


def test_radius_long_segments_and_removals(gpu):
    """Segments longer than the LDS rank sort (radix-sort path), removed states, r = inf."""
    rng = np.random.default_rng(82)
    sp = SE3StateSpace()
    data, q = W.uniform_se3(rng, 5000), W.uniform_se3(rng, 70)
    nn = NearestNeighborsGPU(sp, gpu)
    nn.add(data)
    off = _check_radius(nn, sp, data, q, 2.2)         # most of the set per query: > 1024 entries
    assert np.diff(off).max() > 1024
    gone = rng.choice(5000, 900, replace=False)
    for i in gone:
        nn.remove(int(i))
    keep = np.setdiff1d(np.arange(5000), gone)
    _check_radius(nn, sp, data[keep], q, 0.5, keep)
    off, ids, _ = nn.nearestRBatch(q[:3], float("inf"))
    assert (np.diff(off) == len(keep)).all() and not np.isin(ids.astype(np.int64), gone).any()


def test_radius_device_api_and_edges(gpu):
    rng = np.random.default_rng(83)
    sp = SE3StateSpace()
    data, q = W.uniform_se3(rng, 80000), W.uniform_se3(rng, 400)
    nn = NearestNeighborsGPU(sp, gpu)
    nn.add(data)
    dev = f"cuda:{gpu}"
    dq = torch.from_numpy(q).to(dev)
    off = torch.empty(401, dtype=torch.int64, device=dev)
    r = 0.3
    tot = nn.radius_device(dq.data_ptr(), 400, r, off.data_ptr(), 0, 0, 0)   # size query
    ooff, oids, od = O.radius(sp, data, q, r)
    assert tot == int(ooff[-1])
    np.testing.assert_array_equal(off.cpu().numpy(), ooff.astype(np.int64))
    ids = torch.empty(tot, dtype=torch.int32, device=dev)
    dd = torch.empty(tot, dtype=torch.float64, device=dev)
    assert nn.radius_device(dq.data_ptr(), 400, r, off.data_ptr(), ids.data_ptr(), dd.data_ptr(), tot) == tot
    np.testing.assert_array_equal(ids.cpu().numpy().astype(np.int64), oids.astype(np.int64))
    assert_dist_close(dd.cpu().numpy(), od)
    # BIT* edges: checkMotion(vertex, sample) (BITstar.cpp:815)
    fr = torch.empty((tot, 7), dtype=torch.float64, device=dev)
    to = torch.empty_like(fr)
    nn.edges_device(dq.data_ptr(), 400, off.data_ptr(), ids.data_ptr(), 0, tot, True, fr.data_ptr(), to.data_ptr())
    nn.sync()
    seg = np.repeat(np.arange(400), np.diff(ooff).astype(np.int64))
    np.testing.assert_array_equal(fr.cpu().numpy(), q[seg])
    np.testing.assert_array_equal(to.cpu().numpy(), data[oids.astype(np.int64)])
    # PRM edges over a dense kNN result: checkMotion(state[n], state[m]) (PRM.cpp:582)
    k = 7
    ki = torch.empty((400, k), dtype=torch.int32, device=dev)
    kd = torch.empty((400, k), dtype=torch.float64, device=dev)
    nn.knn_device(dq.data_ptr(), 400, k, ki.data_ptr(), kd.data_ptr())
    fr2 = torch.empty((400 * k, 7), dtype=torch.float64, device=dev)
    to2 = torch.empty_like(fr2)
    nn.edges_device(dq.data_ptr(), 400, None, ki.data_ptr(), k, 400 * k, False, fr2.data_ptr(), to2.data_ptr())
    nn.sync()  # the device-resident calls are asynchronous on the handle's stream
    kin = ki.cpu().numpy().astype(np.int64).reshape(-1)
    np.testing.assert_array_equal(fr2.cpu().numpy(), data[kin])
    np.testing.assert_array_equal(to2.cpu().numpy(), np.repeat(q, k, axis=0))
    # capacity too small: offsets written, nothing else, total reported
    assert nn.radius_device(dq.data_ptr(), 400, r, off.data_ptr(), ids.data_ptr(), dd.data_ptr(), tot - 1) == tot


def _rrt_oracle(sp, ck, tree0, samples, maxd):
    tree = [row for row in tree0]
    near, added = [], []
    for s in samples:
        ids, d, _ = O.knn(sp, np.array(tree), s[None], 1)               # RRT.cpp:137
        j, dj = int(ids[0, 0]), float(d[0, 0])
        to = O.interpolate(sp, tree[j], s, maxd / dj) if dj > maxd else s.copy()   # :141-146
        v, _, _, _ = O.check_motions(sp, ck, np.array(tree[j])[None], to[None])   # :148
        near.append(j)
        if v[0]:
            tree.append(to)                                               # :170-173
            added.append(len(tree) - 1)
        else:
            added.append(abi.NO_ID32)
    return np.array(near), np.array(added, dtype=np.int64), np.array(tree)


@pytest.mark.parametrize("case", ["r6_allvalid", "se3_spheres", "se3_spheres_abort"])
def test_rrt_grow_matches_sequential_loop(gpu, case, monkeypatch):
    """The persistent grid, and (case *_abort: a spin limit of 1 poll makes the grid give up at
    its first wait) the abort path: counters restored, the batch re-run in the two-launch form
     — the same answer as the sequential loop either way."""
    if case.endswith("abort"):
        monkeypatch.setenv("OMPL_GPU_RRT_SPIN_LIMIT", "1")
    rng = np.random.default_rng(84)
    if case == "r6_allvalid":
        sp, ck = RealVectorStateSpace(6), AllValidChecker()
        tree0, samples = W.uniform_rv(rng, 700, 6), W.uniform_rv(rng, 300, 6)
    else:
        c, rr = W.sphere_field(32, 0.1, 7)
        sp, ck = SE3StateSpace(), SpheresChecker(c, rr)
        tree0, samples = W.uniform_se3(rng, 700), W.uniform_se3(rng, 300)
    maxd = 0.2 * sp.getMaximumExtent()
    nn = NearestNeighborsGPU(sp, gpu)
    nn.add(tree0)
    mv = DiscreteMotionValidatorGPU(sp, ck, gpu)
    dev = f"cuda:{gpu}"
    ds = torch.from_numpy(samples).to(dev)
    near = torch.empty(300, dtype=torch.int32, device=dev)
    added = torch.empty(300, dtype=torch.int32, device=dev)
    nn.rrt_grow_device(mv, ds.data_ptr(), 300, maxd, near.data_ptr(), added.data_ptr())
    if case.endswith("abort"):
        assert nn.rrt_aborts() == 1, "the persistent grid did not abort"
    en, ea, tree = _rrt_oracle(sp, ck, tree0, samples, maxd)
    np.testing.assert_array_equal(near.cpu().numpy().astype(np.int64), en)
    np.testing.assert_array_equal(added.cpu().numpy().astype(np.uint32).astype(np.int64), ea)
    assert nn.size() == len(tree) > len(tree0)
    np.testing.assert_array_equal(nn.states(), tree)
    assert mv.getValidMotionCount() == int((ea != abi.NO_ID32).sum())
    assert mv.getValidMotionCount() + mv.getInvalidMotionCount() == 300
    # the grown store answers queries like a store built by add()
    q = samples[:50] + 0.01
    ids, d, _ = nn.nearestKBatch(q, 5)
    oi, od, _ = O.knn(sp, tree, q, 5)
    np.testing.assert_array_equal(ids.astype(np.int64), oi.astype(np.int64))


@pytest.mark.parametrize("case", ["se3_spheres", "se3_hypercube", "r3_spheres", "chain12"])
def test_check_edges_device(gpu, case):
    """ompl_gpu_mv_check_edges_device: checkMotion over a neighbour result's edges read in place equals
    checking the pairs edges_device materialises (validity bits and the FIFO isValid count), for a CSR
    result with edges past the last segment, a dense kNN result with missing ids (k > n of a small
    store: the zero-length motion), both directions; the KinematicChain takes the materialising form."""
    rng = np.random.default_rng(91)
    dev = f"cuda:{gpu}"
    if case == "chain12":
        sp = KinematicChainSpace(12, 1.0 / 12)
        ck = KinematicChainChecker(W.horn_environment(12, math.log(12.0) / 12.0))
        draw = lambda n: W.uniform_chain(rng, n, 12)  # noqa: E731
        r = 0.9
    else:
        c, rad = W.sphere_field(32, 0.1, 7)
        if case == "r3_spheres":
            sp, ck = RealVectorStateSpace(3, 0.0, 1.0), SpheresChecker(c, rad)
            draw = lambda n: rng.uniform(0.0, 1.0, size=(n, 3))  # noqa: E731
            r = 0.08
        else:
            sp = SE3StateSpace()
            ck = SpheresChecker(c, rad) if case == "se3_spheres" else HypercubeChecker(3, 0.1)
            draw = lambda n: W.uniform_se3(rng, n)  # noqa: E731
            r = 0.5
    data, q = draw(30000), draw(300)
    nn = NearestNeighborsGPU(sp, gpu)
    nn.add(data)
    dq = torch.from_numpy(q).to(dev)
    off = torch.empty(301, dtype=torch.int64, device=dev)
    tot = nn.radius_device(dq.data_ptr(), 300, r, off.data_ptr(), 0, 0, 0)
    assert tot > 1000
    ids = torch.empty(tot + 37, dtype=torch.int32, device=dev)
    dd = torch.empty(tot + 37, dtype=torch.float64, device=dev)
    nn.radius_device(dq.data_ptr(), 300, r, off.data_ptr(), ids.data_ptr(), dd.data_ptr(), tot)
    for from_query in (True, False):
        for dense in (False, True):
            if dense:
                k, nq = 9, 300
                small = NearestNeighborsGPU(sp, gpu)
                small.add(data[:5])                                      # k > n: missing ids
                ki = torch.empty((nq, k), dtype=torch.int32, device=dev)
                kd = torch.empty((nq, k), dtype=torch.float64, device=dev)
                small.knn_device(dq.data_ptr(), nq, k, ki.data_ptr(), kd.data_ptr())
                src, offp, idp, stride, m = small, None, ki.data_ptr(), k, nq * k
            else:
                src, offp, idp, stride, m = nn, off.data_ptr(), ids.data_ptr(), 0, tot + 37  # 37 past the end
            fr = torch.zeros((m, sp.dim), dtype=torch.float64, device=dev)
            to = torch.zeros_like(fr)
            src.edges_device(dq.data_ptr(), 300, offp, idp, stride, m, from_query, fr.data_ptr(), to.data_ptr())
            src.sync()
            n_real = tot if not dense else m
            mv1 = DiscreteMotionValidatorGPU(sp, ck, gpu)
            v1 = mv1.checkMotions(fr.cpu().numpy()[:n_real], to.cpu().numpy()[:n_real])
            mv2 = DiscreteMotionValidatorGPU(sp, ck, gpu)
            val = torch.full((m,), 7, dtype=torch.uint8, device=dev)
            mv2.check_edges_device(src, dq.data_ptr(), 300, offp, idp, stride, m, from_query, val.data_ptr())
            mv2.sync()
            got = val.cpu().numpy()
            np.testing.assert_array_equal(got[:n_real].astype(bool), v1)
            assert (got[n_real:] == 0).all()
            assert mv2.stateChecks() == mv1.stateChecks()
            assert mv2.getValidMotionCount() == mv1.getValidMotionCount()
            assert mv2.getInvalidMotionCount() == mv1.getInvalidMotionCount()
    ov, _, _, checks = O.check_motions(sp, ck, fr.cpu().numpy(), to.cpu().numpy())
    np.testing.assert_array_equal(v1, ov)


def test_check_edges_device_back_to_back_streams(gpu):
    """two CSR check_edges_device calls with different query sets on the handles' own (separate,
    non-blocking) streams, synchronised only at the end: the second call's scratch
    (the per-edge query index, the neighbour query's results) must not be overwritten while the
    first call's motion kernel still reads it — every bit against the oracle validator."""
    rng = np.random.default_rng(17)
    dev = f"cuda:{gpu}"
    sp = SE3StateSpace()
    c, rad = W.sphere_field(32, 0.1, 7)
    ck = SpheresChecker(c, rad)
    data = W.uniform_se3(rng, 50000)
    nn = NearestNeighborsGPU(sp, gpu)
    nn.add(data)
    mv = DiscreteMotionValidatorGPU(sp, ck, gpu)
    r, nq = 0.45, 400
    qs = [W.uniform_se3(rng, nq) for _ in range(3)]
    caps = []
    for q in qs:  # sizes first (synchronous), then the timed-style back-to-back calls
        off = torch.empty(nq + 1, dtype=torch.int64, device=dev)
        dq = torch.from_numpy(q).to(dev)
        caps.append(nn.radius_device(dq.data_ptr(), nq, r, off.data_ptr(), 0, 0, 0))
    torch.cuda.synchronize()
    bufs = [(q, torch.from_numpy(q).to(dev), torch.empty(nq + 1, dtype=torch.int64, device=dev),
             torch.empty(cap, dtype=torch.int32, device=dev), torch.empty(cap, dtype=torch.float64, device=dev),
             torch.full((cap,), 7, dtype=torch.uint8, device=dev)) for q, cap in zip(qs, caps)]
    torch.cuda.synchronize()  # the buffers' fills (torch's stream) before the library's streams write them
    for (q, dq, off, ids, dd, val), cap in zip(bufs, caps):
        m = nn.radius_device(dq.data_ptr(), nq, r, off.data_ptr(), ids.data_ptr(), dd.data_ptr(), cap)
        assert m == cap
        mv.check_edges_device(nn, dq.data_ptr(), nq, off.data_ptr(), ids.data_ptr(), 0, m, True, val.data_ptr())
    nn.sync()
    mv.sync()
    for q, _, off, ids, _, val in bufs:
        o = off.cpu().numpy().astype(np.int64)
        i = ids.cpu().numpy().astype(np.int64)
        s1 = np.repeat(q, np.diff(o), axis=0)
        ov = O.check_motions_mt(sp, ck, s1, data[i], 16)
        np.testing.assert_array_equal(val.cpu().numpy().astype(bool), ov)
    mv.close()
    nn.close()
