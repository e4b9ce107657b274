"""Multi-rank tests of the multi-GPU decomposition over gloo (world size 2 and 3, CPU): query
sharding covers every query exactly once; the tree-sharded all_gather + merge reproduces the
single-process top-k exactly (ids and distances, ties by id); the radius CSR exchange (count
all_gather + padded payload) reproduces nearestR; the per-batch state gather delivers every
rank's new states to every replica in rank order.  test_sharded_hip_path_world2 runs the same
with the HIP kernels answering each shard; test_bench_spawn_plumbing covers `bench.py --gpus N`."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from ompl_amd.shard import allgather_merge, merge_topk, shard_bounds


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, result_dir):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import sys

    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "oracle"))
    import pyoracle as O

    from ompl_amd import workloads as W
    from ompl_amd.spaces import SE3StateSpace

    sp = SE3StateSpace()
    data = W.uniform_se3(np.random.default_rng(42), 4000)
    data[3001] = data[17]  # an exact tie across shards
    q = W.uniform_se3(np.random.default_rng(5), 50)
    q[0] = data[17]
    k = 12
    lo, hi = shard_bounds(len(data), rank, world)
    li, ld, lc = O.knn(sp, data[lo:hi], q, k)
    gid = torch.from_numpy(li.astype(np.int64) + lo)
    gid[torch.from_numpy(li == 0xFFFFFFFF)] = -1
    d, i = allgather_merge(torch.from_numpy(ld), gid, k)
    # query sharding: every rank's slice, concatenated, covers all queries once
    qlo, qhi = shard_bounds(len(q), rank, world)
    cover = torch.tensor([qhi - qlo], dtype=torch.int64)
    dist.all_reduce(cover)
    np.savez(os.path.join(result_dir, f"r{rank}.npz"), d=d.numpy(), i=i.numpy(), cover=cover.numpy())
    dist.barrier()
    dist.destroy_process_group()


def test_tree_sharded_merge_world2(tmp_path):
    port = _free_port()
    mp.start_processes(_worker, args=(2, port, str(tmp_path)), nprocs=2, join=True, start_method="spawn")
    import sys

    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "oracle"))
    import pyoracle as O

    from ompl_amd import workloads as W
    from ompl_amd.spaces import SE3StateSpace

    sp = SE3StateSpace()
    data = W.uniform_se3(np.random.default_rng(42), 4000)
    data[3001] = data[17]
    q = W.uniform_se3(np.random.default_rng(5), 50)
    q[0] = data[17]
    oi, od, _ = O.knn(sp, data, q, 12)
    for r in range(2):
        z = np.load(tmp_path / f"r{r}.npz")
        np.testing.assert_array_equal(z["i"], oi.astype(np.int64))
        np.testing.assert_array_equal(z["d"], od)
        assert int(z["cover"][0]) == len(q)
    assert list(oi[0, :2]) == [17, 3001]  # tie resolved by id across shards


def test_shard_bounds_partition():
    for n in (0, 1, 7, 100, 1001):
        for w in (1, 2, 3, 8):
            parts = [shard_bounds(n, r, w) for r in range(w)]
            assert parts[0][0] == 0 and parts[-1][1] == n
            assert all(parts[i][1] == parts[i + 1][0] for i in range(w - 1))
            sizes = [b - a for a, b in parts]
            assert max(sizes) - min(sizes) <= 1


def test_merge_topk_orders_by_distance_then_id():
    d = torch.tensor([[0.5, 0.1, 0.1, float("inf")]], dtype=torch.float64)
    i = torch.tensor([[4, 9, 2, -1]])
    md, mi = merge_topk(d, i, 3)
    assert mi.tolist() == [[2, 9, 4]] and md.tolist() == [[0.1, 0.1, 0.5]]


def _exchange_worker(rank, world, port, result_dir, use_gpu):
    """Tree-sharded kNN + nearestR and the per-batch state gather on `world` gloo ranks.  With
    use_gpu every rank answers its shard with the HIP path (NearestNeighborsGPU on cuda:0; the
    collectives run on CPU tensors over gloo); without it, with the oracle."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import sys

    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "oracle"))
    import pyoracle as O

    from ompl_amd import workloads as W
    from ompl_amd.shard import allgather_radius, allgather_states
    from ompl_amd.spaces import SE3StateSpace

    sp = SE3StateSpace()
    data, q = W.reference_states(sp, (6000, 40), seed=42)
    data[4001] = data[17]  # a tie across shards
    lo, hi = shard_bounds(len(data), rank, world)
    r = 0.45
    if use_gpu:
        from ompl_amd import NearestNeighborsGPU

        nn = NearestNeighborsGPU(sp, 0)
        nn.add(data[lo:hi])
        li, ld, _ = nn.nearestKBatch(q, 12)
        li = np.where(np.isinf(ld), -1, li.astype(np.int64))  # missing entries: (inf, NO_ID)
        off, ri, rd = nn.nearestRBatch(q, r)
    else:
        li, ld, _ = O.knn(sp, data[lo:hi], q, 12)
        li = np.where(li == 0xFFFFFFFF, -1, li.astype(np.int64))
        off, ri, rd = O.radius(sp, data[lo:hi], q, r)
    gid = torch.from_numpy(np.where(li >= 0, li + lo, -1))
    d, i = allgather_merge(torch.from_numpy(ld), gid, 12)
    if use_gpu:  # the device merge kernel on the gathered stack gives the same lists
        from ompl_amd.shard import merge_topk_device

        ws = [torch.empty_like(torch.from_numpy(ld)) for _ in range(world)]
        wi = [torch.empty_like(gid) for _ in range(world)]
        dist.all_gather(ws, torch.from_numpy(ld))
        dist.all_gather(wi, gid)
        dd, di = merge_topk_device(torch.stack(ws).cuda(), torch.stack(wi).to(torch.int32).cuda(), 12)
        torch.cuda.synchronize()
        assert torch.equal(dd.cpu(), d) and torch.equal(di.cpu().to(torch.int64), i)
    goff, gi, gd = allgather_radius(torch.from_numpy(off.astype(np.int64)),
                                    torch.from_numpy(ri.astype(np.int64) + lo), torch.from_numpy(rd))
    if use_gpu:  # the device CSR merge kernel on the gathered (padded) shard results gives the same CSR
        from ompl_amd.shard import _allgather_varlen, ids_int64, merge_csr_device

        offs, _ = _allgather_varlen(torch.from_numpy(off.astype(np.int64)))
        ii, cnt = _allgather_varlen(torch.from_numpy(ri.astype(np.int64) + lo))
        dd2, _ = _allgather_varlen(torch.from_numpy(rd))
        m = max(max(cnt), 1)
        pi = torch.stack([torch.cat([x, torch.zeros(m - len(x), dtype=x.dtype)]) for x in ii]).to(torch.int32)
        pd = torch.stack([torch.cat([x, torch.zeros(m - len(x), dtype=x.dtype)]) for x in dd2])
        oo, oi2, od2 = merge_csr_device(torch.stack(offs).cuda(), pi.cuda(), pd.cuda(), int(sum(cnt)))
        torch.cuda.synchronize()
        assert torch.equal(oo.cpu(), goff) and torch.equal(ids_int64(oi2).cpu(), gi) and torch.equal(od2.cpu(), gd)
    # a batch of new states: rank r contributes r + 3 of them; every rank gets all, rank order
    mine = torch.full((rank + 3, 7), float(rank), dtype=torch.float64)
    batch = allgather_states(mine)
    np.savez(os.path.join(result_dir, f"x{rank}.npz"), d=d.numpy(), i=i.numpy(), off=goff.numpy(), ri=gi.numpy(),
             rd=gd.numpy(), batch=batch.numpy())
    dist.barrier()
    dist.destroy_process_group()


def _check_exchange(tmp_path, world):
    import sys

    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "oracle"))
    import pyoracle as O

    from ompl_amd import workloads as W
    from ompl_amd.spaces import SE3StateSpace

    sp = SE3StateSpace()
    data, q = W.reference_states(sp, (6000, 40), seed=42)
    data[4001] = data[17]
    oi, od, _ = O.knn(sp, data, q, 12)
    ooff, oid, ord_ = O.radius(sp, data, q, 0.45)
    for r in range(world):
        z = np.load(tmp_path / f"x{r}.npz")
        np.testing.assert_array_equal(z["i"], oi.astype(np.int64))
        np.testing.assert_allclose(z["d"], od, rtol=0, atol=4e-16)
        np.testing.assert_array_equal(z["off"], ooff.astype(np.int64))
        np.testing.assert_array_equal(z["ri"], oid.astype(np.int64))
        np.testing.assert_allclose(z["rd"], ord_, rtol=0, atol=4e-16)
        b = z["batch"]
        assert b.shape == (sum(k + 3 for k in range(world)), 7)
        np.testing.assert_array_equal(b[:, 0], np.concatenate([np.full(k + 3, float(k)) for k in range(world)]))


@pytest.mark.parametrize("world", [2, 3])
def test_radius_and_state_exchange_gloo(tmp_path, world):
    port = _free_port()
    mp.start_processes(_exchange_worker, args=(world, port, str(tmp_path), False), nprocs=world, join=True,
                       start_method="spawn")
    _check_exchange(tmp_path, world)


@pytest.mark.gpu
def test_sharded_hip_path_world2(tmp_path, gpu):
    """The same decomposition with each rank's shard answered by the HIP kernels (two ranks
    sharing the box's one GPU, collectives over gloo)."""
    port = _free_port()
    mp.start_processes(_exchange_worker, args=(2, port, str(tmp_path), True), nprocs=2, join=True,
                       start_method="spawn")
    _check_exchange(tmp_path, 2)


def test_bench_spawn_plumbing():
    """`bench.py --gpus 2` without a launcher starts one child per rank with RANK / LOCAL_RANK /
    WORLD_SIZE set; with no GPU visible each rank fails loudly and so does the parent.  A
    WORLD_SIZE that disagrees with --gpus is refused before any GPU work."""
    import subprocess
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env["HIP_VISIBLE_DEVICES"] = "-1"  # no GPU even where one exists
    env["CUDA_VISIBLE_DEVICES"] = "-1"
    r = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--gpus", "2", "--steps", "1"], env=env,
                       capture_output=True, text=True, timeout=300)
    assert r.returncode != 0
    assert "rank 0 needs GPU 0" in r.stderr or "rank 1 needs GPU 1" in r.stderr, r.stderr[-2000:]
    env["WORLD_SIZE"] = "2"
    r = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--gpus", "4"], env=env,
                       capture_output=True, text=True, timeout=300)
    assert r.returncode != 0 and "--gpus 4 but WORLD_SIZE=2" in r.stderr


@pytest.mark.gpu
def test_merge_kernels_random_lists(gpu):
    """The merge-path kernels alone: W sorted shard lists with missing tails (top-k) and ragged
    CSR segments (radius), global ids above 2^31 included, against a torch reference."""
    from ompl_amd.shard import ids_int64, merge_csr_device, merge_topk, merge_topk_device

    g = torch.Generator().manual_seed(5)
    W, Q, k = 5, 300, 12
    d = torch.rand((W, Q, k), generator=g, dtype=torch.float64)
    d[:, :, 3] = d[:, :, 2]  # equal distances across lists: ids decide
    ids = torch.randperm(W * Q * k, generator=g).reshape(W, Q, k).to(torch.int64) + (1 << 31)
    valid = torch.rand((W, Q, k), generator=g) < 0.8
    d = torch.where(valid, d, torch.full_like(d, float("inf")))
    ids = torch.where(valid, ids, torch.full_like(ids, -1))
    key = torch.where(ids < 0, torch.full_like(ids, 1 << 40), ids)
    o = torch.argsort(key, dim=2, stable=True)
    d, ids = torch.gather(d, 2, o), torch.gather(ids, 2, o)
    o = torch.argsort(d, dim=2, stable=True)
    d, ids = torch.gather(d, 2, o), torch.gather(ids, 2, o)
    rd, ri = merge_topk(d.permute(1, 0, 2).reshape(Q, W * k), ids.permute(1, 0, 2).reshape(Q, W * k), k)
    md, mi = merge_topk_device(d.cuda(), ids.to(torch.int32).cuda(), k)
    torch.cuda.synchronize()
    assert torch.equal(md.cpu(), rd) and torch.equal(ids_int64(mi).cpu(), ri)
    # CSR: per shard, segment q = its valid entries of row q
    cnt = valid.sum(dim=2)                                   # [W, Q]
    offs = torch.zeros((W, Q + 1), dtype=torch.int64)
    offs[:, 1:] = torch.cumsum(cnt, dim=1)
    m = int(offs[:, -1].max())
    pi = torch.zeros((W, m), dtype=torch.int32)
    pd = torch.zeros((W, m), dtype=torch.float64)
    for w in range(W):
        sel = ids[w] >= 0
        pi[w, : int(offs[w, -1])] = ids[w][sel].to(torch.int32)
        pd[w, : int(offs[w, -1])] = d[w][sel]
    oo, oi, od = merge_csr_device(offs.cuda(), pi.cuda(), pd.cuda(), int(offs[:, -1].sum()))
    torch.cuda.synchronize()
    tot = torch.zeros(Q + 1, dtype=torch.int64)
    tot[1:] = torch.cumsum(cnt.sum(dim=0), 0)
    assert torch.equal(oo.cpu(), tot)
    for q in range(Q):
        seg = slice(int(tot[q]), int(tot[q + 1]))
        n = int(tot[q + 1] - tot[q])
        assert torch.equal(od.cpu()[seg], rd[q, :n]) if n <= k else True
        allv = torch.cat([d[w, q][ids[w, q] >= 0] for w in range(W)])
        alli = torch.cat([ids[w, q][ids[w, q] >= 0] for w in range(W)])
        o1 = torch.argsort(alli, stable=True)
        o2 = torch.argsort(allv[o1], stable=True)
        assert torch.equal(od.cpu()[seg], allv[o1][o2]) and torch.equal(ids_int64(oi).cpu()[seg], alli[o1][o2])
