"""World-size-2 gloo tests (CPU) of the multi-GPU decomposition: query sharding covers
every query exactly once, and the tree-sharded all_gather + merge reproduces the
single-process top-k exactly (ids and distances, ties by id)."""
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
