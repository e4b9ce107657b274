"""Multi-GPU decomposition of the NN / motion path (one process per GPU).

Default (BASELINE.json configs[2..4]): the state set is REPLICATED and query / edge
batches are SHARDED by rank — queries are independent, so there is no collective in
the data path (weak scaling).

Tree-sharded mode (for state sets beyond one GPU's HBM): each rank holds a contiguous
slice of the ids, answers every query on its slice, and the per-rank top-k candidate
lists are exchanged with one all_gather over RCCL (xGMI) and merged on every rank.
RCCL's built-in reductions cannot merge top-k lists, so the exchange is an all_gather
of Q*k*(8+8) bytes per rank followed by a local (distance, id) merge.
"""
from __future__ import annotations

import torch


def shard_bounds(n: int, rank: int, world: int) -> tuple[int, int]:
    """Contiguous [lo, hi) slice of n items for `rank` (sizes differ by at most one)."""
    base, rem = divmod(n, world)
    lo = rank * base + min(rank, rem)
    return lo, lo + base + (1 if rank < rem else 0)


def merge_topk(d: torch.Tensor, ids: torch.Tensor, k: int):
    """d, ids: [Q, M] candidates (missing = +inf / -1).  Returns the k smallest by
    (distance, id) — the same order the kernels produce."""
    big = torch.iinfo(torch.int64).max
    key_id = torch.where(ids < 0, torch.full_like(ids, big), ids)
    o1 = torch.argsort(key_id, dim=1, stable=True)
    d1 = torch.gather(d, 1, o1)
    i1 = torch.gather(ids, 1, o1)
    o2 = torch.argsort(d1, dim=1, stable=True)[:, :k]
    return torch.gather(d1, 1, o2), torch.gather(i1, 1, o2)


def allgather_merge(d_local: torch.Tensor, ids_global: torch.Tensor, k: int, group=None):
    """Exchange per-rank [Q, k] candidate lists (global ids) and merge to the global top-k."""
    import torch.distributed as dist

    world = dist.get_world_size(group)
    ds = [torch.empty_like(d_local) for _ in range(world)]
    ii = [torch.empty_like(ids_global) for _ in range(world)]
    dist.all_gather(ds, d_local.contiguous(), group=group)
    dist.all_gather(ii, ids_global.contiguous(), group=group)
    return merge_topk(torch.cat(ds, dim=1), torch.cat(ii, dim=1), k)
