"""Multi-GPU decomposition of the NN / motion path (one process per GPU).

Default (BASELINE.json configs[2..4]): the state set is REPLICATED and query / edge
batches are SHARDED by rank — queries are independent, so there is no collective in
the data path (weak scaling).

Tree-sharded mode (for state sets beyond one GPU's HBM): each rank holds a contiguous
slice of the ids, answers every query on its slice, and the per-rank top-k candidate
lists are exchanged with one all_gather over RCCL (xGMI) and merged on every rank.
RCCL's built-in reductions cannot merge top-k lists, so the exchange is an all_gather
of Q*k*(8+8) bytes per rank followed by a local (distance, id) merge.  Radius results are
variable-size: a count all_gather, then padded payload all_gathers (allgather_radius).

Growing sets (BIT* batches, PRM* causal prefixes): each rank contributes its part of a batch
of new states and allgather_states gives every replica the whole batch in rank order.
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


def merge_topk_device(d_stack: torch.Tensor, ids_stack: torch.Tensor, k: int, stream=None):
    """The per-shard lists as an all_gather leaves them — d_stack [W, Q, k] fp64, ids_stack
    [W, Q, k] int32 (global ids, missing = -1, i.e. 0xFFFFFFFF) on the GPU — merged by the
    library's HIP kernel (ompl_gpu_knn_merge_device) into the global [Q, k] top k by
    (distance, id).  Returns (distances fp64, ids int32)."""
    import ctypes as C

    from . import abi

    W, Q, kk = d_stack.shape
    d_stack = d_stack.contiguous()
    ids_stack = ids_stack.to(torch.int32).contiguous()
    od = torch.empty((Q, k), dtype=torch.float64, device=d_stack.device)
    oi = torch.empty((Q, k), dtype=torch.int32, device=d_stack.device)
    if kk != k:
        raise ValueError("every shard list must hold k entries")
    st = stream if stream is not None else torch.cuda.current_stream(d_stack.device).cuda_stream
    abi.check(abi.lib.ompl_gpu_knn_merge_device(C.c_void_p(d_stack.data_ptr()), C.c_void_p(ids_stack.data_ptr()),
                                                int(W), int(Q), int(k), C.c_void_p(od.data_ptr()),
                                                C.c_void_p(oi.data_ptr()), C.c_void_p(st)))
    return od, oi


def ids_int64(ids32: torch.Tensor) -> torch.Tensor:
    """uint32 ids held in an int32 tensor -> int64 with the missing marker 0xFFFFFFFF as -1 (ids
    at or above 2^31 stay positive: the library stores up to 2^32 - 16 states)."""
    u = ids32.to(torch.int64) & 0xFFFFFFFF
    return torch.where(u == 0xFFFFFFFF, torch.full_like(u, -1), u)


def merge_csr_device(offs: torch.Tensor, ids: torch.Tensor, dists: torch.Tensor, total: int, stream=None):
    """W shards' CSR results of the same queries on the GPU — offs [W, Q+1] int64, ids [W, S]
    int32 (global ids), dists [W, S] fp64, as the padded all_gathers leave them — merged by the
    library's HIP kernel (ompl_gpu_csr_merge_device).  Returns (offsets int64 [Q+1], ids int32,
    distances fp64) with `total` = the sum of the shards' counts."""
    import ctypes as C

    from . import abi

    W, Q1 = offs.shape
    dev = offs.device
    offs, ids, dists = offs.to(torch.int64).contiguous(), ids.to(torch.int32).contiguous(), dists.contiguous()
    oo = torch.empty(Q1, dtype=torch.int64, device=dev)
    oi = torch.empty(max(total, 1), dtype=torch.int32, device=dev)
    od = torch.empty(max(total, 1), dtype=torch.float64, device=dev)
    st = stream if stream is not None else torch.cuda.current_stream(dev).cuda_stream
    abi.check(abi.lib.ompl_gpu_csr_merge_device(C.c_void_p(offs.data_ptr()), int(W), int(Q1 - 1),
                                                C.c_void_p(ids.data_ptr()), C.c_void_p(dists.data_ptr()),
                                                int(ids.shape[1]), C.c_void_p(oo.data_ptr()), C.c_void_p(oi.data_ptr()),
                                                C.c_void_p(od.data_ptr()), C.c_void_p(st)))
    return oo, oi[:total], od[:total]


def allgather_merge(d_local: torch.Tensor, ids_global: torch.Tensor, k: int, group=None):
    """Exchange per-rank [Q, k] candidate lists (global ids, missing = -1) and merge to the global
    top-k.  GPU tensors (RCCL): one all_gather per array into a [W, Q, k] stack, merged by the HIP
    kernel (merge_topk_device); CPU tensors (gloo tests): the same merge with torch sorts."""
    import torch.distributed as dist

    world = dist.get_world_size(group)
    if d_local.is_cuda:
        ds = torch.empty((world,) + tuple(d_local.shape), dtype=d_local.dtype, device=d_local.device)
        ii = torch.empty((world,) + tuple(ids_global.shape), dtype=torch.int32, device=d_local.device)
        dist.all_gather_into_tensor(ds, d_local.contiguous(), group=group)
        dist.all_gather_into_tensor(ii, ids_global.to(torch.int32).contiguous(), group=group)
        od, oi = merge_topk_device(ds, ii, k)
        return od, ids_int64(oi)
    ds = [torch.empty_like(d_local) for _ in range(world)]
    ii = [torch.empty_like(ids_global) for _ in range(world)]
    dist.all_gather(ds, d_local.contiguous(), group=group)
    dist.all_gather(ii, ids_global.contiguous(), group=group)
    return merge_topk(torch.cat(ds, dim=1), torch.cat(ii, dim=1), k)


def _allgather_varlen(x: torch.Tensor, group=None):
    """All-gather a tensor whose leading dimension differs per rank: one all_gather of the
    counts, then one of the payload padded to the largest count (RCCL's all_gather needs equal
    shapes).  Returns (list of per-rank tensors, counts)."""
    import torch.distributed as dist

    world = dist.get_world_size(group)
    n = torch.tensor([x.shape[0]], dtype=torch.int64, device=x.device)
    ns = [torch.empty_like(n) for _ in range(world)]
    dist.all_gather(ns, n, group=group)
    counts = [int(c.item()) for c in ns]
    m = max(counts) if counts else 0
    pad = torch.zeros((m,) + tuple(x.shape[1:]), dtype=x.dtype, device=x.device)
    pad[: x.shape[0]] = x
    parts = [torch.empty_like(pad) for _ in range(world)]
    dist.all_gather(parts, pad, group=group)
    return [p[:c] for p, c in zip(parts, counts)], counts


def allgather_states(local: torch.Tensor, group=None) -> torch.Tensor:
    """New states of one batch, contributed by every rank (each samples / validity-filters its
    part: BIT*'s batch of samples, ImplicitGraph.cpp:924-1000; PRM*'s milestones of a causal
    prefix, PRM.cpp:562-596), gathered in rank order on every rank, so that every replica of the
    tree appends the same states in the same order and ids agree across ranks."""
    parts, _ = _allgather_varlen(local.contiguous(), group)
    return torch.cat(parts, dim=0)


def merge_csr(offsets: list, ids: list, dists: list):
    """Per-rank radius results for the same queries (CSR: offsets [Q+1], global ids, distances)
    -> one CSR whose segments hold the union sorted by (distance, id), the order
    NearestNeighborsGNAT::nearestR / Linear report (NearestNeighborsGNAT.h:236-245)."""
    nq = offsets[0].numel() - 1
    seg_d, seg_i, seg_q = [], [], []
    for off, ii, dd in zip(offsets, ids, dists):
        cnt = off[1:] - off[:-1]
        tot = int(off[-1])  # capacity-sized buffers (radius_device) hold more than the CSR
        ii, dd = ii[:tot], dd[:tot]
        seg_q.append(torch.repeat_interleave(torch.arange(nq, dtype=torch.int64, device=off.device), cnt))
        seg_i.append(ii.to(torch.int64))
        seg_d.append(dd)
    q, i, d = torch.cat(seg_q), torch.cat(seg_i), torch.cat(seg_d)
    o = torch.argsort(i, stable=True)           # id, then distance, then query: lexicographic
    o = o[torch.argsort(d[o], stable=True)]
    o = o[torch.argsort(q[o], stable=True)]
    counts = torch.bincount(q, minlength=nq)
    out_off = torch.zeros(nq + 1, dtype=torch.int64, device=q.device)
    out_off[1:] = torch.cumsum(counts, 0)
    return out_off, i[o], d[o]


def allgather_radius(offsets: torch.Tensor, ids_global: torch.Tensor, dists: torch.Tensor, group=None):
    """Tree-sharded nearestR (SURVEY §8e "Radius search"): every rank answers the same queries
    on its slice of the states; the variable-size CSR results are exchanged as a count
    all_gather followed by padded payload all_gathers, and merged on every rank."""
    tot = int(offsets[-1])
    ids_global, dists = ids_global[:tot], dists[:tot]
    if offsets.is_cuda:  # RCCL: padded payload all_gathers, merged by the library's kernel
        import torch.distributed as dist

        world = dist.get_world_size(group)
        offs = torch.empty((world, offsets.numel()), dtype=torch.int64, device=offsets.device)
        dist.all_gather_into_tensor(offs, offsets.to(torch.int64).contiguous(), group=group)
        counts = offs[:, -1].tolist()
        m = max(max(counts), 1)
        pi = torch.zeros(m, dtype=torch.int32, device=offsets.device)
        pd = torch.zeros(m, dtype=torch.float64, device=offsets.device)
        pi[:tot] = ids_global.to(torch.int32)
        pd[:tot] = dists
        ii = torch.empty((world, m), dtype=torch.int32, device=offsets.device)
        dd = torch.empty((world, m), dtype=torch.float64, device=offsets.device)
        dist.all_gather_into_tensor(ii, pi, group=group)
        dist.all_gather_into_tensor(dd, pd, group=group)
        oo, oi, od = merge_csr_device(offs, ii, dd, int(sum(counts)))
        return oo, ids_int64(oi), od
    offs, _ = _allgather_varlen(offsets.to(torch.int64).contiguous(), group)
    ii, _ = _allgather_varlen(ids_global.to(torch.int64).contiguous(), group)
    dd, _ = _allgather_varlen(dists.contiguous(), group)
    return merge_csr(offs, ii, dd)
