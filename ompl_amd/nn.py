"""Python mirror of the reference's ompl::NearestNeighbors<_T> for integer element
ids (the form PRM and Blaze use: NearestNeighbors<Vertex>, PRM.h:125), backed by
the MI355X C ABI.  Method names and semantics follow NearestNeighbors.h:46-115:

  add / remove / clear / size / list / nearest / nearestK / nearestR /
  reportsSortedResults  — plus batched forms (nearestKBatch, nearestRBatch) and
  device-resident forms used by the benchmark.

Element ids are insertion indices.  Results are sorted by (distance, id).
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from . import abi
from .spaces import StateSpace


class NearestNeighborsGPU(abi.Handle):
    _destroy_fn = "ompl_gpu_nn_destroy"

    def __init__(self, space: StateSpace, device: int = 0):
        self.space = space
        self.dim = space.dim
        self._space_struct = space.to_abi()
        h = C.c_void_p()
        abi.check(abi.lib.ompl_gpu_nn_create(C.byref(h), C.byref(self._space_struct), int(device)))
        self._own(h)
        self._removed: set[int] = set()
        self.device = device


    # ---- container ---------------------------------------------------------
    def reportsSortedResults(self) -> bool:
        return True

    def add(self, states) -> np.ndarray:
        s = abi.as_states(states, self.dim)
        first = C.c_uint64(0)
        abi.check(abi.lib.ompl_gpu_nn_add(self._h, abi.dptr(s), s.shape[0], C.byref(first)))
        return np.arange(first.value, first.value + s.shape[0], dtype=np.uint64)

    def remove(self, elem_id: int) -> bool:
        st = abi.lib.ompl_gpu_nn_remove(self._h, int(elem_id))
        if st == abi.ERR_NOT_FOUND:
            return False
        abi.check(st)
        self._removed.add(int(elem_id))
        return True

    def clear(self) -> None:
        abi.check(abi.lib.ompl_gpu_nn_clear(self._h))
        self._removed.clear()

    def size(self) -> int:
        live, tot = C.c_size_t(0), C.c_size_t(0)
        abi.check(abi.lib.ompl_gpu_nn_size(self._h, C.byref(live), C.byref(tot)))
        return live.value

    def total(self) -> int:
        live, tot = C.c_size_t(0), C.c_size_t(0)
        abi.check(abi.lib.ompl_gpu_nn_size(self._h, C.byref(live), C.byref(tot)))
        return tot.value

    def states(self, first: int = 0, n: int | None = None) -> np.ndarray:
        n = self.total() - first if n is None else n
        out = np.empty((n, self.dim), dtype=np.float64)
        abi.check(abi.lib.ompl_gpu_nn_get_states(self._h, int(first), int(n), abi.dptr(out)))
        return out

    # ---- queries -----------------------------------------------------------
    def nearest(self, q) -> int:
        qs = abi.as_states(q, self.dim)
        ids = np.empty(qs.shape[0], dtype=np.uint64)
        d = np.empty(qs.shape[0], dtype=np.float64)
        abi.check(abi.lib.ompl_gpu_nn_nearest(self._h, abi.dptr(qs), qs.shape[0],
                                              ids.ctypes.data_as(abi._U64), abi.dptr(d)))
        return int(ids[0])

    def nearestKBatch(self, queries, k: int):
        """ids [nq, k] (uint64, NO_ID64 padding), dists [nq, k], counts [nq]."""
        qs = abi.as_states(queries, self.dim)
        nq = qs.shape[0]
        ids = np.full((nq, max(k, 1)), abi.NO_ID64, dtype=np.uint64)
        d = np.full((nq, max(k, 1)), np.inf, dtype=np.float64)
        cnt = np.zeros(nq, dtype=np.uint32)
        abi.check(abi.lib.ompl_gpu_nn_knn(self._h, abi.dptr(qs), nq, int(k), ids.ctypes.data_as(abi._U64),
                                          abi.dptr(d), cnt.ctypes.data_as(abi._U32)))
        return ids[:, :k], d[:, :k], cnt

    def nearestK(self, q, k: int) -> list:
        ids, _, cnt = self.nearestKBatch(q, k)
        return [int(x) for x in ids[0, :cnt[0]]]

    def nearestRBatch(self, queries, radius: float):
        """CSR: (offsets [nq+1], ids, dists) sorted by (distance, id) per query."""
        qs = abi.as_states(queries, self.dim)
        nq = qs.shape[0]
        pid = abi._U64()
        pd = abi._D()
        off = np.zeros(nq + 1, dtype=np.uint64)
        abi.check(abi.lib.ompl_gpu_nn_radius(self._h, abi.dptr(qs), nq, float(radius), C.byref(pid), C.byref(pd),
                                             off.ctypes.data_as(abi._U64)))
        tot = int(off[-1])
        try:
            ids = np.ctypeslib.as_array(pid, shape=(max(tot, 1),))[:tot].copy()
            d = np.ctypeslib.as_array(pd, shape=(max(tot, 1),))[:tot].copy()
        finally:
            abi.lib.ompl_gpu_free(C.cast(pid, C.c_void_p))
            abi.lib.ompl_gpu_free(C.cast(pd, C.c_void_p))
        return off, ids, d

    def nearestR(self, q, radius: float) -> list:
        off, ids, _ = self.nearestRBatch(q, radius)
        return [int(x) for x in ids[int(off[0]):int(off[1])]]

    def list(self) -> list:
        """Live element ids (insertion order; the reference's order is unspecified)."""
        return [i for i in range(self.total()) if i not in self._removed]

    def set_exact(self, exact_only: bool) -> None:
        """Force the exact fp64 scan (default: fp32 screen + fp64 certificate)."""
        self.set_mode(1 if exact_only else 0)

    def set_mode(self, mode: int) -> None:
        """0: fp32 screen (culled for R^n / SE3) + fp64 certificate; 1: exact fp64 scan;
        2: fp32 screen without culling.  All modes return identical results."""
        abi.check(abi.lib.ompl_gpu_nn_set_exact(self._h, int(mode)))

    def stats(self) -> tuple[int, int]:
        """(queries that took the fp32 screen, queries re-run exactly after a failed certificate)."""
        a, b = C.c_uint64(0), C.c_uint64(0)
        abi.check(abi.lib.ompl_gpu_nn_stats(self._h, C.byref(a), C.byref(b)))
        return a.value, b.value

    def rerun_stats(self) -> int:
        """Re-run queries whose bounded exact pass overflowed its candidate cap and took the
        full exact scan (a subset of stats()[1])."""
        a = C.c_uint64(0)
        abi.check(abi.lib.ompl_gpu_nn_rerun_stats(self._h, C.byref(a)))
        return a.value

    def large_stats(self) -> tuple[int, int]:
        """Large-k select: (queries whose candidates spilled to the per-query pool, queries re-run
        on the exact fallback), summed over calls."""
        a, b = C.c_uint64(), C.c_uint64()
        abi.check(abi.lib.ompl_gpu_nn_large_stats(self._h, C.byref(a), C.byref(b)))
        return a.value, b.value

    def build_index(self) -> None:
        """Bring the culled walks' sorted copy up to date now (asynchronous on the handle's stream)."""
        abi.check(abi.lib.ompl_gpu_nn_build_index(self._h))

    def index_stats(self) -> tuple[int, int]:
        """(device k-d builds of the sorted copy, tail appends that avoided a rebuild)."""
        a, b = C.c_uint64(0), C.c_uint64(0)
        abi.check(abi.lib.ompl_gpu_nn_index_stats(self._h, C.byref(a), C.byref(b)))
        return a.value, b.value

    def cull_stats(self) -> tuple[int, int, int]:
        """(64-state tiles the culled screen fetched, tiles a full scan would have fetched,
        (tile, query) pairs scanned — 64 distance evaluations each)."""
        a, b, c = C.c_uint64(0), C.c_uint64(0), C.c_uint64(0)
        abi.check(abi.lib.ompl_gpu_nn_cull_stats(self._h, C.byref(a), C.byref(b), C.byref(c)))
        return a.value, b.value, c.value

    def profile(self, enable: bool = True) -> None:
        abi.check(abi.lib.ompl_gpu_nn_profile(self._h, 1 if enable else 0))

    def kernel_time(self) -> tuple[float, int, str]:
        """(summed ms, launches, name) of the dominant scan kernel, from HIP events recorded
        on the launch stream while profiling was enabled."""
        ms, n, name = C.c_double(0), C.c_uint64(0), C.c_char_p()
        abi.check(abi.lib.ompl_gpu_nn_kernel_time(self._h, C.byref(ms), C.byref(n), C.byref(name)))
        return ms.value, n.value, (name.value or b"").decode()

    # ---- device-resident (benchmark / pipelines); pointers are device addresses
    def set_stream(self, stream_ptr: int | None) -> None:
        abi.check(abi.lib.ompl_gpu_nn_set_stream(self._h, C.c_void_p(stream_ptr or 0)))

    def sync(self) -> None:
        abi.check(abi.lib.ompl_gpu_nn_sync(self._h))

    def knn_device(self, d_queries: int, nq: int, k: int, d_ids: int, d_dist: int) -> None:
        abi.check(abi.lib.ompl_gpu_nn_knn_device(self._h, C.c_void_p(d_queries), nq, k, C.c_void_p(d_ids),
                                                 C.c_void_p(d_dist)))

    def radius_device(self, d_queries: int, nq: int, radius: float, d_offsets: int, d_ids: int, d_dist: int,
                      capacity: int) -> int:
        """nearestR into caller device buffers: offsets [nq+1] (int64), ids (int32) and dists
        (fp64) of `capacity` entries, sorted by (distance, id) per query.  Returns the number of
        results; when it exceeds capacity only the offsets are written."""
        tot = C.c_uint64(0)
        st = abi.lib.ompl_gpu_nn_radius_device(self._h, C.c_void_p(d_queries), nq, float(radius),
                                               C.c_void_p(d_offsets), C.c_void_p(d_ids or None),
                                               C.c_void_p(d_dist or None), int(capacity), C.byref(tot))
        if st != abi.OK and not (st == abi.ERR_INVALID_ARG and tot.value > capacity):
            abi.check(st)
        return tot.value

    def radius_cull_stats(self) -> tuple[int, int]:
        """(64-state tiles the radius walk fetched, (tile, query) pairs it scanned)."""
        a, b = C.c_uint64(0), C.c_uint64(0)
        abi.check(abi.lib.ompl_gpu_nn_radius_cull_stats(self._h, C.byref(a), C.byref(b)))
        return a.value, b.value

    def radius_path_stats(self) -> tuple[int, int]:
        """(culled nearestR calls answered by the one slab walk, calls that overflowed a slab)."""
        a, b = C.c_uint64(0), C.c_uint64(0)
        abi.check(abi.lib.ompl_gpu_nn_radius_path_stats(self._h, C.byref(a), C.byref(b)))
        return a.value, b.value

    def edges_device(self, d_queries: int, nq: int, d_offsets: int | None, d_ids: int, stride: int, m: int,
                     from_query: bool, d_from: int, d_to: int) -> None:
        """Motion endpoints of neighbour results (PRM.cpp:582 from_query=False, BITstar.cpp:815
        from_query=True): CSR offsets from radius_device, or None with a dense nq x stride id matrix."""
        abi.check(abi.lib.ompl_gpu_nn_edges_device(self._h, C.c_void_p(d_queries), nq, C.c_void_p(d_offsets or None),
                                                   C.c_void_p(d_ids), int(stride), int(m), 1 if from_query else 0,
                                                   C.c_void_p(d_from), C.c_void_p(d_to)))

    def rrt_grow_device(self, mv, d_samples: int, ns: int, max_distance: float, d_nearest: int, d_added: int) -> None:
        """ns RRT iterations on device (RRT.cpp:128-192 without the goal test) with motion
        validator `mv` (a DiscreteMotionValidatorGPU over the same space)."""
        abi.check(abi.lib.ompl_gpu_rrt_grow_device(self._h, mv._h, C.c_void_p(d_samples), int(ns), float(max_distance),
                                                   C.c_void_p(d_nearest), C.c_void_p(d_added)))

    def rrt_aborts(self) -> int:
        """Persistent RRT runs that gave up (spin limit) and were re-run in the two-launch form."""
        a = C.c_uint64(0)
        abi.check(abi.lib.ompl_gpu_rrt_aborts(self._h, C.byref(a)))
        return a.value

    def rrt_solve_device(self, mv, d_samples: int, ns: int, max_distance: float, goal, goal_threshold: float,
                         d_nearest: int, d_added: int):
        """RRT iterations with the goal test (RRT.cpp:128-192): stops at the first added state
        within goal_threshold of `goal`.  Returns (solved iteration or None, approximate-solution id
        or None, its distance)."""
        g = abi.as_states(goal, self.dim).reshape(-1)
        sol = C.c_uint64(0)
        aid = C.c_uint32(0)
        ad = C.c_double(0.0)
        abi.check(abi.lib.ompl_gpu_rrt_solve_device(self._h, mv._h, C.c_void_p(d_samples), int(ns),
                                                    float(max_distance), abi.dptr(g), float(goal_threshold),
                                                    C.c_void_p(d_nearest), C.c_void_p(d_added), C.byref(sol),
                                                    C.byref(aid), C.byref(ad)))
        return (None if sol.value == 2 ** 64 - 1 else sol.value, None if aid.value == abi.NO_ID32 else aid.value,
                ad.value)

    def prm_add_milestones(self, mv, states, k_const: float, k_cap: int, j0: int = 0, j1: int | None = None):
        """PRM* causal batch (PRM.cpp:562-596, KStarStrategy): the milestones, in order, connect to
        their k_i nearest among every earlier vertex, edges checked with mv, then join the structure.
        Returns host arrays (neighbours [m, k_cap] uint32 with 0xFFFFFFFF padding, counts [m],
        edge validity [m, k_cap] bool) and the number of edges checked."""
        import torch

        x = abi.as_states(states, self.dim)
        m = x.shape[0]
        j1 = m if j1 is None else j1
        r = j1 - j0
        dev = torch.device("cuda", self.device)
        nbr = torch.empty((max(r, 1), k_cap), dtype=torch.int32, device=dev)
        cnt = torch.empty(max(r, 1), dtype=torch.int32, device=dev)
        val = torch.empty((max(r, 1), k_cap), dtype=torch.uint8, device=dev)
        e = C.c_uint64(0)
        abi.check(abi.lib.ompl_gpu_prm_add_milestones(self._h, mv._h, abi.dptr(x), m, int(j0), int(j1), float(k_const),
                                                      int(k_cap), C.c_void_p(nbr.data_ptr()),
                                                      C.c_void_p(cnt.data_ptr()), C.c_void_p(val.data_ptr()),
                                                      C.byref(e)))
        torch.cuda.synchronize(dev)
        return (nbr[:r].cpu().numpy().view(np.uint32), cnt[:r].cpu().numpy().view(np.uint32),
                val[:r].cpu().numpy().astype(bool), e.value)

    def lazyprm_add_milestones(self, states, k_const: float, k_cap: int, j0: int = 0, j1: int | None = None):
        """LazyPRM::addMilestone for a batch (LazyPRM.cpp:285-309): the PRM* neighbours, no edge
        checked; returns (neighbours [r, k_cap], counts [r], edge weights = distances [r, k_cap])."""
        import torch

        x = abi.as_states(states, self.dim)
        m = x.shape[0]
        j1 = m if j1 is None else j1
        r = j1 - j0
        dev = torch.device("cuda", self.device)
        nbr = torch.empty((max(r, 1), k_cap), dtype=torch.int32, device=dev)
        cnt = torch.empty(max(r, 1), dtype=torch.int32, device=dev)
        dist = torch.empty((max(r, 1), k_cap), dtype=torch.float64, device=dev)
        abi.check(abi.lib.ompl_gpu_lazyprm_add_milestones(self._h, abi.dptr(x), m, int(j0), int(j1), float(k_const),
                                                          int(k_cap), C.c_void_p(nbr.data_ptr()),
                                                          C.c_void_p(cnt.data_ptr()), C.c_void_p(dist.data_ptr())))
        torch.cuda.synchronize(dev)
        return (nbr[:r].cpu().numpy().view(np.uint32), cnt[:r].cpu().numpy().view(np.uint32),
                dist[:r].cpu().numpy())

    def prm_add_milestones_device(self, mv, states, k_const: float, k_cap: int, d_nbr: int, d_cnt: int,
                                  d_valid: int, j0: int = 0, j1: int | None = None) -> int:
        """The same into caller-owned device buffers ((j1 - j0) rows); returns the number of edges checked."""
        x = abi.as_states(states, self.dim)
        j1 = x.shape[0] if j1 is None else j1
        e = C.c_uint64(0)
        abi.check(abi.lib.ompl_gpu_prm_add_milestones(self._h, mv._h, abi.dptr(x), x.shape[0], int(j0), int(j1),
                                                      float(k_const), int(k_cap), C.c_void_p(d_nbr),
                                                      C.c_void_p(d_cnt), C.c_void_p(d_valid), C.byref(e)))
        return e.value

    def steer_device(self, d_queries: int, nq: int, d_nearest: int, stride: int, max_distance: float,
                     d_from: int, d_to: int) -> None:
        abi.check(abi.lib.ompl_gpu_steer_device(self._h, C.c_void_p(d_queries), nq, C.c_void_p(d_nearest),
                                                int(stride), float(max_distance), C.c_void_p(d_from),
                                                C.c_void_p(d_to)))
