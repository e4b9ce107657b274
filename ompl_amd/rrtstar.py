"""ompl::geometric::RRTstar's iterations with their geometric work on the device.

RRTstar::solve (geometric/planners/rrt/src/RRTstar.cpp:247-542) with its defaults — k-nearest
neighbourhoods (useKNearest_, RRTstar.h:445), delayed collision checking (delayCC_, :458), rewire
factor 1.1 (:449), no new-state rejection, no tree pruning — under the path-length objective
(motionCost = distance, combineCosts = +, isCostBetterThan = <).  One call processes a batch of
samples in order:

  device (ompl_gpu_rrtstar_batch_device): nearest, steer, checkMotion, which states join the tree,
      every neighbourhood nearestK(x, ceil(k_rrt ln(size + 1))) and both motion bits of every
      (neighbour, x) pair — exact for the sequential loop (sample i sees the states of samples < i)
  host (this module): the cost logic that the reference interleaves with it, sample by sample —
      the parent in cost order (:319-357), the motion's cost, the rewiring (:414-457) and
      updateChildCosts (:633-643) — as lookups into the device's bits.

The tree is held as arrays over the nearest-neighbour ids: parent (-1 = a start state), incCost,
cost and the children lists.  The goal handling (:459-537) is planner logic outside the hot path.
"""
from __future__ import annotations

import ctypes as C
import math

import numpy as np

from . import abi
from .motion import DiscreteMotionValidatorGPU
from .nn import NearestNeighborsGPU


def k_rrt(dim: int, rewire_factor: float = 1.1) -> float:
    """calculateRewiringLowerBounds, k-nearest form (RRTstar.cpp:1147-1152)."""
    d = float(dim)
    return rewire_factor * (2.0 ** (d + 1) * math.e * (1.0 + 1.0 / d))


class RRTstarGPU:
    def __init__(self, space, checker, max_distance: float, device: int = 0, stream=None):
        self.space, self.dim = space, space.dim
        self.nn = NearestNeighborsGPU(space, device)
        self.mv = DiscreteMotionValidatorGPU(space, checker, device)
        if stream is not None:
            self.nn.set_stream(stream)
            self.mv.set_stream(stream)
        self.max_distance = float(max_distance)
        self.k_rrt = k_rrt(space.getDimension())
        self.device = device
        self.parent = np.zeros(0, np.int64)
        self.inc = np.zeros(0)
        self.cost = np.zeros(0)
        self.children: list = []
        self.n = 0
        self.stats = {"samples": 0, "added": 0, "rewires": 0, "checks_used": 0, "rounds": 0, "neighbours": 0}

    # ---- the tree ---------------------------------------------------------------------------
    def _grow(self, need: int) -> None:
        if need <= len(self.parent):
            return
        cap = max(need, 2 * len(self.parent), 1024)
        for name, fill in (("parent", -1), ("inc", 0.0), ("cost", 0.0)):
            a = getattr(self, name)
            b = np.full(cap, fill, dtype=a.dtype)
            b[: len(a)] = a
            setattr(self, name, b)

    def add_tree(self, states, parent=None, inc=None, cost=None) -> None:
        """Start states (parent -1, cost 0: the identity cost, RRTstar.cpp:208-213) or an existing
        tree given by its arrays (ids are the row indices, parents index earlier or equal rows)."""
        x = abi.as_states(states, self.dim)
        m = x.shape[0]
        first = self.n
        ids = self.nn.add(x)
        assert int(ids[0]) == first
        self._grow(first + m)
        self.parent[first:first + m] = -1 if parent is None else np.asarray(parent, np.int64)
        self.inc[first:first + m] = 0.0 if inc is None else np.asarray(inc, np.float64)
        self.cost[first:first + m] = 0.0 if cost is None else np.asarray(cost, np.float64)
        self.children.extend([] for _ in range(m))
        for v in range(first, first + m):
            p = int(self.parent[v])
            if p >= 0:
                self.children[p].append(v)
        self.n = first + m

    # ---- one batch ----------------------------------------------------------------------------
    def batch_device(self, d_samples: int, ns: int, d_nearest: int, d_added: int, d_inc: int, d_states: int = 0):
        """The device part of a batch (device pointers); returns the result record."""
        res = abi.RrtStarResult()
        abi.check(abi.lib.ompl_gpu_rrtstar_batch_device(self.nn._h, self.mv._h, C.c_void_p(d_samples), int(ns),
                                                        self.max_distance, self.k_rrt, C.c_void_p(d_nearest),
                                                        C.c_void_p(d_added), C.c_void_p(d_inc),
                                                        C.c_void_p(d_states or None), C.byref(res)))
        return res

    def solve_batch(self, samples):
        """Process the samples in order (host or torch device array).  Returns per sample
        (nearest id, added id or -1, chosen parent or -1)."""
        import torch

        dev = torch.device("cuda", self.device)
        s = torch.as_tensor(np.ascontiguousarray(samples, dtype=np.float64) if isinstance(samples, np.ndarray)
                            else samples).to(dev).contiguous()
        ns = s.shape[0]
        near = torch.empty(ns, dtype=torch.int32, device=dev)
        added = torch.empty(ns, dtype=torch.int32, device=dev)
        inc = torch.empty(ns, dtype=torch.float64, device=dev)
        res = self.batch_device(s.data_ptr(), ns, near.data_ptr(), added.data_ptr(), inc.data_ptr())
        return self.commit(near, added, inc, res)

    @staticmethod
    def _host(ptr: int, n: int, dtype):
        """copy n elements of a library-owned device array to the host (a torch view of the
        pointer through __cuda_array_interface__, then a device-to-host copy)"""
        import torch

        if n == 0 or not ptr:
            return np.zeros(n, dtype=torch.empty(0, dtype=dtype).numpy().dtype)
        typestr = {torch.int64: "<i8", torch.int32: "<i4", torch.float64: "<f8", torch.uint8: "|u1"}[dtype]

        class _View:
            __cuda_array_interface__ = {"shape": (n,), "typestr": typestr, "data": (int(ptr), False), "version": 3}

        return torch.as_tensor(_View(), device="cuda").cpu().numpy()

    def commit(self, near, added, inc, res):
        """The cost logic of RRTstar.cpp:287-457 for the batch's added states, in sample order."""
        import torch

        near = near.cpu().numpy().view(np.uint32).astype(np.int64)
        added = added.cpu().numpy().view(np.uint32).astype(np.int64)
        inc = inc.cpu().numpy()
        ns = len(near)
        E = int(res.total)
        off = self._host(res.offsets, ns + 1, torch.int64).astype(np.int64)
        ids = self._host(res.ids, E, torch.int32).view(np.uint32).astype(np.int64)
        dist = self._host(res.dist, E, torch.float64)
        bits = self._host(res.bits, E, torch.uint8)
        self.stats["rounds"] = max(self.stats["rounds"], int(res.rounds))
        self.stats["neighbours"] += E
        self.stats["samples"] += ns
        maxd = self.max_distance
        chosen = np.full(ns, -1, np.int64)
        added_out = np.where(added == abi.NO_ID32, -1, added)
        new = np.flatnonzero(added_out >= 0)
        if len(new):
            self._grow(int(added_out[new].max()) + 1)
        cost, parent, incs, children = self.cost, self.parent, self.inc, self.children
        for i in new:
            x = int(added_out[i])
            nm = int(near[i])
            a, b = int(off[i]), int(off[i + 1])
            nb, d, bt = ids[a:b], dist[a:b], bits[a:b]
            # the motion as created (RRTstar.cpp:285-289)
            m_inc = float(inc[i])
            m_cost = cost[nm] + m_inc
            m_parent = nm
            # delayCC: neighbours in cost order, the first with a valid connection (:319-357)
            costs = cost[nb] + d
            order = np.argsort(costs, kind="stable")
            ok = (nb == nm) | ((d < maxd) & ((bt & 1) != 0))
            valid = np.zeros(len(nb), np.int8)
            hit = np.flatnonzero(ok[order])
            if len(hit):
                f = int(hit[0])
                r = int(order[f])
                valid[order[:f]] = -1
                valid[r] = 1
                m_inc, m_cost, m_parent = float(d[r]), float(costs[r]), int(nb[r])
                self.stats["checks_used"] += f + (0 if nb[r] == nm else 1)
            else:
                valid[:] = -1
                self.stats["checks_used"] += int(np.count_nonzero((nb != nm) & (d < maxd)))
            # the motion joins the tree (:410-411)
            parent[x], incs[x], cost[x] = m_parent, m_inc, m_cost
            while len(children) <= x:
                children.append([])
            children[m_parent].append(x)
            self.n = max(self.n, x + 1)
            chosen[i] = m_parent
            # rewiring (:414-457), in neighbour order; a rewire changes the costs of a subtree
            # (updateChildCosts), which later candidates of this loop must see
            start = 0
            while True:
                newc = cost[x] + d[start:]
                cand = (newc < cost[nb[start:]]) & (nb[start:] != m_parent)
                if not cand.any():
                    break
                for rr in np.flatnonzero(cand):
                    r = start + int(rr)
                    v = int(nb[r])
                    nc = cost[x] + d[r]
                    if not (nc < cost[v]):  # costs moved since the mask (an earlier rewire's subtree)
                        continue
                    if valid[r] == 0:
                        mv_ok = bool(d[r] < maxd) and bool(bt[r] & 2)
                        self.stats["checks_used"] += 1 if d[r] < maxd else 0
                    else:
                        mv_ok = valid[r] == 1
                    if not mv_ok:
                        continue
                    children[int(parent[v])].remove(v)  # removeFromParent (:620-631)
                    parent[v], incs[v], cost[v] = x, d[r], nc
                    children[x].append(v)
                    self._update_child_costs(v)
                    self.stats["rewires"] += 1
                    start = r + 1
                    break
                else:
                    break
        self.stats["added"] += len(new)
        return near, added_out, chosen

    def _update_child_costs(self, m: int) -> None:  # RRTstar.cpp:633-643
        cost, inc, children = self.cost, self.inc, self.children
        stack = [m]
        while stack:
            u = stack.pop()
            cu = cost[u]
            for c in children[u]:
                cost[c] = cu + inc[c]
                if children[c]:
                    stack.append(c)

    def close(self) -> None:
        self.nn.close()
        self.mv.close()
