"""ompl::geometric::RRTstar's iterations with their geometric work on the device.

RRTstar::solve (geometric/planners/rrt/src/RRTstar.cpp:247-542) with its defaults — k-nearest
neighbourhoods (useKNearest_, RRTstar.h:445), delayed collision checking (delayCC_, :458), rewire
factor 1.1 (:449), no new-state rejection, no tree pruning — under the path-length objective
(motionCost = distance, combineCosts = +, isCostBetterThan = <).  One call processes a batch of
samples in order:

  device (ompl_gpu_rrtstar_batch_device): nearest, steer, checkMotion, which states join the tree,
      every neighbourhood nearestK(x, ceil(k_rrt ln(size + 1))) and both motion bits of every
      (neighbour, x) pair — exact for the sequential loop (sample i sees the states of samples < i)
  host (ompl_gpu_rrtstar_stage / _commit, native C++): the cost logic that the reference
      interleaves with it, sample by sample — the parent in cost order (:319-357), the motion's
      cost, the rewiring (:414-457) and updateChildCosts (:633-643) — as lookups into the bits.

The tree's costs live in the library's tree object as arrays over the nearest-neighbour ids:
parent (-1 = a start state), incCost, cost and the children lists.  solve_batches overlaps the
cost logic of batch i (a host thread; ctypes releases the GIL) with the device work of batch i + 1,
which needs only the states, never the costs.  The goal handling (:459-537) is planner logic
outside the hot path.
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


class _Tree(abi.Handle):
    _destroy_fn = "ompl_gpu_rrtstar_tree_destroy"

    def __init__(self):
        h = C.c_void_p()
        abi.check(abi.lib.ompl_gpu_rrtstar_tree_create(C.byref(h)))
        self._own(h)


def _ptr(a: np.ndarray):
    return C.c_void_p(a.ctypes.data) if a is not None else None


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
        self.tree = _Tree()
        self.rounds = 0

    # ---- the tree ---------------------------------------------------------------------------
    @property
    def n(self) -> int:
        n = C.c_size_t()
        abi.check(abi.lib.ompl_gpu_rrtstar_tree_size(self.tree._h, C.byref(n)))
        return int(n.value)

    def _read(self):
        n = self.n
        parent, inc, cost = np.empty(n, np.int64), np.empty(n), np.empty(n)
        abi.check(abi.lib.ompl_gpu_rrtstar_tree_read(self.tree._h, 0, n, _ptr(parent), _ptr(inc), _ptr(cost)))
        return parent, inc, cost

    @property
    def parent(self) -> np.ndarray:
        return self._read()[0]

    @property
    def inc(self) -> np.ndarray:
        return self._read()[1]

    @property
    def cost(self) -> np.ndarray:
        return self._read()[2]

    @property
    def stats(self) -> dict:
        t = (C.c_uint64 * 6)()
        abi.check(abi.lib.ompl_gpu_rrtstar_tree_totals(self.tree._h, t))
        return {"rewires": int(t[0]), "checks_used": int(t[1]), "added": int(t[2]), "neighbours": int(t[3]),
                "samples": int(t[4]), "child_cost_updates": int(t[5]), "rounds": self.rounds}

    def add_tree(self, states, parent=None, inc=None, cost=None) -> None:
        """Start states (parent -1, cost 0: the identity cost, RRTstar.cpp:208-213) or an existing
        tree given by its arrays (ids are the row indices, parents index earlier rows)."""
        x = abi.as_states(states, self.dim)
        m = x.shape[0]
        first = self.n
        ids = self.nn.add(x)
        assert int(ids[0]) == first
        arr = lambda a, dt: None if a is None else np.ascontiguousarray(a, dtype=dt)  # noqa: E731
        p, i, c = arr(parent, np.int64), arr(inc, np.float64), arr(cost, np.float64)
        abi.check(abi.lib.ompl_gpu_rrtstar_tree_add(self.tree._h, m, _ptr(p), _ptr(i), _ptr(c)))

    # ---- one batch ----------------------------------------------------------------------------
    def batch_device(self, d_samples: int, ns: int, d_nearest: int, d_added: int, d_inc: int, d_states: int = 0):
        """The device part of a batch (device pointers); returns the result record."""
        res = abi.RrtStarResult()
        abi.check(abi.lib.ompl_gpu_rrtstar_batch_device(self.nn._h, self.mv._h, C.c_void_p(d_samples), int(ns),
                                                        self.max_distance, self.k_rrt, C.c_void_p(d_nearest),
                                                        C.c_void_p(d_added), C.c_void_p(d_inc),
                                                        C.c_void_p(d_states or None), C.byref(res)))
        self.rounds = max(self.rounds, int(res.rounds))
        return res

    def stage(self, ns: int, d_nearest: int, d_added: int, d_inc: int, res) -> None:
        """Copy the batch's results to the host and queue them for commit."""
        abi.check(abi.lib.ompl_gpu_rrtstar_stage(self.tree._h, self.nn._h, int(ns), C.c_void_p(d_nearest),
                                                 C.c_void_p(d_added), C.c_void_p(d_inc), C.byref(res)))

    def commit(self, ns: int):
        """The cost logic (RRTstar.cpp:285-457) of the oldest staged batch.  Returns per sample
        (nearest id, added id or -1, chosen parent or -1)."""
        near, added, chosen = (np.empty(ns, np.int64) for _ in range(3))
        got = C.c_size_t()
        abi.check(abi.lib.ompl_gpu_rrtstar_commit(self.tree._h, self.max_distance, ns, _ptr(near), _ptr(added),
                                                  _ptr(chosen), C.byref(got)))
        assert got.value == ns
        return near, added, chosen

    def _device_batch(self, samples):
        import torch

        dev = torch.device("cuda", self.device)
        s = torch.as_tensor(np.ascontiguousarray(samples, dtype=np.float64) if isinstance(samples, np.ndarray)
                            else samples).to(dev).contiguous()
        ns = s.shape[0]
        near = torch.empty(ns, dtype=torch.int32, device=dev)
        added = torch.empty(ns, dtype=torch.int32, device=dev)
        inc = torch.empty(ns, dtype=torch.float64, device=dev)
        res = self.batch_device(s.data_ptr(), ns, near.data_ptr(), added.data_ptr(), inc.data_ptr())
        self.stage(ns, near.data_ptr(), added.data_ptr(), inc.data_ptr(), res)
        return ns

    def solve_batch(self, samples):
        """Process the samples in order (host or torch device array).  Returns per sample
        (nearest id, added id or -1, chosen parent or -1)."""
        return self.commit(self._device_batch(samples))

    def solve_batches(self, batches):
        """solve_batch over a sequence of batches, the cost logic of each overlapping the device
        work of the next.  Returns the per-batch results."""
        from concurrent.futures import ThreadPoolExecutor

        out, pending = [], None
        with ThreadPoolExecutor(1) as ex:
            for b in batches:
                ns = self._device_batch(b)
                if pending is not None:
                    out.append(pending.result())
                pending = ex.submit(self.commit, ns)
            if pending is not None:
                out.append(pending.result())
        return out

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

    def close(self) -> None:
        self.tree.close()
        self.nn.close()
        self.mv.close()
