"""Python mirror of ompl::base::DiscreteMotionValidator / StateValidityChecker
(MotionValidator.h:56-145, DiscreteMotionValidator.cpp:48-145) over the MI355X
C ABI, for the closed set of device checkers in :mod:`ompl_amd.checkers`.
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from . import abi
from .checkers import Checker
from .spaces import StateSpace


class DiscreteMotionValidatorGPU(abi.Handle):
    _destroy_fn = "ompl_gpu_mv_destroy"

    def __init__(self, space: StateSpace, checker: Checker, device: int = 0):
        self.space = space
        self.checker = checker
        self.dim = space.dim
        self._space_struct = space.to_abi()
        self._checker_struct = checker.to_abi()
        h = C.c_void_p()
        abi.check(abi.lib.ompl_gpu_mv_create(C.byref(h), C.byref(self._space_struct),
                                             C.byref(self._checker_struct), int(device)))
        self._own(h)

    def checkMotions(self, s1, s2, want_nd: bool = False, want_first_invalid: bool = False):
        a = abi.as_states(s1, self.dim)
        b = abi.as_states(s2, self.dim)
        if a.shape != b.shape:
            raise ValueError("s1 and s2 must have the same shape")
        m = a.shape[0]
        valid = np.zeros(m, dtype=np.uint8)
        nd = np.zeros(m, dtype=np.int32) if want_nd else None
        fi = np.zeros(m, dtype=np.int32) if want_first_invalid else None
        abi.check(abi.lib.ompl_gpu_mv_check(
            self._h, abi.dptr(a), abi.dptr(b), m, valid.ctypes.data_as(abi._U8),
            nd.ctypes.data_as(abi._I32) if nd is not None else None,
            fi.ctypes.data_as(abi._I32) if fi is not None else None))
        out = [valid.astype(bool)]
        if want_nd:
            out.append(nd)
        if want_first_invalid:
            out.append(fi)
        return out[0] if len(out) == 1 else tuple(out)

    def checkMotion(self, s1, s2, lastValid: bool = False):
        """checkMotion(s1,s2) -> bool; with lastValid=True returns (bool, t) where t is
        lastValid.second = (j-1)/nd of the first invalid sample (DiscreteMotionValidator.cpp:63-77)."""
        if not lastValid:
            return bool(self.checkMotions(s1, s2)[0])
        v, nd, fi = self.checkMotions(s1, s2, want_nd=True, want_first_invalid=True)
        if v[0]:
            return True, None
        j, n = int(fi[0]), int(nd[0])
        return False, (j - 1) / n if n else float("-inf")

    def getValidMotionCount(self) -> int:
        v, i = C.c_uint64(0), C.c_uint64(0)
        abi.check(abi.lib.ompl_gpu_mv_counters(self._h, C.byref(v), C.byref(i)))
        return v.value

    def getInvalidMotionCount(self) -> int:
        v, i = C.c_uint64(0), C.c_uint64(0)
        abi.check(abi.lib.ompl_gpu_mv_counters(self._h, C.byref(v), C.byref(i)))
        return i.value

    def stateChecks(self) -> int:
        c = C.c_uint64(0)
        abi.check(abi.lib.ompl_gpu_mv_state_checks(self._h, C.byref(c)))
        return c.value

    def resetMotionCounter(self) -> None:
        abi.check(abi.lib.ompl_gpu_mv_reset_counters(self._h))

    def isValid(self, states) -> np.ndarray:
        s = abi.as_states(states, self.dim)
        out = np.zeros(s.shape[0], dtype=np.uint8)
        abi.check(abi.lib.ompl_gpu_svc_check(self._h, abi.dptr(s), s.shape[0], out.ctypes.data_as(abi._U8)))
        return out.astype(bool)

    def getMotionStates(self, s1, s2, count: int, endpoints: bool = True) -> np.ndarray:
        """SpaceInformation::getMotionStates (SpaceInformation.cpp:201-275, alloc = true) for a
        batch of motions: [m, count + (2 if endpoints else 0), dim]."""
        a = abi.as_states(s1, self.dim)
        b = abi.as_states(s2, self.dim)
        if a.shape != b.shape:
            raise ValueError("s1 and s2 must have the same shape")
        if count < 0:
            raise ValueError("count must be >= 0")
        per = count + (2 if endpoints else 0)
        out = np.zeros((a.shape[0], per, self.dim))
        abi.check(abi.lib.ompl_gpu_mv_motion_states(self._h, abi.dptr(a), abi.dptr(b), a.shape[0], int(count),
                                                    int(bool(endpoints)), abi.dptr(out)))
        return out

    def distance(self, a, b) -> np.ndarray:
        """StateSpace::distance(a[i], b[i]) per pair, evaluated on the device (RealVectorStateSpace.cpp:230-242,
        SO3StateSpace.cpp:254-262, StateSpace.cpp:1068-1076, KinematicChain.h:105-124)."""
        x, y = abi.as_states(a, self.dim), abi.as_states(b, self.dim)
        if x.shape != y.shape:
            raise ValueError("a and b must have the same shape")
        out = np.zeros(x.shape[0])
        abi.check(abi.lib.ompl_gpu_mv_space_pairs(self._h, abi.dptr(x), abi.dptr(y), None, x.shape[0],
                                                  abi.dptr(out)))
        return out

    def interpolate(self, a, b, t) -> np.ndarray:
        """StateSpace::interpolate(a[i], b[i], t[i]) per pair, evaluated on the device
        (RealVectorStateSpace.cpp:257-265, SO3StateSpace.cpp:289-318, StateSpace.cpp:1109-1116,
        KinematicChain.h:150-175); t is a scalar or one fraction per pair."""
        x, y = abi.as_states(a, self.dim), abi.as_states(b, self.dim)
        if x.shape != y.shape:
            raise ValueError("a and b must have the same shape")
        tt = np.ascontiguousarray(np.broadcast_to(np.asarray(t, dtype=np.float64), (x.shape[0],)))
        out = np.zeros_like(x)
        abi.check(abi.lib.ompl_gpu_mv_space_pairs(self._h, abi.dptr(x), abi.dptr(y), abi.dptr(tt), x.shape[0],
                                                  abi.dptr(out)))
        return out

    # device-resident
    def set_stream(self, stream_ptr: int | None) -> None:
        abi.check(abi.lib.ompl_gpu_mv_set_stream(self._h, C.c_void_p(stream_ptr or 0)))

    def sync(self) -> None:
        abi.check(abi.lib.ompl_gpu_mv_sync(self._h))

    def check_edges_device(self, nn, d_queries: int, nq: int, d_offsets, d_ids: int, stride: int, m: int,
                           from_query: bool, d_valid: int) -> None:
        """checkMotion over the edges of a neighbour result read in place (ompl_gpu_mv_check_edges_device):
        the pairs NearestNeighborsGPU.edges_device would write, without writing them."""
        abi.check(abi.lib.ompl_gpu_mv_check_edges_device(self._h, nn._h, C.c_void_p(d_queries), nq,
                                                         C.c_void_p(d_offsets or None), C.c_void_p(d_ids), stride, m,
                                                         1 if from_query else 0, C.c_void_p(d_valid)))

    def check_device(self, d_s1: int, d_s2: int, m: int, d_valid: int, d_nd: int = 0, d_fi: int = 0) -> None:
        abi.check(abi.lib.ompl_gpu_mv_check_device(self._h, C.c_void_p(d_s1), C.c_void_p(d_s2), m,
                                                   C.c_void_p(d_valid), C.c_void_p(d_nd or None),
                                                   C.c_void_p(d_fi or None)))
