"""ctypes binding of the C ABI in include/ompl_gpu.h (libompl_gpu.so).

The library is the product path: there is no CPU fallback.  If the shared
object is missing this module raises at import time; if no HIP device is present
every handle constructor raises :class:`GpuError` (``OMPL_GPU_ERR_DEVICE``).
"""
from __future__ import annotations

import atexit
import ctypes as C
import itertools
import os
import weakref

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("OMPL_GPU_LIB", os.path.join(HERE, "lib", "libompl_gpu.so"))

# ---- enums (include/ompl_gpu.h) ------------------------------------------------
OK, ERR_INVALID_ARG, ERR_EMPTY, ERR_DEVICE, ERR_OOM, ERR_UNSUPPORTED, ERR_NOT_FOUND = range(7)
SPACE_REALVECTOR, SPACE_SO3, SPACE_SE3, SPACE_KCHAIN = range(4)
CHECK_ALL_VALID, CHECK_HYPERCUBE, CHECK_SPHERES, CHECK_KCHAIN, CHECK_CIRCLES2D = range(5)
NO_ID32 = 0xFFFFFFFF
NO_ID64 = 0xFFFFFFFFFFFFFFFF


class SpaceStruct(C.Structure):
    _fields_ = [
        ("kind", C.c_int32),
        ("dim", C.c_int32),
        ("weight", C.c_double * 2),
        ("lvs", C.c_double * 2),
        ("factor", C.c_uint32 * 2),
        ("link_length", C.c_double),
    ]


class CheckerStruct(C.Structure):
    _fields_ = [
        ("kind", C.c_int32),
        ("ndim", C.c_int32),
        ("edge_width", C.c_double),
        ("count", C.c_int32),
        ("reserved", C.c_int32),
        ("data", C.POINTER(C.c_double)),
    ]


class RrtStarResult(C.Structure):
    """ompl_gpu_rrtstar_result: library-owned device arrays of one RRT* batch"""
    _fields_ = [
        ("offsets", C.c_void_p),
        ("ids", C.c_void_p),
        ("dist", C.c_void_p),
        ("bits", C.c_void_p),
        ("total", C.c_uint64),
        ("added", C.c_uint64),
        ("rounds", C.c_uint32),
        ("reserved", C.c_uint32),
    ]


class GpuError(RuntimeError):
    def __init__(self, status: int, msg: str):
        super().__init__(f"[ompl_gpu status {status}] {msg}")
        self.status = status


class EmptyError(GpuError):
    """Raised where the reference throws ompl::Exception("No elements found in
    nearest neighbors data structure") (NearestNeighborsGNAT.h:218)."""


_P = C.c_void_p
_D = C.POINTER(C.c_double)
_U8 = C.POINTER(C.c_uint8)
_U32 = C.POINTER(C.c_uint32)
_I32 = C.POINTER(C.c_int32)
_U64 = C.POINTER(C.c_uint64)

# name -> (restype, argtypes); every symbol include/ompl_gpu.h declares
SIGNATURES = {
    "ompl_gpu_abi_version": (C.c_int, []),
    "ompl_gpu_last_error": (C.c_char_p, []),
    "ompl_gpu_device_count": (C.c_int, [C.POINTER(C.c_int)]),
    "ompl_gpu_free": (None, [_P]),
    "ompl_gpu_nn_create": (C.c_int, [C.POINTER(_P), C.POINTER(SpaceStruct), C.c_int]),
    "ompl_gpu_nn_destroy": (C.c_int, [_P]),
    "ompl_gpu_nn_set_stream": (C.c_int, [_P, _P]),
    "ompl_gpu_nn_sync": (C.c_int, [_P]),
    "ompl_gpu_nn_add": (C.c_int, [_P, _D, C.c_size_t, _U64]),
    "ompl_gpu_nn_remove": (C.c_int, [_P, C.c_uint64]),
    "ompl_gpu_nn_clear": (C.c_int, [_P]),
    "ompl_gpu_nn_size": (C.c_int, [_P, C.POINTER(C.c_size_t), C.POINTER(C.c_size_t)]),
    "ompl_gpu_nn_get_states": (C.c_int, [_P, C.c_uint64, C.c_size_t, _D]),
    "ompl_gpu_nn_knn": (C.c_int, [_P, _D, C.c_size_t, C.c_uint32, _U64, _D, _U32]),
    "ompl_gpu_nn_nearest": (C.c_int, [_P, _D, C.c_size_t, _U64, _D]),
    "ompl_gpu_nn_radius": (C.c_int, [_P, _D, C.c_size_t, C.c_double, C.POINTER(_U64), C.POINTER(_D), _U64]),
    "ompl_gpu_nn_knn_device": (C.c_int, [_P, _P, C.c_size_t, C.c_uint32, _P, _P]),
    "ompl_gpu_nn_set_exact": (C.c_int, [_P, C.c_int]),
    "ompl_gpu_nn_stats": (C.c_int, [_P, _U64, _U64]),
    "ompl_gpu_nn_rerun_stats": (C.c_int, [_P, _U64]),
    "ompl_gpu_nn_large_stats": (C.c_int, [_P, _U64, _U64]),
    "ompl_gpu_nn_index_stats": (C.c_int, [_P, _U64, _U64]),
    "ompl_gpu_nn_build_index": (C.c_int, [_P]),
    "ompl_gpu_nn_profile": (C.c_int, [_P, C.c_int]),
    "ompl_gpu_nn_cull_stats": (C.c_int, [_P, _U64, _U64, _U64]),
    "ompl_gpu_nn_kernel_time": (C.c_int, [_P, _D, _U64, C.POINTER(C.c_char_p)]),
    "ompl_gpu_steer_device": (C.c_int, [_P, _P, C.c_size_t, _P, C.c_uint32, C.c_double, _P, _P]),
    "ompl_gpu_nn_radius_device": (C.c_int, [_P, _P, C.c_size_t, C.c_double, _P, _P, _P, C.c_uint64, _U64]),
    "ompl_gpu_nn_radius_cull_stats": (C.c_int, [_P, _U64, _U64]),
    "ompl_gpu_nn_radius_path_stats": (C.c_int, [_P, _U64, _U64]),
    "ompl_gpu_nn_edges_device": (C.c_int, [_P, _P, C.c_size_t, _P, _P, C.c_uint32, C.c_size_t, C.c_int, _P, _P]),
    "ompl_gpu_rrt_grow_device": (C.c_int, [_P, _P, _P, C.c_size_t, C.c_double, _P, _P]),
    "ompl_gpu_rrt_aborts": (C.c_int, [_P, _U64]),
    "ompl_gpu_rrtstar_batch_device": (C.c_int, [_P, _P, _P, C.c_size_t, C.c_double, C.c_double, _P, _P, _P, _P,
                                                C.POINTER(RrtStarResult)]),
    "ompl_gpu_rrtstar_tree_create": (C.c_int, [C.POINTER(_P)]),
    "ompl_gpu_rrtstar_tree_destroy": (None, [_P]),
    "ompl_gpu_rrtstar_tree_add": (C.c_int, [_P, C.c_size_t, _P, _P, _P]),
    "ompl_gpu_rrtstar_tree_size": (C.c_int, [_P, C.POINTER(C.c_size_t)]),
    "ompl_gpu_rrtstar_tree_read": (C.c_int, [_P, C.c_size_t, C.c_size_t, _P, _P, _P]),
    "ompl_gpu_rrtstar_tree_totals": (C.c_int, [_P, _U64]),
    "ompl_gpu_rrtstar_stage": (C.c_int, [_P, _P, C.c_size_t, _P, _P, _P, C.POINTER(RrtStarResult)]),
    "ompl_gpu_rrtstar_stage_host": (C.c_int, [_P, C.c_size_t, _P, _P, _P, _P, _P, _P, _P]),
    "ompl_gpu_rrtstar_commit": (C.c_int, [_P, C.c_double, C.c_size_t, _P, _P, _P, C.POINTER(C.c_size_t)]),
    "ompl_gpu_csr_merge_device": (C.c_int, [_P, C.c_uint32, C.c_size_t, _P, _P, C.c_size_t, _P, _P, _P, _P]),
    "ompl_gpu_knn_merge_device": (C.c_int, [_P, _P, C.c_uint32, C.c_size_t, C.c_uint32, _P, _P, _P]),
    "ompl_gpu_rrt_solve_device": (C.c_int, [_P, _P, _P, C.c_size_t, C.c_double, _D, C.c_double, _P, _P, _U64,
                                            _U32, _D]),
    "ompl_gpu_prm_add_milestones": (C.c_int, [_P, _P, _D, C.c_size_t, C.c_size_t, C.c_size_t, C.c_double, C.c_uint32,
                                              _P, _P, _P, _U64]),
    "ompl_gpu_lazyprm_add_milestones": (C.c_int, [_P, _D, C.c_size_t, C.c_size_t, C.c_size_t, C.c_double, C.c_uint32,
                                                  _P, _P, _P]),
    "ompl_gpu_bitstar_update_samples": (C.c_int, [_P, _P, _P, C.c_uint64, C.c_uint64, C.c_uint64, _U64, _U64, _U64]),
    "ompl_gpu_mv_create": (C.c_int, [C.POINTER(_P), C.POINTER(SpaceStruct), C.POINTER(CheckerStruct), C.c_int]),
    "ompl_gpu_mv_destroy": (C.c_int, [_P]),
    "ompl_gpu_mv_set_stream": (C.c_int, [_P, _P]),
    "ompl_gpu_mv_sync": (C.c_int, [_P]),
    "ompl_gpu_mv_check": (C.c_int, [_P, _D, _D, C.c_size_t, _U8, _I32, _I32]),
    "ompl_gpu_mv_check_device": (C.c_int, [_P, _P, _P, C.c_size_t, _P, _P, _P]),
    "ompl_gpu_mv_check_edges_device": (C.c_int, [_P, _P, _P, C.c_size_t, _P, _P, C.c_uint32, C.c_size_t, C.c_int, _P]),
    "ompl_gpu_mv_counters": (C.c_int, [_P, _U64, _U64]),
    "ompl_gpu_mv_reset_counters": (C.c_int, [_P]),
    "ompl_gpu_mv_state_checks": (C.c_int, [_P, _U64]),
    "ompl_gpu_svc_check": (C.c_int, [_P, _D, C.c_size_t, _U8]),
    "ompl_gpu_svc_check_host": (C.c_int, [_P, _D, C.c_size_t, _U8]),
    "ompl_gpu_svc_check_device": (C.c_int, [_P, _P, C.c_size_t, _P]),
    "ompl_gpu_nn_distance_host": (C.c_int, [_P, _D, _D, C.c_size_t, _D]),
    "ompl_gpu_rng_set_seed": (None, [C.c_uint32]),
    "ompl_gpu_rng_get_seed": (C.c_uint32, []),
    "ompl_gpu_rng_seeds_drawn": (C.c_uint64, []),
    "ompl_gpu_rng_next_seed": (C.c_uint32, []),
    "ompl_gpu_rng_uniform_real": (C.c_int, [C.c_uint32, C.c_size_t, C.c_double, C.c_double, _D]),
    "ompl_gpu_sampler_create": (C.c_int, [C.POINTER(_P), C.POINTER(SpaceStruct), _D, _D]),
    "ompl_gpu_sampler_destroy": (C.c_int, [_P]),
    "ompl_gpu_sampler_sample_uniform": (C.c_int, [_P, C.c_size_t, _D]),
    "ompl_gpu_sampler_local_seeds": (C.c_int, [_P, _U32, C.POINTER(C.c_int)]),
    "ompl_gpu_mv_motion_states": (C.c_int, [_P, _D, _D, C.c_size_t, C.c_uint32, C.c_int, _D]),
    "ompl_gpu_mv_motion_states_device": (C.c_int, [_P, _P, _P, C.c_size_t, C.c_uint32, C.c_int, _P]),
    "ompl_gpu_mv_space_pairs": (C.c_int, [_P, _D, _D, _D, C.c_size_t, _D]),
    "ompl_gpu_mv_space_pairs_device": (C.c_int, [_P, _P, _P, _P, C.c_size_t, _P]),
}


def _share_torch_runtime():
    """PyTorch-ROCm ships its own HIP runtime (torch/lib/libamdhip64.so, SONAME
    libamdhip64.so.7).  Loading torch first makes the dynamic linker bind this library's
    libamdhip64.so.7 dependency to that same runtime, so device pointers and streams
    from torch (plumbing for the device-resident API and RCCL) are valid here.  Without
    torch the system ROCm runtime is used."""
    if os.environ.get("OMPL_GPU_NO_TORCH") == "1":
        return
    try:
        import torch  # noqa: F401
    except ImportError:
        pass


def _load():
    _share_torch_runtime()
    if not os.path.exists(LIB_PATH):
        raise ImportError(
            f"ompl_amd: {LIB_PATH} is missing — build it with `python -c 'import __graft_entry__ as g; g.build()'` "
            "(there is no CPU fallback for the GPU backend)")
    lib = C.CDLL(LIB_PATH)
    for name, (res, args) in SIGNATURES.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    return lib


lib = _load()


def check(status: int) -> None:
    if status != OK:
        msg = (lib.ompl_gpu_last_error() or b"").decode(errors="replace")
        if status == ERR_EMPTY:
            raise EmptyError(status, msg)
        raise GpuError(status, msg)


def device_count() -> int:
    n = C.c_int(0)
    st = lib.ompl_gpu_device_count(C.byref(n))
    return n.value if st == OK else 0


def dptr(a: np.ndarray):
    return a.ctypes.data_as(_D)


def as_states(x, dim: int) -> np.ndarray:
    a = np.ascontiguousarray(np.asarray(x, dtype=np.float64))
    if a.ndim == 1:
        a = a.reshape(1, -1)
    if a.shape[-1] != dim:
        raise ValueError(f"expected states with {dim} reals, got shape {a.shape}")
    return a


# ---- handle lifetime -------------------------------------------------------------
# Every C handle is released by close() (idempotent), by __del__, or — for the ones still
# alive when the interpreter exits — by the atexit hook below, newest first, while the HIP
# runtime (and a profiler attached to it) is still up.  After that hook no destroy call
# runs: a handle left to the C library's static teardown would call into a HIP runtime
# that may already be gone (round-2 exit-time SIGSEGV under rocprofv3).
_live: dict = {}
_serial = itertools.count()
_closed_all = False


class Handle:
    """Owner of one C handle (`_h`) released with the C function named `_destroy_fn`."""

    _destroy_fn = ""
    _h = None

    def _own(self, h) -> None:
        self._h = h
        self._serial = next(_serial)
        _live[self._serial] = weakref.ref(self)

    def close(self) -> None:
        h = self._h
        self._h = None
        if h is not None and h.value and not _closed_all:
            self._destroy(h)
        _live.pop(getattr(self, "_serial", None), None)

    def _destroy(self, h) -> None:
        getattr(lib, self._destroy_fn)(h)

    def __del__(self):
        try:
            self.close()
        except Exception:  # interpreter teardown: modules may already be cleared
            pass

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()
        return False


def close_all() -> None:
    """Destroy every live handle, newest first (samplers / validators before the NN
    structures they were created after).  Registered with atexit."""
    global _closed_all
    for key in sorted(_live, reverse=True):
        ref = _live.get(key)
        obj = ref() if ref is not None else None
        if obj is not None:
            obj.close()
    _live.clear()
    _closed_all = True


atexit.register(close_all)
