"""TEST INFRASTRUCTURE ONLY — ctypes access to the CPU oracle.

  liboracle.so            restatement of the reference hot path (oracle.cpp, gnat.cpp)
  _ref/libref_linear.so   the reference's own NearestNeighborsLinear.h compiled from
                          /root/reference (present only where it was built)

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import
this module, and only as the checker / the CPU baseline.
"""
from __future__ import annotations

import ctypes as C
import os

import numpy as np

from ompl_amd import abi

HERE = os.path.dirname(os.path.abspath(__file__))
ORACLE_PATH = os.path.join(HERE, "liboracle.so")
REF_PATH = os.path.join(HERE, "_ref", "libref_linear.so")

_SP = C.POINTER(abi.SpaceStruct)
_CK = C.POINTER(abi.CheckerStruct)
_D, _U8, _U32, _I32, _U64 = abi._D, abi._U8, abi._U32, abi._I32, abi._U64
_I64 = C.POINTER(C.c_int64)

_ORACLE_SIGS = {
    "oracle_distance": (C.c_double, [_SP, _D, _D]),
    "oracle_interpolate": (None, [_SP, _D, _D, C.c_double, _D]),
    "oracle_valid_segment_count": (C.c_uint32, [_SP, _D, _D]),
    "oracle_motion_states": (C.c_uint32, [_SP, _D, _D, C.c_size_t, C.c_uint32, C.c_int, _D]),
    "oracle_is_valid": (C.c_int, [_SP, _CK, _D]),
    "oracle_check_motions": (C.c_uint64, [_SP, _CK, _D, _D, C.c_size_t, _U8, _I32, _I32]),
    "oracle_check_motions_mt": (C.c_uint64, [_SP, _CK, _D, _D, C.c_size_t, _U8, C.c_int]),
    "oracle_knn": (None, [_SP, _D, C.c_size_t, _D, C.c_size_t, C.c_uint32, _U32, _D, _U32]),
    "oracle_radius": (None, [_SP, _D, C.c_size_t, _D, C.c_size_t, C.c_double, _U64, _U32, _D, _U64]),
    "oracle_gnat_create": (C.c_void_p, [_SP, C.c_uint32, C.c_uint32, C.c_uint32, C.c_uint32, C.c_uint64]),
    "oracle_gnat_destroy": (None, [C.c_void_p]),
    "oracle_gnat_add": (None, [C.c_void_p, _D, C.c_size_t]),
    "oracle_gnat_add_bulk": (None, [C.c_void_p, _D, C.c_size_t]),
    "oracle_gnat_size": (C.c_size_t, [C.c_void_p]),
    "oracle_gnat_knn": (None, [C.c_void_p, _D, C.c_size_t, C.c_uint32, _U32, _D, _U32, C.c_int]),
    "oracle_gnat_radius_count": (C.c_uint64, [C.c_void_p, _D, C.c_size_t, C.c_double, _U64, C.c_int]),
    "oracle_gnat_radius": (C.c_uint64, [C.c_void_p, _D, C.c_size_t, C.c_double, _U64, C.c_int]),
    "oracle_gnat_radius_fetch": (None, [C.c_void_p, _U32, _D]),
    "oracle_prm_causal": (None, [_SP, _CK, _D, C.c_size_t, C.c_double, C.c_uint32, _U32, _U32, _U8]),
    "oracle_rrtstar": (C.c_uint64, [_SP, _CK, _D, C.c_size_t, _I64, _D, _D, _D, C.c_size_t, C.c_double, C.c_double,
                                    C.c_int, C.c_double, _U32, _U32, _I64, _I64, _D, _D, _U64]),
    "oracle_mt19937_10000th": (C.c_uint32, []),
    "oracle_ranlux24_base_10000th": (C.c_uint32, []),
    "oracle_seed_stream": (None, [C.c_uint32, C.c_size_t, _U32]),
    "oracle_sample_uniform": (None, [_SP, _U32, _D, _D, C.c_size_t, _D]),
}
_REF_SIGS = {
    "ref_linear_knn": (C.c_int, [_SP, _D, C.c_size_t, _D, C.c_size_t, C.c_uint32, _U32, _D, _U32]),
    "ref_linear_nearest": (C.c_int, [_SP, _D, C.c_size_t, _D, C.c_size_t, _U32, C.c_char_p]),
    "ref_linear_radius": (C.c_int, [_SP, _D, C.c_size_t, _D, C.c_size_t, C.c_double, _U64, _U32, _U64]),
}


def _load(path, sigs):
    lib = C.CDLL(path)
    for n, (r, a) in sigs.items():
        f = getattr(lib, n)
        f.restype, f.argtypes = r, a
    return lib


lib = _load(ORACLE_PATH, _ORACLE_SIGS)
ref = _load(REF_PATH, _REF_SIGS) if os.path.exists(REF_PATH) else None


def _arr(a):
    return np.ascontiguousarray(np.asarray(a, dtype=np.float64))


def distance(sp, a, b) -> float:
    s = sp.to_abi()
    a, b = _arr(a), _arr(b)
    return lib.oracle_distance(C.byref(s), abi.dptr(a), abi.dptr(b))


def interpolate(sp, a, b, t) -> np.ndarray:
    s = sp.to_abi()
    a, b = _arr(a), _arr(b)
    o = np.empty(sp.dim)
    lib.oracle_interpolate(C.byref(s), abi.dptr(a), abi.dptr(b), float(t), abi.dptr(o))
    return o


def motion_states(sp, s1, s2, count, endpoints=True) -> np.ndarray:
    """getMotionStates for each motion: [m, count + (2 if endpoints else 0), dim]."""
    s = sp.to_abi()
    a, b = abi.as_states(s1, sp.dim), abi.as_states(s2, sp.dim)
    per = count + (2 if endpoints else 0)
    o = np.zeros((a.shape[0], per, sp.dim))
    got = lib.oracle_motion_states(C.byref(s), abi.dptr(a), abi.dptr(b), a.shape[0], count, int(endpoints),
                                   abi.dptr(o))
    assert got == per
    return o


def valid_segment_count(sp, a, b) -> int:
    s = sp.to_abi()
    a, b = _arr(a), _arr(b)
    return int(lib.oracle_valid_segment_count(C.byref(s), abi.dptr(a), abi.dptr(b)))


def is_valid(sp, ck, states) -> np.ndarray:
    s, c = sp.to_abi(), ck.to_abi()
    x = _arr(states).reshape(-1, sp.dim)
    return np.array([bool(lib.oracle_is_valid(C.byref(s), C.byref(c), abi.dptr(r))) for r in x])


def check_motions(sp, ck, s1, s2):
    s, c = sp.to_abi(), ck.to_abi()
    a, b = _arr(s1).reshape(-1, sp.dim), _arr(s2).reshape(-1, sp.dim)
    m = a.shape[0]
    valid = np.zeros(m, np.uint8)
    nd = np.zeros(m, np.int32)
    fi = np.zeros(m, np.int32)
    checks = lib.oracle_check_motions(C.byref(s), C.byref(c), abi.dptr(a), abi.dptr(b), m,
                                      valid.ctypes.data_as(_U8), nd.ctypes.data_as(_I32), fi.ctypes.data_as(_I32))
    return valid.astype(bool), nd, fi, int(checks)


def check_motions_mt(sp, ck, s1, s2, nthreads=1):
    s, c = sp.to_abi(), ck.to_abi()
    a, b = _arr(s1).reshape(-1, sp.dim), _arr(s2).reshape(-1, sp.dim)
    valid = np.zeros(a.shape[0], np.uint8)
    lib.oracle_check_motions_mt(C.byref(s), C.byref(c), abi.dptr(a), abi.dptr(b), a.shape[0],
                                valid.ctypes.data_as(_U8), int(nthreads))
    return valid.astype(bool)


def knn(sp, data, queries, k):
    s = sp.to_abi()
    d, q = _arr(data).reshape(-1, sp.dim), _arr(queries).reshape(-1, sp.dim)
    nq = q.shape[0]
    ids = np.zeros((nq, k), np.uint32)
    dist = np.zeros((nq, k))
    cnt = np.zeros(nq, np.uint32)
    lib.oracle_knn(C.byref(s), abi.dptr(d), d.shape[0], abi.dptr(q), nq, k, ids.ctypes.data_as(_U32), abi.dptr(dist),
                   cnt.ctypes.data_as(_U32))
    return ids, dist, cnt


def radius(sp, data, queries, r):
    s = sp.to_abi()
    d, q = _arr(data).reshape(-1, sp.dim), _arr(queries).reshape(-1, sp.dim)
    nq = q.shape[0]
    cnt = np.zeros(nq, np.uint64)
    lib.oracle_radius(C.byref(s), abi.dptr(d), d.shape[0], abi.dptr(q), nq, float(r), None, None, None,
                      cnt.ctypes.data_as(_U64))
    off = np.zeros(nq + 1, np.uint64)
    off[1:] = np.cumsum(cnt)
    tot = int(off[-1])
    ids = np.zeros(max(tot, 1), np.uint32)
    dist = np.zeros(max(tot, 1))
    lib.oracle_radius(C.byref(s), abi.dptr(d), d.shape[0], abi.dptr(q), nq, float(r), off.ctypes.data_as(_U64),
                      ids.ctypes.data_as(_U32), abi.dptr(dist), cnt.ctypes.data_as(_U64))
    return off, ids[:tot], dist[:tot]


def prm_causal(sp, ck, states, k_const, k_cap):
    """Sequential PRM* construction: (neighbours [n, k_cap], counts [n], validity [n, k_cap])."""
    s, c = sp.to_abi(), ck.to_abi()
    x = _arr(states).reshape(-1, sp.dim)
    n = x.shape[0]
    nbr = np.zeros((n, k_cap), np.uint32)
    cnt = np.zeros(n, np.uint32)
    val = np.zeros((n, k_cap), np.uint8)
    lib.oracle_prm_causal(C.byref(s), C.byref(c), abi.dptr(x), n, float(k_const), int(k_cap),
                          nbr.ctypes.data_as(_U32), cnt.ctypes.data_as(_U32), val.ctypes.data_as(_U8))
    return nbr, cnt, val


def rrtstar(sp, ck, states0, parent0, inc0, cost0, samples, maxd, k_rrt, use_gnat=False, time_budget_s=0.0):
    """RRT*'s sequential iteration (oracle/rrtstar.cpp) from the given tree over the samples:
    dict with nearest / added / parent_choice per sample, the final tree's parent / inc / cost,
    and stats (processed, added, rewires, checkMotion calls)."""
    s, c = sp.to_abi(), ck.to_abi()
    x0 = _arr(states0).reshape(-1, sp.dim)
    smp = _arr(samples).reshape(-1, sp.dim)
    n0, ns = x0.shape[0], smp.shape[0]
    p0 = np.ascontiguousarray(parent0, dtype=np.int64)
    i0, c0 = _arr(inc0), _arr(cost0)
    near = np.zeros(ns, np.uint32)
    added = np.zeros(ns, np.uint32)
    choice = np.zeros(ns, np.int64)
    par = np.zeros(n0 + ns, np.int64)
    inc = np.zeros(n0 + ns)
    cost = np.zeros(n0 + ns)
    st = np.zeros(5, np.uint64)
    lib.oracle_rrtstar(C.byref(s), C.byref(c), abi.dptr(x0), n0, p0.ctypes.data_as(_I64), abi.dptr(i0), abi.dptr(c0),
                       abi.dptr(smp), ns, float(maxd), float(k_rrt), int(use_gnat), float(time_budget_s),
                       near.ctypes.data_as(_U32), added.ctypes.data_as(_U32), choice.ctypes.data_as(_I64),
                       par.ctypes.data_as(_I64), abi.dptr(inc), abi.dptr(cost), st.ctypes.data_as(_U64))
    m = n0 + int(st[1])
    return {"nearest": near, "added": added, "parent_choice": choice, "parent": par[:m], "inc": inc[:m],
            "cost": cost[:m], "processed": int(st[0]), "n_added": int(st[1]), "rewires": int(st[2]),
            "checks": int(st[3]), "loop_s": float(st[4]) * 1e-9}


def seed_stream(seed, n):
    """The first n RNG() seeds after RNG::setSeed(seed)."""
    out = np.zeros(n, np.uint32)
    lib.oracle_seed_stream(int(seed), int(n), out.ctypes.data_as(_U32))
    return out


def sample_uniform(sp, local_seeds, n, low=None, high=None):
    """n sampleUniform() of the space's default sampler with the given RNG local seeds."""
    s = sp.to_abi()
    seeds = np.ascontiguousarray(local_seeds, dtype=np.uint32)
    lo = _arr(low if low is not None else getattr(sp, "low", [0.0]))
    hi = _arr(high if high is not None else getattr(sp, "high", [1.0]))
    out = np.zeros((int(n), sp.dim))
    lib.oracle_sample_uniform(C.byref(s), seeds.ctypes.data_as(_U32), abi.dptr(lo), abi.dptr(hi), int(n),
                              abi.dptr(out))
    return out


class Gnat:
    """GNAT restatement (oracle/gnat.cpp), reference defaults 8/4/12/50."""

    def __init__(self, sp, degree=8, min_degree=4, max_degree=12, leaf=50, seed=1):
        self.sp = sp
        self._s = sp.to_abi()
        self._h = lib.oracle_gnat_create(C.byref(self._s), degree, min_degree, max_degree, leaf, seed)

    def __del__(self):
        if getattr(self, "_h", None) and lib is not None:  # lib is None at interpreter shutdown
            lib.oracle_gnat_destroy(self._h)
            self._h = None

    def add(self, states, bulk=False):
        x = _arr(states).reshape(-1, self.sp.dim)
        (lib.oracle_gnat_add_bulk if bulk else lib.oracle_gnat_add)(self._h, abi.dptr(x), x.shape[0])

    def size(self):
        return lib.oracle_gnat_size(self._h)

    def knn(self, queries, k, nthreads=1):
        q = _arr(queries).reshape(-1, self.sp.dim)
        nq = q.shape[0]
        ids = np.zeros((nq, k), np.uint32)
        dist = np.zeros((nq, k))
        cnt = np.zeros(nq, np.uint32)
        lib.oracle_gnat_knn(self._h, abi.dptr(q), nq, k, ids.ctypes.data_as(_U32), abi.dptr(dist),
                            cnt.ctypes.data_as(_U32), int(nthreads))
        return ids, dist, cnt

    def radius_count(self, queries, r, nthreads=1):
        q = _arr(queries).reshape(-1, self.sp.dim)
        cnt = np.zeros(q.shape[0], np.uint64)
        tot = lib.oracle_gnat_radius_count(self._h, abi.dptr(q), q.shape[0], float(r), cnt.ctypes.data_as(_U64),
                                           int(nthreads))
        return cnt, int(tot)

    def radius(self, queries, r, nthreads=1):
        """nearestR: CSR (offsets [nq + 1], ids, distances), each segment sorted by (distance, id)."""
        q = _arr(queries).reshape(-1, self.sp.dim)
        off = np.zeros(q.shape[0] + 1, np.uint64)
        tot = lib.oracle_gnat_radius(self._h, abi.dptr(q), q.shape[0], float(r), off.ctypes.data_as(_U64),
                                     int(nthreads))
        ids = np.zeros(max(int(tot), 1), np.uint32)
        dist = np.zeros(max(int(tot), 1))
        lib.oracle_gnat_radius_fetch(self._h, ids.ctypes.data_as(_U32), abi.dptr(dist))
        return off, ids[:tot], dist[:tot]


# ---- the reference's own NearestNeighborsLinear (built from /root/reference) ----
def ref_knn(sp, data, queries, k):
    s = sp.to_abi()
    d, q = _arr(data).reshape(-1, sp.dim), _arr(queries).reshape(-1, sp.dim)
    nq = q.shape[0]
    ids = np.zeros((nq, k), np.uint32)
    dist = np.zeros((nq, k))
    cnt = np.zeros(nq, np.uint32)
    ref.ref_linear_knn(C.byref(s), abi.dptr(d), d.shape[0], abi.dptr(q), nq, k, ids.ctypes.data_as(_U32),
                       abi.dptr(dist), cnt.ctypes.data_as(_U32))
    return ids, dist, cnt


def ref_nearest(sp, data, queries):
    s = sp.to_abi()
    d, q = _arr(data).reshape(-1, sp.dim), _arr(queries).reshape(-1, sp.dim)
    ids = np.zeros(q.shape[0], np.uint32)
    err = C.create_string_buffer(128)
    rc = ref.ref_linear_nearest(C.byref(s), abi.dptr(d) if d.size else None, d.shape[0], abi.dptr(q), q.shape[0],
                                ids.ctypes.data_as(_U32), err)
    return rc, ids, err.value.decode()


def ref_radius(sp, data, queries, r):
    s = sp.to_abi()
    d, q = _arr(data).reshape(-1, sp.dim), _arr(queries).reshape(-1, sp.dim)
    nq = q.shape[0]
    cnt = np.zeros(nq, np.uint64)
    ref.ref_linear_radius(C.byref(s), abi.dptr(d), d.shape[0], abi.dptr(q), nq, float(r), None, None,
                          cnt.ctypes.data_as(_U64))
    off = np.zeros(nq + 1, np.uint64)
    off[1:] = np.cumsum(cnt)
    ids = np.zeros(max(int(off[-1]), 1), np.uint32)
    ref.ref_linear_radius(C.byref(s), abi.dptr(d), d.shape[0], abi.dptr(q), nq, float(r), off.ctypes.data_as(_U64),
                          ids.ctypes.data_as(_U32), cnt.ctypes.data_as(_U64))
    return off, ids[:int(off[-1])]
