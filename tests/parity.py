"""Parity helpers shared by the GPU tests.

Definition: per-rank fp64 distances bit-identical (DIST_ULPS = 0: the device's
acos / sin / cos are glibc's own algorithms, glibc_acos.h / glibc_sincos.h, so every space's metric
is exact in the reference's operation order); ids equal at every rank outside a tie class (states at
exactly the same distance); inside a tie class the id sets are equal, except for the class
straddling the k-th rank, where any members are accepted (the reference itself resolves that class
by heap / traversal order).
"""
import numpy as np

DIST_ULPS = 0


def dist_tol(d):
    d = np.asarray(d, dtype=np.float64)
    return DIST_ULPS * np.spacing(np.maximum(np.abs(d), 1.0))  # 0: exact


def assert_dist_close(gd, od):
    gd, od = np.asarray(gd), np.asarray(od)
    fin = np.isfinite(od)
    assert np.array_equal(fin, np.isfinite(gd)), "finite / missing entries differ"
    err = np.abs(gd[fin] - od[fin])
    tol = dist_tol(od[fin])
    bad = err > tol
    assert not bad.any(), f"{bad.sum()} distances beyond {DIST_ULPS} ulps, max err {err.max():.3e}"
    return float(np.mean(gd[fin] == od[fin])) if fin.any() else 1.0


def assert_knn_parity(gi, gd, oi_ext, od_ext, k):
    """gi/gd: GPU [nq, k]; oi_ext/od_ext: oracle [nq, K>=k] (K > k exposes the boundary class)."""
    gi, gd = np.asarray(gi, dtype=np.int64), np.asarray(gd)
    oi_ext, od_ext = np.asarray(oi_ext, dtype=np.int64), np.asarray(od_ext)
    exact = assert_dist_close(gd, od_ext[:, :k])
    mism = 0
    for q in range(gi.shape[0]):
        od = od_ext[q]
        tol = dist_tol(od)
        j = 0
        while j < k and np.isfinite(od[j]):
            e = j
            while e + 1 < len(od) and np.isfinite(od[e + 1]) and od[e + 1] - od[e] <= tol[e]:
                e += 1
            cls = set(oi_ext[q, j:e + 1].tolist())
            got = set(gi[q, j:min(e + 1, k)].tolist())
            if e < k:  # class entirely inside the first k ranks: same ids (as a set)
                if got != cls:
                    mism += 1
            elif not got <= cls:  # boundary class: GPU picks any members
                mism += 1
            j = e + 1
    assert mism == 0, f"{mism} tie classes with different ids"
    return exact


def assert_knn_parity_rows(gi, gd, oi_ext, od_ext, k):
    """assert_knn_parity for large batches: distances vectorised, the per-row tie-class walk only
    on the rows whose ids differ from the oracle's first k."""
    gi, gd = np.asarray(gi, dtype=np.int64), np.asarray(gd)
    oi_ext, od_ext = np.asarray(oi_ext, dtype=np.int64), np.asarray(od_ext)
    exact = assert_dist_close(gd, od_ext[:, :k])
    bad = np.flatnonzero(np.any(gi[:, :k] != oi_ext[:, :k], axis=1))
    if len(bad):
        assert_knn_parity(gi[bad], gd[bad], oi_ext[bad], od_ext[bad], k)
    return exact, len(bad)


CPU_THREADS = 16  # the GPU box's CPU share per GPU (the oracle's const queries run on this many threads)


def oracle_knn_mt(O, sp, data, queries, k, threads=8):
    """The oracle's brute force over query slices on `threads` threads (ctypes drops the GIL),
    for parity checks at the configs' full store sizes."""
    from concurrent.futures import ThreadPoolExecutor

    parts = np.array_split(np.arange(len(queries)), min(threads, len(queries)))
    with ThreadPoolExecutor(len(parts)) as ex:
        res = list(ex.map(lambda ix: O.knn(sp, data, queries[ix], k), parts))
    return (np.concatenate([r[0] for r in res]), np.concatenate([r[1] for r in res]))
