"""Benchmark: NN queries/s + motion checks/s on a 10^6-state SE(3) tree (BASELINE.json).

Default workload (BASELINE.json configs[2]): an SE(3) tree of 10^6 states
(translation in [0,1]^3, uniform rotations, seed 42) resident in HBM; per GPU a batch of
10^5 sampled states (the RRT* sampling step).  One step = for every sample
    nearestK(k=10)                                   (NearestNeighborsGNAT.h:222-233)
    steer from its nearest to range 0.2*extent        (RRT.cpp:137-146)
    checkMotion(nearest, steered) with the HypercubeBenchmark predicate on the
    translation, resolution 0.01                      (DiscreteMotionValidator.cpp:93-145)
all on device, inputs resident in HBM.  value = (NN queries + motion checks) per second
over all ranks.  Multi-GPU: the tree is replicated, samples are sharded (weak scaling,
no collective in the data path).

The other configurations are measured with --workload (same JSON line, same unit):
    cfg2  R^6, 10^5 states, batched nearestK(k=10)                       (configs[1], M1)
    cfg4  PRM* roadmap construction in the KinematicChain R^12 space, causal: a 10^6-vertex
          valid roadmap, then per step the next B valid milestones, each connected to its
          k_i = ceil((e + e/12) ln(i + 1)) nearest among ALL earlier vertices (the roadmap and
          the batch's earlier milestones) + checkMotion(neighbour, milestone) per edge, then
          inserted (PRM.cpp:562-596)                                     (configs[3], M3)
    cfg5  BIT* batch on SE(3): 10^7 valid samples, per step 10^5 vertices -> nearestR
          (r = 0.1528, ImplicitGraph.cpp:1372-1381) + checkMotion(vertex, sample) for every
          edge, 32-sphere checker                                     (configs[4], M4)

    python bench.py [--gpus N] [--steps K] [--warmup W] [--workload cfg3|cfg2|cfg4|cfg5]
"""
from __future__ import annotations

import argparse
import json
import math
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "NN queries/sec + motion checks/sec on 10^6-state SE(3) tree"
UNIT = "(NN queries + motion checks)/s"
PEAK_TFLOPS = {"f32": 157.3, "f64": 78.6}  # MI355X vector peaks (MI355X_MICROARCH.md)
HBM_PEAK_GBS = 8000.0                       # HBM3E spec
# flops per distance evaluation (SURVEY.md §8d constants; sqrt and acos counted as 1 each)
F_SE3, F_L2_6, F_CHAIN = 21, 18, 84
B_SE3 = {"f32": 28, "f64": 56}              # bytes per stored SE(3) state streamed by a scan
# committed PMC passes per workload, newest round first (cfg5k = configs[4] in kNN mode)
PMC_PROFILES = {w: [f"r6_{w}", f"r5_{w}", f"r4_{w}", f"r3_{w}"] for w in ("cfg3", "cfg2", "cfg4", "cfg5")}
PMC_PROFILES["cfg5k"] = ["r6_cfg5k", "r5_cfg5k", "r4_cfg5k"]
PMC_PROFILES["rrt_star"] = ["r6_rrt_star", "r5_rrt_star"]
DEFAULTS = {  # tree states, queries (samples / milestones / vertices) per GPU per step, k
    "cfg3": (1_000_000, 100_000, 10),
    "cfg2": (100_000, 100_000, 10),
    "cfg4": (1_000_000, 8_192, 0),
    "cfg5": (10_000_000, 100_000, 0),
}


def pmc_traffic(workload, kernel):
    """HBM bytes per launch of `kernel` from the committed rocprofv3 --pmc passes
    (FETCH_SIZE doubled per MI355X_MICROARCH.md's gfx950 correction, + WRITE_SIZE)."""
    for d in PMC_PROFILES.get(workload, ()):
        path = os.path.join(ROOT, "profiles", d, "pmc_summary.json")
        try:
            with open(path) as f:
                per = json.load(f)["per_kernel_mean"]
        except (OSError, ValueError, KeyError):
            continue
        # the timed launch is the kernel's dominant instance (the chain cull: its MODE 2 pass, not
        # the pre-pass): the largest per-dispatch traffic among the instances of that name
        best = None
        for name, c in per.items():
            if name.split("<")[0].endswith(kernel) and "FETCH_SIZE" in c and "WRITE_SIZE" in c:
                b = (2 * c["FETCH_SIZE"] + c["WRITE_SIZE"]) * 1024.0
                if best is None or b > best["bytes"]:
                    best = {"bytes": b, "source": os.path.relpath(path, ROOT) + f" [{name}]"}
        if best:
            return best
    return None


def sq_issue(workload, kernel, waves, kern_ms):
    """VALU issue utilisation of `kernel` from the committed SQ pass (tools/sq_counters.sh): VALU
    instructions per wave (SQ_INSTS_VALU / SQ_WAVES of the sampled SQ instances) x the launch's waves x
    2 cycles per wave64 VALU instruction (SIMD-32 with >= 2 waves resident, MI355X_MICROARCH.md
    'Wave scheduling') over 1,024 SIMDs x 2.4 GHz x the measured kernel time; the SALU figure the same
    way at one SALU instruction per cycle per CU (256 CUs)."""
    for d in PMC_PROFILES.get(workload, ()):
        path = os.path.join(ROOT, "profiles", d, "sq_summary.json")
        try:
            with open(path) as f:
                per = json.load(f)["per_kernel_mean"]
        except (OSError, ValueError, KeyError):
            continue
        for name, c in per.items():
            if name.split("<")[0].endswith(kernel) and c.get("SQ_WAVES") and c.get("SQ_INSTS_VALU"):
                valu = c["SQ_INSTS_VALU"] / c["SQ_WAVES"]
                salu = c.get("SQ_INSTS_SALU", 0.0) / c["SQ_WAVES"]
                busy = valu * waves * 2 / (1024 * 2.4e9 * kern_ms * 1e-3)
                sbusy = salu * waves / (256 * 2.4e9 * kern_ms * 1e-3)
                out = {"valu_per_wave": round(valu), "salu_per_wave": round(salu), "waves": waves,
                       "valu_issue_busy": round(busy, 3), "salu_issue_busy": round(sbusy, 3),
                       "source": os.path.relpath(path, ROOT) + f" [{name}]"}
                if c.get("SQ_WAVE_CYCLES") and c.get("SQ_WAIT_ANY"):
                    out["wait_any_frac"] = round(c["SQ_WAIT_ANY"] / c["SQ_WAVE_CYCLES"], 3)
                return out
    return None


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--workload", default="cfg3", choices=sorted(DEFAULTS))
    ap.add_argument("--tree", type=int, default=None)
    ap.add_argument("--queries", type=int, default=None, help="samples / milestones / vertices per GPU per step")
    ap.add_argument("--k", type=int, default=None)
    ap.add_argument("--exact", action="store_true", help="force the exact fp64 scan (no fp32 screen)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-seconds", type=float, default=12.0, help="budget of the CPU baseline sample")
    ap.add_argument("--single-query-reps", type=int, default=200, help="RRT-style one-query scans (0 = skip)")
    ap.add_argument("--rrt-iters", type=int, default=2000, help="device RRT iterations after the bench (0 = skip)")
    ap.add_argument("--no-extras", action="store_true",
                    help="skip the extra measurements (index maintenance, sphere checker, RRT* k) after the timed steps")
    ap.add_argument("--scaling", default="weak", choices=["weak", "strong"],
                    help="replicated tree: --queries per GPU (weak, the default) or --queries in total split over "
                         "the GPUs (strong)")
    ap.add_argument("--partition", default="replicated", choices=["replicated", "tree"],
                    help="cfg3: replicated tree + sharded samples (default, weak scaling), or the tree sharded over "
                         "the ranks with every sample answered by every shard and the per-shard top-k lists merged "
                         "(all_gather over RCCL + the library's merge kernel; strong scaling)")
    ap.add_argument("--bitstar-knn", action="store_true",
                    help="cfg5: BIT*'s default kNN neighbourhood (useKNearest_, bitstar/ImplicitGraph.h:463), "
                         "k = ceil(1.1 (e + e/6) ln n) = 57 at 10^7, instead of the radius mode")
    ap.add_argument("--rrt-star-queries", type=int, default=1000,
                    help="cfg3: batch of RRT* neighbourhood queries at k = 6,169 (0 = skip)")
    ap.add_argument("--rrt-star-samples", type=int, default=10_000,
                    help="RRT* workload (configs[2], the `workloads` record's rrt_star entry): samples per step "
                         "(0 = skip)")
    ap.add_argument("--workloads", default="auto",
                    help="configs measured after the headline into the line's `workloads` record: 'auto' = "
                         f"{','.join(SUB_WORKLOADS)} when the headline is cfg3 replicated, 'none', or a comma list")
    ap.add_argument("--sub-cpu-seconds", type=float, default=6.0, help="CPU baseline budget of each sub-workload")
    ap.add_argument("--lanes", type=int, default=2,
                    help="steps in flight for workloads whose batches are independent (cfg3, cfg2, cfg5 kNN): step i "
                         "runs on stream i %% lanes with its own NN / validator handles over the same tree, so the next "
                         "step's walk fills the CUs the current walk's tail leaves idle (1 = one stream)")
    ap.add_argument("--detail", default=os.path.join("gpurun_out", "bench_detail.json"),
                    help="file for the full record (the stdout line is the compact form); '' = none")
    a = ap.parse_args()
    if a.partition == "tree" and (a.workload not in ("cfg3", "cfg5") or a.bitstar_knn):
        ap.error("--partition tree is implemented for --workload cfg3 and the cfg5 radius mode")
    t, q, k = DEFAULTS[a.workload]
    a.tree = t if a.tree is None else a.tree
    a.queries = q if a.queries is None else a.queries
    a.k = k if a.k is None else a.k
    return a


def reference_inputs(sp, n_tree, nq, rank, valid=None):
    """The reference's input streams: RNG::setSeed(42), then a tree sampler and a query sampler
    (space->allocStateSampler() twice, RandomNumbers.cpp:53-279, StateSpace.cpp:800-806).  The
    tree is identical on every rank; rank r takes queries [r*nq, (r+1)*nq) of the query stream.
    With `valid`, only valid states are kept, in stream order (UniformValidStateSampler)."""
    tree, q = _stream_inputs(sp, n_tree, nq * (rank + 1), valid)
    return tree, np.ascontiguousarray(q[rank * nq:])


def _stream_inputs(sp, n_tree, n_q, valid=None):
    """(tree, the first n_q states of the query stream) — see reference_inputs."""
    from ompl_amd import sampling as S
    from ompl_amd import workloads as W

    S.set_seed(42)
    ts, qs = S.StateSampler(sp), S.StateSampler(sp)
    if valid is None:
        return ts.sample_uniform(n_tree), qs.sample_uniform(n_q)
    tree, _ = W.reference_valid_states(sp, n_tree, valid, sampler=ts, chunk=min(2_000_000, max(4 * n_tree, 4096)))
    q, _ = W.reference_valid_states(sp, n_q, valid, sampler=qs, chunk=min(2_000_000, max(4 * n_q, 4096)))
    return tree, q


_INPUTS = {}  # (space, checker, n_tree, n_q) -> (tree, queries): cfg5's radius and kNN lines share one sample set


def shared_inputs(key, sp, n_tree, n_q, valid, dist, dev):
    """The tree and the first n_q query-stream states, drawn once per process and, with several
    ranks, drawn on rank 0 only and broadcast over RCCL (the replicas are identical by
    construction; at N = 8 this keeps eight ranks from re-sampling 10^7 valid states on the same
    host cores)."""
    k = (key, n_tree, n_q)
    if k in _INPUTS:
        return _INPUTS[k]
    if dist is None:
        out = _stream_inputs(sp, n_tree, n_q, valid)
    else:
        import torch

        root = dist.get_rank() == 0
        arrs = _stream_inputs(sp, n_tree, n_q, valid) if root else None
        meta = [[a.shape for a in arrs] if root else None]
        dist.broadcast_object_list(meta, src=0, device=dev)
        out = []
        for i, shape in enumerate(meta[0]):
            t = (torch.from_numpy(np.ascontiguousarray(arrs[i])).to(dev) if root
                 else torch.empty(shape, dtype=torch.float64, device=dev))
            dist.broadcast(t, src=0)
            out.append(t.cpu().numpy())
            del t
        out = tuple(out)
    _INPUTS.clear()  # keep one set: the next workload either reuses it or needs another
    _INPUTS[k] = out
    return out


CPU_THREADS = 8  # SURVEY §8d protocol: 1 core and all 8 cores of the reference container


def _gnat_knn_rate(sp, tree, queries, k, budget_s, nthreads):
    """GNAT restatement (oracle/gnat.cpp, reference defaults) over the tree: queries/s of
    nearestK on `nthreads` threads (const queries on one structure, like the reference's
    thread-safe GNAT), on as many queries as fit the budget.  Build time reported apart."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import pyoracle as O

    g = O.Gnat(sp)
    t0 = time.perf_counter()
    g.add(tree)
    build_s = time.perf_counter() - t0
    out = {"build_s": build_s}
    for nt in (1, nthreads):
        t0 = time.perf_counter()
        g.knn(queries[:200 * nt], k, nt)
        per = (time.perf_counter() - t0) / (200 * nt)
        nq = int(min(len(queries), max(200 * nt, 0.3 * budget_s / max(per, 1e-9))))
        t0 = time.perf_counter()
        ids, d, _ = g.knn(queries[:nq], k, nt)
        out[nt] = (nq, nq / (time.perf_counter() - t0), ids, d)
    return out


def _motion_rate(sp, ck, s1, s2, budget_s, nthreads):
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import pyoracle as O

    t0 = time.perf_counter()
    O.check_motions_mt(sp, ck, s1, s2, nthreads)
    t = time.perf_counter() - t0
    reps = 1
    if t < budget_s:
        reps = int(max(1, budget_s / max(t, 1e-9)))
        t0 = time.perf_counter()
        for _ in range(reps):
            O.check_motions_mt(sp, ck, s1, s2, nthreads)
        t = (time.perf_counter() - t0) / reps
    return len(s1) / t, reps


def cpu_baseline(workload, sp, ck, tree, queries, k, budget_s, radius=None):
    """The oracle restatement on a bounded sample of the same workload (the run's own queries) on
    this host, on 1 thread and on CPU_THREADS threads: GNAT (oracle/gnat.cpp,
    reference defaults) where building it over the tree is affordable (cfg2, cfg3), else the
    Linear brute force (cfg4: 10^6 chain states, cfg5: 10^7 SE(3) samples) — a slower CPU path
    than the reference's GNAT, said so in `sample`.  `value` is the all-threads figure."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import pyoracle as O

    T = CPU_THREADS
    if workload in ("cfg3", "cfg2"):
        r = _gnat_knn_rate(sp, tree, queries, k, budget_s, T)
        (nq1, qps1, ids, d), (nqT, qpsT, _, _) = r[1], r[T]
        if workload == "cfg2":
            return {"value": qpsT, "unit": "NN queries/s", "cores": T, "kind": "port",
                    "sample": (f"GNAT restatement (oracle/gnat.cpp, degree 8/4/12, 50/leaf) over the same 10^5-state "
                               f"R^6 store, the run's own queries: {nqT} nearestK(k={k}) on {T} threads "
                               f"(const queries on one structure); index build {r['build_s']:.2f} s excluded"),
                    "single_thread": {"value": qps1, "queries": nq1}, "nn_queries_per_s": qpsT}
        maxd = 0.2 * sp.getMaximumExtent()
        s1 = tree[ids[:, 0].astype(np.int64)]
        q = queries[:nq1]
        s2 = np.empty_like(q)
        for i in range(nq1):  # steering is not timed on the CPU side (favours the CPU)
            s2[i] = O.interpolate(sp, s1[i], q[i], maxd / d[i, 0]) if d[i, 0] > maxd else q[i]
        mps1, _ = _motion_rate(sp, ck, s1, s2, 0.15 * budget_s, 1)
        mpsT, reps = _motion_rate(sp, ck, s1, s2, 0.15 * budget_s, T)
        comb = lambda a, b: 2.0 / (1.0 / a + 1.0 / b)  # noqa: E731  (one query + one motion check per sample)
        return {"value": comb(qpsT, mpsT), "unit": UNIT, "cores": T, "kind": "port",
                "sample": (f"GNAT restatement (oracle/gnat.cpp, degree 8/4/12, 50/leaf) over the same 10^6-state "
                           f"SE(3) tree and the run's own samples: {nqT} nearestK(k={k}) queries, then {nq1} "
                           f"checkMotion(nearest, steered) x{reps} with the oracle DiscreteMotionValidator, on {T} "
                           f"threads; index build {r['build_s']:.2f} s excluded"),
                "single_thread": {"value": comb(qps1, mps1), "nn_queries_per_s": qps1, "motion_checks_per_s": mps1},
                "nn_queries_per_s": qpsT, "motion_checks_per_s": mpsT, "gnat_build_s": r["build_s"]}
    if workload == "cfg4":
        return _cpu_prm_causal(sp, ck, tree, queries, k, budget_s, T)
    return _cpu_bitstar_radius(sp, ck, tree, queries, radius, budget_s, T, k)


def _cpu_prm_causal(sp, ck, tree, milestones, k_cap, budget_s, T):
    """PRM*'s causal insertion on the GNAT restatement (PRM.cpp:562-596, KStarStrategy
    ConnectionStrategy.h:124-156): milestone i queries its k_i = ceil((e + e/d) ln(i + 1)) nearest
    among every vertex before it, is inserted, and its edges checkMotion(state[n], state[m]) are
    checked.  1 thread: exactly that sequential loop.  T threads: the decomposition the GPU uses
    for a batch — the batch's kNN over the stored roadmap as const queries on T threads, then its
    edges on T threads (the in-batch causal candidates, < 1 % of the neighbours, are left out of the
    threaded sample, which favours the CPU).  `value` is the T-thread figure."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import pyoracle as O

    g = O.Gnat(sp)
    t0 = time.perf_counter()
    g.add(tree, bulk=True)
    build_s = time.perf_counter() - t0
    kc = math.e + math.e / sp.dim
    n0 = len(tree)
    # T threads over the stored roadmap (queries before any insert: every milestone sees the n0 states)
    kq = min(int(math.ceil(kc * math.log(n0 + 1))), k_cap)
    t0 = time.perf_counter()
    g.knn(milestones[:16 * T], kq, T)
    per = (time.perf_counter() - t0) / (16 * T)
    nT = int(min(len(milestones), max(16 * T, 0.3 * budget_s / max(per, 1e-9))))
    t0 = time.perf_counter()
    idsT, _, cntT = g.knn(milestones[:nT], kq, T)
    t_nnT = time.perf_counter() - t0
    s1T = tree[idsT[:, :kq].reshape(-1).astype(np.int64)]
    s2T = np.repeat(milestones[:nT], kq, axis=0)
    mpsT, repsT = _motion_rate(sp, ck, s1T, s2T, 0.15 * budget_s, T)
    mT = len(s1T)
    # 1 thread: the sequential causal loop
    s1, s2, nq = [], [], 0
    t_nn = 0.0
    for i, q in enumerate(milestones):
        kq1 = min(int(math.ceil(kc * math.log(n0 + i + 1))), k_cap)
        t0 = time.perf_counter()
        ids, _, cnt = g.knn(q, kq1)
        g.add(q)
        t_nn += time.perf_counter() - t0
        nq += 1
        for j in ids[0, :cnt[0]].astype(np.int64):
            s1.append(tree[j] if j < n0 else milestones[j - n0])
            s2.append(q)
        if t_nn > 0.3 * budget_s:
            break
    s1, s2 = np.asarray(s1), np.asarray(s2)
    mps1, reps = _motion_rate(sp, ck, s1, s2, 0.15 * budget_s, 1)
    m = len(s1)
    return {"value": (nT + mT) / (t_nnT + mT / mpsT), "unit": UNIT, "cores": T, "kind": "port",
            "sample": (f"GNAT restatement (oracle/gnat.cpp, degree 8/4/12, 50/leaf) over the same {n0}-vertex roadmap: "
                       f"{nT} milestones' nearestK(k={kq}) over the roadmap as const queries on {T} threads, then their "
                       f"{mT} checkMotion edges x{repsT} with the oracle DiscreteMotionValidator on {T} threads; index "
                       f"build {build_s:.1f} s excluded"),
            "nn_queries_per_s": nT / t_nnT, "motion_checks_per_s": mpsT, "gnat_build_s": build_s,
            "single_thread": {"value": (nq + m) / (t_nn + m / mps1), "nn_queries_per_s": nq / t_nn,
                              "motion_checks_per_s": mps1,
                              "sample": f"the first {nq} milestones inserted causally (k_i nearest, then add), "
                                        f"their {m} edges x{reps}"}}


def _cpu_bitstar_radius(sp, ck, tree, queries, radius, budget_s, T, k=0):
    """BIT*'s batch on the GNAT restatement: nearestR(r) — or, with k, nearestK(k) (BIT*'s kNN
    mode) — of each vertex over the sample set (ImplicitGraph.cpp:313-320, GNAT nearestR / nearestK
    NearestNeighborsGNAT.h:222-245) on 1 and T threads (const queries), plus checkMotion(vertex,
    sample) of the edges.  The edges' motion rate is measured on the pairs of a few queries."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import pyoracle as O

    g = O.Gnat(sp)
    t0 = time.perf_counter()
    g.add(tree, bulk=True)
    build_s = time.perf_counter() - t0
    rate = {}

    def query(qs, nt):
        if k:
            g.knn(qs, k, nt)
            return len(qs) * k
        return g.radius_count(qs, radius, nt)[1]

    for nt in (1, T):
        t0 = time.perf_counter()
        query(queries[:4 * nt], nt)
        per = (time.perf_counter() - t0) / (4 * nt)
        nq = int(min(len(queries), max(4 * nt, 0.25 * budget_s / max(per, 1e-9))))
        t0 = time.perf_counter()
        tot = query(queries[:nq], nt)
        rate[nt] = (nq, time.perf_counter() - t0, tot)
    if k:
        ids, _, _ = O.knn(sp, tree, queries[:8], k)
        s1 = np.repeat(queries[:8], k, axis=0)
        s2 = tree[ids.reshape(-1).astype(np.int64)]
    else:
        off, ids, _ = O.radius(sp, tree, queries[:8], radius)
        s1 = np.repeat(queries[:8], np.diff(off).astype(np.int64), axis=0)
        s2 = tree[ids.astype(np.int64)]
    mps = {nt: _motion_rate(sp, ck, s1, s2, 0.15 * budget_s, nt) for nt in (1, T)}

    def comb(nt):
        nq, t, tot = rate[nt]
        return (nq + tot) / (t + tot / mps[nt][0])

    nqT, tT, totT = rate[T]
    what = f"nearestK(k={k})" if k else f"nearestR(r={radius:.4f})"
    return {"value": comb(T), "unit": UNIT, "cores": T, "kind": "port",
            "sample": (f"GNAT restatement (oracle/gnat.cpp, degree 8/4/12, 50/leaf) over the same {len(tree)}-sample "
                       f"set: {nqT} {what} of the run's vertices ({totT} neighbours) on {T} threads "
                       f"(const queries), their checkMotion(vertex, sample) edges at the rate measured on "
                       f"{len(s1)} edges of 8 vertices; index build {build_s:.1f} s excluded"),
            "single_thread": {"value": comb(1), "nn_queries_per_s": rate[1][0] / rate[1][1],
                              "motion_checks_per_s": mps[1][0]},
            "nn_queries_per_s": nqT / tT, "motion_checks_per_s": mps[T][0], "gnat_build_s": build_s}


def single_query_scan(torch, nn, dev, reps, n_tree, note=None):
    """RRT semantics (RRT.cpp:137): one nearest() per iteration -> the fp32 stream kernel
    (knn_stream32.hip: 28 B per SE(3) state, exact by in-chunk fp64 refinement), HBM bound."""
    from ompl_amd import workloads as W

    q = torch.from_numpy(W.uniform_se3(np.random.default_rng(99), reps)).to(dev)
    ids = torch.empty(reps, dtype=torch.int32, device=dev)
    dd = torch.empty(reps, dtype=torch.float64, device=dev)
    for i in range(5):
        nn.knn_device(q[i].data_ptr(), 1, 1, ids[i].data_ptr(), dd[i].data_ptr())
    torch.cuda.synchronize(dev)
    nn.profile(True)
    ms0, n0, _ = nn.kernel_time()
    t0 = time.perf_counter()
    for i in range(reps):
        nn.knn_device(q[i].data_ptr(), 1, 1, ids[i].data_ptr(), dd[i].data_ptr())
    torch.cuda.synchronize(dev)
    wall = time.perf_counter() - t0
    ms1, n1, name = nn.kernel_time()
    kern_ms = (ms1 - ms0) / max(n1 - n0, 1)
    b = B_SE3["f64"] if name == "knn_stream_kernel" else B_SE3["f32"]  # the fp64 stream reads 56 B per state
    achieved = n_tree * b / (kern_ms * 1e-3) / 1e9
    return {"queries_per_s": reps / wall, "kernel": name, "kernel_us": kern_ms * 1e3, "tree_states": n_tree,
            "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": achieved / HBM_PEAK_GBS,
                         "algorithmic": f"{n_tree} states x {b} B per query ({'fp32' if b == 28 else 'fp64'} SoA rows)",
                         "note": note or ""}}


def single_query_large(torch, dev, reps, n=10_000_000):
    """The same one-query scan over a 10^7-state SE(3) store (280 MB of fp32 rows, larger than
    the 256 MB Infinity Cache): the HBM-bound case of SURVEY M2(i)."""
    from ompl_amd import NearestNeighborsGPU, workloads as W
    from ompl_amd.spaces import SE3StateSpace

    nn = NearestNeighborsGPU(SE3StateSpace(), dev.index or 0)
    nn.set_stream(torch.cuda.current_stream(dev).cuda_stream)
    nn.add(W.uniform_se3(np.random.default_rng(1234), n))
    r = single_query_scan(torch, nn, dev, reps, n, "10^7 states: 280 MB of fp32 rows, above the 256 MB Infinity "
                                                   "Cache, so every scan streams from HBM")
    del nn
    return r


def _timed(torch, stream, fn, reps):
    """mean ms of fn() over reps, HIP events on the library's stream"""
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    fn()
    torch.cuda.synchronize()
    ev[0].record(stream)
    for _ in range(reps):
        fn()
    ev[1].record(stream)
    torch.cuda.synchronize()
    return ev[0].elapsed_time(ev[1]) / reps


def sphere_variant(torch, run, local, reps=5):
    """SURVEY §8d M2's 32-sphere field (r = 0.1, centres from RNG(7)) on the same (nearest,
    steered) edges as the timed step, for realistic early-exit rates: the hypercube passage of
    the headline rejects most motions at their first isValid(s2)."""
    from ompl_amd import DiscreteMotionValidatorGPU
    from ompl_amd import workloads as W
    from ompl_amd.checkers import SpheresChecker

    c, r = W.sphere_field(32, 0.1, 7)
    mv = DiscreteMotionValidatorGPU(run.sp, SpheresChecker(c, r), local)
    mv.set_stream(run.stream.cuda_stream)
    valid = torch.empty(run.m, dtype=torch.uint8, device=run.dev)
    c0 = mv.stateChecks()
    ms = _timed(torch, run.stream, lambda: mv.check_device(run.s_from.data_ptr(), run.s_to.data_ptr(), run.m,
                                                           valid.data_ptr()), reps)
    checks = (mv.stateChecks() - c0) / (reps + 1)
    return {"checker": "32 spheres r=0.1, centres RNG(7)", "motion_checks_per_s": run.m / (ms * 1e-3),
            "ms_per_batch": ms, "edges": run.m, "valid_fraction": float(valid.float().mean().item()),
            "isValid_calls_per_edge": checks / run.m}


def rrt_star_knn(torch, run, n_tree, nq=1000, reps=3):
    """M2(iii): RRT*'s neighbourhood query k = ceil(k_rrt ln(n+1)) = 6,169 at n = 10^6
    (RRTstar.cpp:603-618, :1147-1159) for a batch of the run's samples, through the large-k path
    (knn_large.hip: fp32 histogram threshold + exact fp64 candidates + segmented sort)."""
    from ompl_amd import workloads as W

    k = W.rrt_star_k(n_tree, 6)
    nq = min(nq, run.nq)
    ids = torch.empty((nq, k), dtype=torch.int32, device=run.dev)
    dd = torch.empty((nq, k), dtype=torch.float64, device=run.dev)
    q = run.queries.data_ptr()
    run.nn.profile(True)  # HIP events around sel_fill_kernel (the first query block's launch)
    ms0, n0, _ = run.nn.kernel_time()
    ms = _timed(torch, run.stream, lambda: run.nn.knn_device(q, nq, k, ids.data_ptr(), dd.data_ptr()), reps)
    ms1, n1, name = run.nn.kernel_time()
    run.nn.profile(False)
    if n1 == n0:
        raise RuntimeError("large-k path recorded no kernel time")
    kern_ms = (ms1 - ms0) / (n1 - n0)
    assert bool((dd[:, 1:] >= dd[:, :-1]).all().item()), "large-k lists must be sorted"
    return {"k": k, "queries": nq, "queries_per_s": nq / (ms * 1e-3), "ms_per_batch": ms, "kernel": name,
            "kernel_ms": kern_ms, "pairs_per_batch": float(nq) * n_tree}


def _rrtstar_tree(torch, sp, mv, n_tree, local, batch=10_000):
    """configs[2]'s starting tree: the first n_tree valid states of the reference stream
    (RNG::setSeed(42), a tree sampler; UniformValidStateSampler order) joined in batches of `batch`,
    each state's parent its nearest state among the earlier batches (the first batch hangs off
    state 0), incCost = that distance, cost = the path length from state 0 — an RRT-like tree built
    on the device (batched nearest), so that the RRT* steps rewire a realistic tree."""
    from ompl_amd import NearestNeighborsGPU
    from ompl_amd import sampling as S
    from ompl_amd import workloads as W

    S.set_seed(42)
    ts, qs = S.StateSampler(sp), S.StateSampler(sp)
    tree, _ = W.reference_valid_states(sp, n_tree, mv.isValid, sampler=ts, chunk=4_000_000)
    parent = np.zeros(n_tree, np.int64)
    inc = np.zeros(n_tree)
    cost = np.zeros(n_tree)
    parent[0] = -1
    first = tree[1:batch]
    inc[1:batch] = mv.distance(np.repeat(tree[:1], len(first), axis=0), first)
    cost[1:batch] = inc[1:batch]
    nn = NearestNeighborsGPU(sp, local)
    nn.add(tree[:batch])
    for b in range(batch, n_tree, batch):
        x = tree[b:b + batch]
        ids, d, _ = nn.nearestKBatch(x, 1)
        p = ids[:, 0].astype(np.int64)
        parent[b:b + len(x)] = p
        inc[b:b + len(x)] = d[:, 0]
        cost[b:b + len(x)] = cost[p] + d[:, 0]
        nn.add(x)
    nn.close()
    return tree, parent, inc, cost, qs


def rrt_star_workload(torch, dev, local, stream, steps, warmup, ns=10_000, n_tree=1_000_000, cpu_seconds=8.0,
                      cpu=True):
    """configs[2], RRT* (SURVEY §8f row 1): SE(3) [0,1]^3, the HypercubeBenchmark passage on the
    translation (edgeWidth 0.1, resolution 0.01), a 10^6-state tree (_rrtstar_tree), then per step a
    batch of ns samples through RRTstar::solve's iteration (RRTstar.cpp:247-542, defaults:
    k-nearest, delayCC): the device batch (nearest, steer, checkMotion, neighbourhoods
    k = ceil(446.5 ln(size + 1)) ~ 6,169, both motion bits of every neighbour — exact for the
    sequential loop) and the host cost logic (parent in cost order, rewiring, child costs;
    ompl_gpu_rrtstar_commit, native), the latter overlapping the next batch's device work.  value = RRT* iterations (samples processed) per second, device + host.
    cpu_baseline: the oracle's sequential RRT* loop (oracle/rrtstar.cpp) over the GNAT restatement
    on the same tree and samples, one thread (the reference's RRT* is single-threaded)."""
    from ompl_amd import DiscreteMotionValidatorGPU
    from ompl_amd.checkers import HypercubeChecker
    from ompl_amd.rrtstar import RRTstarGPU
    from ompl_amd.spaces import SE3StateSpace

    # at least 5 warm batches: the first commits pay the host side's first-touch allocations and
    # the cost-logic threads' start (a 2-batch warmup left them in the timed steps)
    warmup = max(warmup, 5)
    t_setup = time.perf_counter()
    sp, ck = SE3StateSpace(0.0, 1.0), HypercubeChecker(3, 0.1)
    maxd = 0.2 * sp.getMaximumExtent()
    mv0 = DiscreteMotionValidatorGPU(sp, ck, local)
    tree, parent, inc, cost, qs = _rrtstar_tree(torch, sp, mv0, n_tree, local)
    mv0.close()
    samples_h = qs.sample_uniform(ns * (warmup + steps))
    samples = torch.from_numpy(samples_h).to(dev)
    planner = RRTstarGPU(sp, ck, maxd, local, stream.cuda_stream)
    planner.add_tree(tree, parent, inc, cost)
    near = torch.empty(ns, dtype=torch.int32, device=dev)
    added = torch.empty(ns, dtype=torch.int32, device=dev)
    incs = torch.empty(ns, dtype=torch.float64, device=dev)
    setup_s = time.perf_counter() - t_setup
    from concurrent.futures import ThreadPoolExecutor

    pool = ThreadPoolExecutor(1)
    host_s = [0.0, 0.0]  # stage (device -> host copies), commit (the cost logic)

    def commit():
        t0 = time.perf_counter()
        planner.commit(ns)
        host_s[1] += time.perf_counter() - t0

    def device_step(i, ev=None):
        """the device batch, then its results staged on the host; the previous batch's cost logic
        runs meanwhile on the pool thread (it needs none of this batch's results)"""
        if ev:
            ev[0].record(stream)
        res = planner.batch_device(samples[i * ns].data_ptr(), ns, near.data_ptr(), added.data_ptr(), incs.data_ptr())
        if ev:
            ev[1].record(stream)
        t0 = time.perf_counter()
        planner.stage(ns, near.data_ptr(), added.data_ptr(), incs.data_ptr(), res)
        host_s[0] += time.perf_counter() - t0
        return res

    def run_steps(first, count, evs=None):
        rounds, pending = [], None
        for j in range(count):
            res = device_step(first + j, evs[j] if evs else None)
            rounds.append(int(res.rounds))
            if pending is not None:
                pending.result()
            pending = pool.submit(commit)
        if pending is not None:
            pending.result()
        return rounds

    run_steps(0, warmup)
    torch.cuda.synchronize(dev)
    planner.nn.profile(True)
    planner.nn.kernel_time()
    k0 = planner.nn.kernel_time()
    ev = [[torch.cuda.Event(enable_timing=True) for _ in range(2)] for _ in range(steps)]
    st0 = planner.stats
    a0, e0 = st0["added"], st0["neighbours"]
    host_s[0] = host_s[1] = 0.0
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    rounds = run_steps(warmup, steps, ev)  # every batch committed before the clock stops
    torch.cuda.synchronize(dev)
    elapsed = time.perf_counter() - t0
    pool.shutdown()
    k1 = planner.nn.kernel_time()
    planner.nn.profile(False)
    dev_ms = float(np.mean([e[0].elapsed_time(e[1]) for e in ev]))
    n_added = planner.stats["added"] - a0
    E = planner.stats["neighbours"] - e0
    units = steps * 2 * ns + n_added + 2 * E  # nearest + steer checkMotion per sample, kNN per added, 2 bits per entry
    kern_ms = (k1[0] - k0[0]) / max(k1[1] - k0[1], 1)
    n_mid = n_tree + planner.stats["added"] - n_added / 2
    pairs = (n_added / steps) * n_mid  # the neighbourhood kNN's fill pass: every (added state, stored state) pair
    achieved = pairs * F_SE3 / (kern_ms * 1e-3) / 1e12
    traffic = pmc_traffic("rrt_star", k1[2])
    line = {
        "metric": "RRT* iterations/sec (nearest + steer + checkMotion + neighbourhood + motion bits + cost logic), "
                  "SE(3) 10^6-state tree",
        "value": steps * ns / elapsed, "unit": "RRT* iterations/s", "steps": steps, "warmup": warmup,
        "ms_per_step": elapsed * 1e3 / steps, "higher_is_better": True, "dtype": "f32 screen + f64 exact",
        "config": {"workload": "configs[2]: SE(3) RRT* (k-nearest, delayCC), HypercubeBenchmark passage on the "
                               "translation (edgeWidth 0.1), resolution 0.01", "tree_states": n_tree,
                   "samples_per_step": ns, "k_rrt": planner.k_rrt, "max_distance": maxd,
                   "tree": "the first 10^6 valid states of the reference stream, parents = nearest among earlier "
                           "batches of 10^4 (an RRT-like tree), costs = path lengths"},
        "nn_queries_plus_motion_checks_per_s": units / elapsed,
        # the device batch alone (HIP events around ompl_gpu_rrtstar_batch_device): the rate without the host
        # cost logic (planner control logic) that bounds `value`
        "device_only_value": ns / (dev_ms * 1e-3),
        "phase_ms": {"device_batch": dev_ms, "stage_to_host": host_s[0] * 1e3 / steps,
                     "host_cost_logic": host_s[1] * 1e3 / steps,
                     "note": "the cost logic of batch i (native, ompl_gpu_rrtstar_commit) overlaps the device batch "
                             "i + 1 on a host thread"},
        "added_per_step": n_added / steps, "neighbourhood_entries_per_step": E / steps,
        "fixed_point_rounds": rounds,
        "per_step": {k: (planner.stats[k] - st0[k]) / steps for k in ("rewires", "checks_used", "child_cost_updates")},
        "setup_s": setup_s,
        "roofline": {"bound": "valu", "achieved": achieved, "peak": PEAK_TFLOPS["f32"], "unit": "TFLOP/s",
                     "frac": achieved / PEAK_TFLOPS["f32"], "traffic": traffic["bytes"] if traffic else None,
                     "traffic_source": traffic["source"] if traffic else None, "kernel": k1[2], "kernel_ms": kern_ms,
                     "algorithmic": f"the neighbourhood kNN's fp32 fill pass ({k1[2]}): every (added state, stored "
                                    f"state) pair, {pairs:.4g} per step x {F_SE3} flop"},
    }
    if cpu:
        sys.path.insert(0, os.path.join(ROOT, "oracle"))
        import pyoracle as O

        t1 = time.perf_counter()
        ref = O.rrtstar(sp, ck, tree, parent, inc, cost, samples_h[warmup * ns:(warmup + 1) * ns], maxd,
                        planner.k_rrt, use_gnat=True, time_budget_s=cpu_seconds)
        line["cpu_baseline"] = {
            "value": ref["processed"] / ref["loop_s"], "unit": "RRT* iterations/s", "cores": 1, "kind": "port",
            "sample": (f"the oracle's sequential RRT* loop (oracle/rrtstar.cpp) over the GNAT restatement, same tree "
                       f"and the first timed step's samples: {ref['processed']} iterations ({ref['n_added']} added, "
                       f"{ref['rewires']} rewires, {ref['checks']} checkMotion calls) in {ref['loop_s']:.2f} s on one "
                       f"thread (the reference's RRT* is single-threaded); GNAT build excluded"),
            "wall_s": time.perf_counter() - t1}
    planner.close()
    return line


def index_maintenance(torch, run, local, batches=10, batch=100, nq=1000):
    """The culled index kept current on the device: a full k-d build of a fresh
    structure over the tree, then a BIT*-style loop — add a batch of new samples (host upload,
    ImplicitGraph.cpp:682-692 addToSamples), place them in the index's tail, answer a batch of
    queries — timed with HIP events on the library's stream."""
    from ompl_amd import NearestNeighborsGPU
    from ompl_amd import sampling as S

    nn = NearestNeighborsGPU(run.sp, local)
    nn.add(run.tree)
    nn.set_stream(run.stream.cuda_stream)
    torch.cuda.synchronize()
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    ev[0].record(run.stream)
    nn.build_index()
    ev[1].record(run.stream)
    torch.cuda.synchronize()
    build_ms = ev[0].elapsed_time(ev[1])
    new = S.StateSampler(run.sp).sample_uniform(batches * batch)
    ids = torch.empty((nq, run.k), dtype=torch.int32, device=run.dev)
    dd = torch.empty((nq, run.k), dtype=torch.float64, device=run.dev)
    q = run.queries.data_ptr()
    t_app = t_q = 0.0
    for b in range(batches):
        nn.add(new[b * batch:(b + 1) * batch])
        ev[0].record(run.stream)
        nn.build_index()
        ev[1].record(run.stream)
        nn.knn_device(q, nq, run.k, ids.data_ptr(), dd.data_ptr())
        e2 = torch.cuda.Event(enable_timing=True)
        e2.record(run.stream)
        torch.cuda.synchronize()
        t_app += ev[0].elapsed_time(ev[1])
        t_q += ev[1].elapsed_time(e2)
    builds, appends = nn.index_stats()
    return {"states": len(run.tree), "full_build_ms": build_ms, "append_ms_per_batch": t_app / batches,
            "batch_states": batch, "query_ms_per_batch": t_q / batches, "queries_per_batch": nq,
            "builds": builds, "appends": appends,
            "note": ("device k-d build: global levels as median partitions (histogram, median bin, stable scatter of "
                     "whole rows), the deep levels in LDS; appends place new states in a Morton-ordered tail")}


def rrt_device(torch, nn, mv, sp, dev, iters):
    """The RRT loop itself (RRT.cpp:128-192 without the goal test), `iters` dependent iterations
    queued on the device with no host round trip (ompl_gpu_rrt_grow_device).  Grows the tree,
    so it runs after every other measurement."""
    from ompl_amd import workloads as W

    s = torch.from_numpy(W.uniform_se3(np.random.default_rng(98), iters)).to(dev)
    near = torch.empty(iters, dtype=torch.int32, device=dev)
    added = torch.empty(iters, dtype=torch.int32, device=dev)
    maxd = 0.2 * sp.getMaximumExtent()
    nn.rrt_grow_device(mv, s.data_ptr(), 8, maxd, near.data_ptr(), added.data_ptr())  # warm
    torch.cuda.synchronize(dev)
    n0 = nn.size()
    t0 = time.perf_counter()
    nn.rrt_grow_device(mv, s.data_ptr(), iters, maxd, near.data_ptr(), added.data_ptr())
    wall = time.perf_counter() - t0
    return {"iterations_per_s": iters / wall, "iterations": iters, "states_added": nn.size() - n0,
            "semantics": "nearest + steer + checkMotion + add per iteration, each iteration seeing the previous ones"}


class Runner:
    """One workload: builds the inputs, the step, and the roofline of its dominant kernel."""

    def __init__(self, args, torch, dev, local, rank, stream, dist=None):
        from ompl_amd import DiscreteMotionValidatorGPU, NearestNeighborsGPU
        from ompl_amd import workloads as W
        from ompl_amd.checkers import HypercubeChecker, KinematicChainChecker, SpheresChecker
        from ompl_amd.spaces import KinematicChainSpace, RealVectorStateSpace, SE3StateSpace

        self.args, self.torch, self.dev = args, torch, dev
        wl, nq, k = args.workload, args.queries, args.k
        self.radius = None
        self.tree_mode = args.partition == "tree"
        world = int(os.environ.get("WORLD_SIZE", "1"))
        # strong scaling (replicated tree): a fixed global batch of args.queries samples, rank r
        # answering its contiguous share; weak: args.queries per rank
        self.strong = getattr(args, "scaling", "weak") == "strong" and not self.tree_mode
        if self.strong:
            if wl not in ("cfg3", "cfg2"):
                raise SystemExit("bench.py: --scaling strong is implemented for cfg3 / cfg2")
            self.global_q = nq
            nq = (nq + world - 1) // world
        if wl == "cfg3":
            self.sp, self.ck = SE3StateSpace(0.0, 1.0), HypercubeChecker(3, 0.1)
        elif wl == "cfg2":
            self.sp, self.ck = RealVectorStateSpace(6), HypercubeChecker(6, 0.1)
        elif wl == "cfg4":
            self.sp = KinematicChainSpace(12, 1.0 / 12)                   # KinematicChainBenchmark.cpp:48-49
            self.ck = KinematicChainChecker(W.horn_environment(12, math.log(12.0) / 12.0))
            self.kc = math.e + math.e / 12.0                              # KStarStrategy (ConnectionStrategy.h:141)
            last = args.tree + nq * (args.warmup + args.steps) * world
            self.k = int(math.ceil(self.kc * math.log(last)))           # k_cap: the largest k_i of the run
        else:
            self.sp = SE3StateSpace(0.0, 1.0)
            c, r = W.sphere_field(32, 0.1, 7)
            self.ck = SpheresChecker(c, r)
            self.radius = W.bitstar_radius(args.tree, 6, math.pi ** 2)
        if wl in ("cfg3", "cfg2"):
            self.k = k
        elif wl == "cfg5":
            # BIT* kNN mode: k = ceil(1.1 (e + e/d) ln n) (bitstar/src/ImplicitGraph.cpp:313-316, 1383-1387)
            self.k = int(math.ceil(1.1 * (math.e + math.e / 6.0) * math.log(args.tree))) if args.bitstar_knn else 0
        self.mv = DiscreteMotionValidatorGPU(self.sp, self.ck, local)
        if wl in ("cfg3", "cfg2"):
            # tree mode: one global batch of samples for every rank (the rank-0 slice of the stream)
            tree, qa = shared_inputs(wl, self.sp, args.tree, nq * world, None, dist, dev)
            r0 = 0 if self.tree_mode else rank
            hi = min((r0 + 1) * nq, self.global_q) if self.strong else (r0 + 1) * nq
            self.tree, q = tree, np.ascontiguousarray(qa[r0 * nq:hi])
            nq = len(q)
        elif wl == "cfg5":  # sample sets hold valid states (ImplicitGraph.cpp:981)
            self.tree, qa = shared_inputs("cfg5", self.sp, args.tree, nq * world, self.mv.isValid, dist, dev)
            r0 = 0 if self.tree_mode else rank  # tree mode: every shard answers the same vertices
            q = np.ascontiguousarray(qa[r0 * nq:(r0 + 1) * nq])
        else:  # cfg4: roadmap + the milestones of every step: valid states (PRM.cpp:356-378)
            # one causal batch per step holds world * nq milestones of the query stream; every rank
            # inserts the whole batch (replicas stay identical) and computes the neighbours and edges
            # of its slice [rank * nq, (rank + 1) * nq) — no collective in the data path
            nsteps = args.warmup + args.steps
            self.tree, q = shared_inputs("cfg4", self.sp, args.tree, nq * world * nsteps, self.mv.isValid, dist, dev)
            self.milestones = [q[i * nq * world:(i + 1) * nq * world] for i in range(nsteps)]
            self.slice = (rank * nq, (rank + 1) * nq)
            self.step_i = 0
            self.n_mid = args.tree + nq * world * (args.warmup + args.steps / 2.0)  # mean store size, timed steps
        self.q_host = q
        self.nq = nq
        self.queries = torch.from_numpy(q).to(dev)
        self.nn = NearestNeighborsGPU(self.sp, local)
        self.nn.set_exact(args.exact)
        if self.tree_mode:  # this rank's contiguous slice of the ids (ompl_amd/shard.py)
            from ompl_amd.shard import shard_bounds

            self.world = int(os.environ.get("WORLD_SIZE", "1"))
            self.rank = rank
            self.lo, self.hi = shard_bounds(len(self.tree), rank, self.world)
            self.nn.add(self.tree[self.lo:self.hi])
            self.owned = torch.zeros((), dtype=torch.int64, device=dev)
        else:
            self.nn.add(self.tree)
        self.nn.set_stream(stream.cuda_stream)
        self.mv.set_stream(stream.cuda_stream)
        dim = self.sp.dim
        if wl in ("cfg3", "cfg2", "cfg4") or self.k:
            self.ids = torch.empty((nq, self.k), dtype=torch.int32, device=dev)
            self.dd = torch.empty((nq, self.k), dtype=torch.float64, device=dev)
        if wl == "cfg4":
            self.cnt = torch.empty(nq, dtype=torch.int32, device=dev)
            self.evalid = torch.empty((nq, self.k), dtype=torch.uint8, device=dev)
        m = nq * self.k if (wl == "cfg4" or (wl == "cfg5" and self.k)) else nq
        if wl == "cfg5" and not self.k:
            self.off = torch.empty(nq + 1, dtype=torch.int64, device=dev)
            m = self.nn.radius_device(self.queries.data_ptr(), nq, self.radius, self.off.data_ptr(), 0, 0, 0)
            self.cap = m
            self.ids = torch.empty(max(m, 1), dtype=torch.int32, device=dev)
            self.dd = torch.empty(max(m, 1), dtype=torch.float64, device=dev)
        self.m = m
        # endpoint rows: the steered motions (cfg3 / cfg2) and the tree-sharded cfg5 edges; the
        # replicated cfg5 step checks its edges in place (ompl_gpu_mv_check_edges_device)
        rows = 1 if (wl == "cfg5" and not self.tree_mode) else max(m, 1)
        self.s_from = torch.empty((rows, dim), dtype=torch.float64, device=dev)
        self.s_to = torch.empty_like(self.s_from)
        self.valid = torch.empty(max(m, 1), dtype=torch.uint8, device=dev)
        self.maxd = 0.2 * self.sp.getMaximumExtent()                    # RRT range default (SelfConfig.cpp:98)
        # steps in flight: the batches of cfg3 / cfg2 / cfg5's kNN mode are independent (a step adds
        # nothing to the tree), so step i runs on lane i % L — its own stream, NN and validator
        # handles over the same tree, its own outputs — and step i + 1's walk starts on the CUs that
        # step i's walk tail (its last groups) and the small kernels after it leave idle.  cfg4's
        # causal PRM* batches and the radius mode (a host read of the result size per call) keep one.
        self.stream = stream
        keys = ("nn", "mv", "stream", "ids", "dd", "s_from", "s_to", "valid") + (("off",) if hasattr(self, "off") else ())
        self.lanes = [{key: getattr(self, key) for key in keys}]
        nl = max(1, getattr(args, "lanes", 1))
        if self.tree_mode or wl not in ("cfg3", "cfg2", "cfg5"):
            nl = 1
        # the radius mode reads each call's result size on the host: its lanes get host threads
        self.threaded = nl > 1 and wl == "cfg5" and not self.k
        for _ in range(nl - 1):
            ln = {"stream": torch.cuda.Stream(dev), "nn": NearestNeighborsGPU(self.sp, local),
                  "mv": DiscreteMotionValidatorGPU(self.sp, self.ck, local)}
            ln["nn"].set_exact(args.exact)
            ln["nn"].add(self.tree)
            ln["nn"].set_stream(ln["stream"].cuda_stream)
            ln["mv"].set_stream(ln["stream"].cuda_stream)
            for key in ("ids", "dd", "s_from", "s_to", "valid") + (("off",) if "off" in self.lanes[0] else ()):
                ln[key] = torch.empty_like(getattr(self, key))
            self.lanes.append(ln)
        self.si = 0

    def use_lane(self, i):
        for key, v in self.lanes[i].items():
            setattr(self, key, v)

    def next_lane(self):
        self.use_lane(self.si % len(self.lanes))
        self.si += 1

    def step(self, e=None):
        self.next_lane()
        a, nn, mv, q = self.args, self.nn, self.mv, self.queries.data_ptr()
        if a.workload == "cfg4":  # one causal PRM* batch (synchronous: its kNN, scan, edges, insert)
            if e:
                e[0].record(self.stream)
            batch = self.milestones[self.step_i]
            self.step_i += 1
            self.m = nn.prm_add_milestones_device(mv, batch, self.kc, self.k, self.ids.data_ptr(),
                                                  self.cnt.data_ptr(), self.evalid.data_ptr(), *self.slice)
            if e:
                for j in (1, 2, 3):
                    e[j].record(self.stream)
            return
        if self.tree_mode:
            (self.step_tree_radius if a.workload == "cfg5" else self.step_tree)(e)
            return
        self.m = self.step_on(self.lanes[(self.si - 1) % len(self.lanes)], e)

    def step_on(self, L, e=None):
        """one replicated step of cfg3 / cfg2 / cfg5 on lane L (its handles, stream and outputs);
        returns the step's edge count.  Touches no Runner state: lanes may run on their own host
        threads (threaded_lanes)."""
        a, nn, mv, q, st = self.args, L["nn"], L["mv"], self.queries.data_ptr(), L["stream"]
        if e:
            e[0].record(st)
        m = self.m
        if a.workload == "cfg5" and not self.k:
            m = nn.radius_device(q, self.nq, self.radius, L["off"].data_ptr(), L["ids"].data_ptr(), L["dd"].data_ptr(),
                                 self.cap)
        else:
            nn.knn_device(q, self.nq, self.k, L["ids"].data_ptr(), L["dd"].data_ptr())
        if e:
            e[1].record(st)
        if a.workload in ("cfg3", "cfg2"):   # RRT extend: nearest -> steer (RRT.cpp:137-146)
            nn.steer_device(q, self.nq, L["ids"].data_ptr(), self.k, self.maxd, L["s_from"].data_ptr(),
                            L["s_to"].data_ptr())
        # BIT* (cfg5, both modes): checkMotion(vertex, sample) (BITstar.cpp:815) over the neighbour
        # result's edges read in place (ompl_gpu_mv_check_edges_device: no endpoint rows written)
        if e:
            e[2].record(st)
        if a.workload == "cfg5":
            mv.check_edges_device(nn, q, self.nq, None if self.k else L["off"].data_ptr(), L["ids"].data_ptr(),
                                  self.k, m, True, L["valid"].data_ptr())
        elif a.workload != "cfg2":
            mv.check_device(L["s_from"].data_ptr(), L["s_to"].data_ptr(), m, L["valid"].data_ptr())
        if e:
            e[3].record(st)
        return m

    def run_threaded(self, steps, ev):
        """the timed steps with one host thread per lane (lane j takes steps j, j + L, ...): a lane
        whose call waits on the host (nearestR reads its result size) leaves the other lanes' host
        threads free to keep their streams fed.  Returns the units issued."""
        import torch
        from concurrent.futures import ThreadPoolExecutor

        nl = len(self.lanes)

        def lane(j):
            torch.cuda.set_device(self.dev)
            for s in range(j, steps, nl):
                self.step_on(self.lanes[j], ev[s] if ev else None)
            return len(range(j, steps, nl))

        with ThreadPoolExecutor(nl) as ex:
            n = sum(ex.map(lane, range(nl)))
        return n * self.units_per_step()

    def step_tree_radius(self, e=None):
        """Tree-sharded BIT* batch (cfg5 radius): every rank answers every vertex's nearestR on its
        slice of the samples; the per-shard CSR results (global ids) are exchanged — a count
        all_gather, then padded id / distance all_gathers over RCCL — and merged by the library's
        kernel (ompl_gpu_csr_merge_device), so every rank holds each vertex's whole neighbourhood
        (NearestNeighborsGNAT.h:236-245); each edge (vertex, sample) is checked by the rank that
        stores the sample (BITstar.cpp:815), from its own rows, so no state rows travel."""
        import torch

        from ompl_amd.shard import allgather_radius, merge_csr_device

        nn, mv, q = self.nn, self.mv, self.queries
        with torch.cuda.stream(self.stream):
            if e:
                e[0].record(self.stream)
            self.m = nn.radius_device(q.data_ptr(), self.nq, self.radius, self.off.data_ptr(), self.ids.data_ptr(),
                                      self.dd.data_ptr(), self.cap)
            gid = self.ids[: self.m].to(torch.int64) + self.lo
            if self.world > 1:
                self._merged = allgather_radius(self.off, gid, self.dd[: self.m])
            else:
                self._merged = merge_csr_device(self.off[None], gid[None].to(torch.int32), self.dd[None, : self.m],
                                                self.m, stream=self.stream.cuda_stream)
            if e:
                e[1].record(self.stream)
            nn.edges_device(q.data_ptr(), self.nq, self.off.data_ptr(), self.ids.data_ptr(), 0, self.m, True,
                            self.s_from.data_ptr(), self.s_to.data_ptr())
            if e:
                e[2].record(self.stream)
            mv.check_device(self.s_from.data_ptr(), self.s_to.data_ptr(), self.m, self.valid.data_ptr())
            if e:
                e[3].record(self.stream)

    def step_tree(self, e=None):
        """Tree-sharded step: every rank answers the whole batch on its shard, the per-shard top-k
        lists (global ids) are exchanged with an all_gather over RCCL and merged by the library's
        kernel (ompl_gpu_knn_merge_device); the rank that owns a sample's nearest state steers and
        checks that sample's motion on its own store (RRT.cpp:137-148), so no state rows travel."""
        import torch

        from ompl_amd.shard import allgather_merge, merge_topk_device

        nn, mv, q = self.nn, self.mv, self.queries
        with torch.cuda.stream(self.stream):
            if e:
                e[0].record(self.stream)
            nn.knn_device(q.data_ptr(), self.nq, self.k, self.ids.data_ptr(), self.dd.data_ptr())
            if e:
                e[1].record(self.stream)
            gid = torch.where(self.ids >= 0, self.ids + self.lo, -1)
            if self.world > 1:
                md, mi = allgather_merge(self.dd, gid, self.k)
            else:
                md, mi = merge_topk_device(self.dd[None], gid[None].to(torch.int32), self.k,
                                           stream=self.stream.cuda_stream)
            near = mi[:, 0].to(torch.int64)
            # no host round trip: every sample is steered, the ones whose nearest state another
            # rank owns with a missing id (from = to = the sample: a zero-length motion, one
            # isValid) — the owned count stays on the device until the timed loop is over
            mine = (near >= self.lo) & (near < self.hi)
            nl = torch.where(mine, near - self.lo, -1).to(torch.int32)
            self.owned = self.owned + mine.sum()
            self.last_owned = mine.sum()
            self._keep = nl
            nn.steer_device(q.data_ptr(), self.nq, nl.data_ptr(), 1, self.maxd, self.s_from.data_ptr(),
                            self.s_to.data_ptr())
            if e:
                e[2].record(self.stream)
            mv.check_device(self.s_from.data_ptr(), self.s_to.data_ptr(), self.nq, self.valid.data_ptr())
            if e:
                e[3].record(self.stream)

    def units_per_step(self):
        """NN queries + motion checks one step issues on this rank (tree mode: the batch's queries
        once, on rank 0; the owned motion checks are summed on the device, see owned_units)."""
        if self.tree_mode:  # cfg5: each edge is checked by the rank storing its sample
            return (self.nq if self.rank == 0 else 0) + (self.m if self.args.workload == "cfg5" else 0)
        if self.args.workload == "cfg2":
            return self.nq
        return self.nq + self.m

    def metric(self):
        wl = self.args.workload
        if wl == "cfg2":
            return "NN queries/sec, R^6 10^5 states, batched nearestK(k=10)", "NN queries/s"
        if wl == "cfg4":
            return "NN queries/sec + motion checks/sec, PRM* KinematicChain R^12, 10^6-vertex roadmap", UNIT
        if wl == "cfg5":
            mode = f"kNN (k={self.k})" if self.k else "radius"
            return f"NN queries/sec + motion checks/sec, BIT* SE(3) {mode} batch, 10^7 samples", UNIT
        return METRIC, UNIT

    def config(self, world):
        a = self.args
        base = {"tree_states": a.tree, "queries_per_gpu": self.nq,
                "parallelism": f"queries sharded over {world} GPU(s), tree replicated",
                "steps_in_flight": len(self.lanes)}
        if self.strong:
            base.update(queries_per_gpu=None, queries_per_step=self.global_q, queries_this_rank=self.nq,
                        parallelism=(f"a fixed global batch of {self.global_q} samples split over {world} GPU(s) "
                                     f"(about {self.global_q // world} each), tree replicated, no collective in the "
                                     f"data path"))
        if self.tree_mode and a.workload == "cfg5":
            base.update(queries_per_gpu=None, queries_per_step=self.nq, partition="tree",
                        parallelism=(f"sample set sharded over {world} GPU(s) ({a.tree // world} samples each), every "
                                     f"vertex's nearestR answered on every shard, the per-shard CSR results exchanged "
                                     f"(count all_gather + padded id / distance all_gathers over RCCL) and merged on "
                                     f"the device; each edge checked by the rank storing its sample"),
                        exchange_bytes_per_rank=(self.nq + 1) * 8 + self.m * 12)
        elif self.tree_mode:
            base.update(queries_per_gpu=None, queries_per_step=self.nq, partition="tree",
                        parallelism=(f"tree sharded over {world} GPU(s) ({a.tree // world} states each), every sample "
                                     f"answered on every shard, per-shard top-{self.k} lists all_gathered (RCCL) and "
                                     f"merged on the device; the owner of each nearest state steers + checks it"),
                        exchange_bytes_per_rank=self.nq * self.k * 12)
        if a.workload == "cfg3":
            base.update(workload="configs[2]: SE(3) RRT*-style batch — nearestK(k=10) + steer + checkMotion "
                                 "(HypercubeBenchmark predicate on translation, edgeWidth 0.1, resolution 0.01)",
                        k=self.k, state_space="SE3 [0,1]^3")
        elif a.workload == "cfg2":
            base.update(workload="configs[1]: R^6 RealVectorStateSpace, batched nearestK(k=10)", k=self.k,
                        state_space="R^6 [0,1]^6")
        elif a.workload == "cfg4":
            base.update(workload="configs[3]: PRM* roadmap construction, causal batches, KinematicChain R^12 (horn "
                                 "environment) — milestone i: nearestK(k_i = ceil((e + e/12) ln(i+1))) over every "
                                 "earlier vertex + checkMotion(neighbour, milestone) per edge + insert",
                        k_max=self.k, state_space="KinematicChain 12 links, linkLength 1/12",
                        edges_last_step=self.m,
                        note=("roadmap vertices and milestones are valid states (rejection); the batch's "
                              "milestones are uploaded from the host inside each step (~1 MB, <0.1% of the step)"))
        elif self.k:
            base.update(workload="configs[4]: BIT* batch on SE(3), kNN mode (useKNearest_ default, "
                                 "bitstar/ImplicitGraph.h:463) — nearestK(k = ceil(1.1 (e + e/6) ln n)) + "
                                 "checkMotion(vertex, sample) per edge, 32 spheres r=0.1",
                        k=self.k, state_space="SE3 [0,1]^3", edges_per_step=self.m,
                        note="samples and vertices are valid states (rejection)")
        else:
            base.update(workload="configs[4]: BIT* batch on SE(3) — nearestR(r = 1.1 r_RGG (ln n / n)^(1/6)) + "
                                 "checkMotion(vertex, sample) per edge, 32 spheres r=0.1",
                        radius=self.radius, state_space="SE3 [0,1]^3", edges_per_step=self.m,
                        note="samples and vertices are valid states (rejection)")
        return base

    def roofline(self, kern_ms, kern_name, before, after, launches):
        wl, nq = self.args.workload, self.nq
        n = getattr(self, "n_mid", self.args.tree)
        traffic = pmc_traffic("cfg5k" if wl == "cfg5" and self.k else wl, kern_name)
        if kern_name == "radius32_group_kernel":
            pairs = (after["rq"] - before["rq"]) * 64 / launches
            flop, dt, frac_of = F_SE3, "f32", f"{pairs / (float(nq) * n):.4%}"
            what = (f"{pairs:.4g} (query, state) fp32 distance evaluations per launch x {F_SE3} flop (SURVEY §8d); "
                    f"the culled radius walk scanned {frac_of} of the {nq} x {n} pairs")
        elif kern_name == "knn32_group_kernel":
            pairs = (after["kq"] - before["kq"]) * 64 / launches
            flop = F_L2_6 if wl == "cfg2" else F_SE3
            dt = "f32"
            what = (f"{pairs:.4g} (query, state) fp32 distance evaluations per launch x {flop} flop (SURVEY §8d); "
                    f"the culled walk scanned {pairs / (float(nq) * n):.4%} of the {nq} x {n} pairs")
        elif kern_name == "knn32_chain_cull_kernel":
            pairs = (after["kq"] - before["kq"]) * 64 / launches
            flop, dt = F_CHAIN, "f32"
            what = (f"{pairs:.4g} (query, state) fp32 chain distances per launch x {F_CHAIN} flop (SURVEY §8d); the "
                    f"culled chain scan evaluated {pairs / (float(nq) * n):.4%} of the {nq} x {n} pairs, each counted "
                    "at the full 84 flop although a wave leaves a pair's remaining links once no lane's partial sum is "
                    "below its threshold (an upper bound of the work done)")
        else:  # brute-force scans (exact fp64 tiled kernel, or the chunked fp32 screen)
            pairs = float(nq) * n
            flop = {"cfg3": F_SE3, "cfg2": F_L2_6, "cfg4": F_CHAIN, "cfg5": F_SE3}[wl]
            dt = "f32" if kern_name.startswith("knn32") else "f64"
            what = f"{nq} x {n} (query, state) pairs per launch x {flop} flop (SURVEY §8d), brute force"
            if kern_name == "knn32_wave_scan_kernel":
                what += ("; every pair counted at the full 84 flop although a wave skips the remaining links once "
                         "no lane's partial sum is below its list threshold (an upper bound of the work done)")
        achieved = pairs * flop / (kern_ms * 1e-3) / 1e12
        out = {"bound": "valu", "achieved": achieved, "peak": PEAK_TFLOPS[dt], "unit": "TFLOP/s",
               "frac": achieved / PEAK_TFLOPS[dt], "traffic": traffic["bytes"] if traffic else None,
               "kernel": kern_name, "kernel_ms": kern_ms,
               "algorithmic": what + f"; {dt} VALU peak (compute-bound on VALU, no MFMA)",
               "brute_force_equivalent_tflops": float(nq) * n * flop / (kern_ms * 1e-3) / 1e12,
               "traffic_source": traffic["source"] if traffic else None}
        if kern_name == "knn32_group_kernel" and wl in ("cfg3", "cfg2") and not self.k > 16:
            # the walk's waves: one per G = 2 queries (knn_fast_impl.h group_queries)
            iss = sq_issue(wl, kern_name, (nq + 1) // 2, kern_ms)
            if iss:
                out["issue"] = iss
        return out

    def close(self):
        """release the library handles (the next workload gets the HBM back)"""
        for ln in self.lanes:
            for h in (ln["nn"], ln["mv"]):
                h.close()

    def counters(self):
        """walk counters summed over the lanes' handles"""
        kq = sum(ln["nn"].cull_stats()[2] for ln in self.lanes)
        rq = sum(ln["nn"].radius_cull_stats()[1] for ln in self.lanes)
        return {"kq": kq, "rq": rq}

    def profile(self, on):
        for ln in self.lanes:
            ln["nn"].profile(on)

    def kernel_time(self):
        """(total ms, launches, name) of the dominant kernel over every lane (HIP events on each
        handle's own stream)"""
        tot, n, name = 0.0, 0, ""
        for ln in self.lanes:
            ms, c, nm = ln["nn"].kernel_time()
            tot, n, name = tot + ms, n + c, nm or name
        return tot, n, name

    def stats(self):
        s = [ln["nn"].stats() for ln in self.lanes]
        return sum(x[0] for x in s), sum(x[1] for x in s)

    def radius_path_stats(self):
        s = [ln["nn"].radius_path_stats() for ln in self.lanes]
        return [sum(x[i] for x in s) for i in range(len(s[0]))]


def spawn_ranks(n):
    """`bench.py --gpus N` without a launcher: start N fresh child processes of this script, one
    per GPU, with RANK / LOCAL_RANK / WORLD_SIZE / MASTER_* set (the same environment
    torch.distributed.run provides).  The parent never imports torch nor touches a GPU; it waits
    for the children and exits with the first failure's code (the others are stopped)."""
    import socket
    import subprocess

    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        port = so.getsockname()[1]
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:], env=env))
    rc = 0
    live = list(procs)
    while live:
        time.sleep(0.2)
        for p in list(live):
            if p.poll() is not None:
                live.remove(p)
                if p.returncode != 0 and rc == 0:
                    rc = p.returncode
                    for q in live:
                        q.terminate()
    sys.exit(rc)


SUB_WORKLOADS = {  # the default line's `workloads` record: every other config, same steps / warmup (cfg4: at most 5 / 2, sub_args)
    # the headline's strong-scaling forms: 10^5 samples in total over the N GPUs on the replicated
    # tree, and the tree sharded over the ranks (every sample answered by every shard, merged)
    "cfg3_strong": {"workload": "cfg3", "scaling": "strong"},
    "cfg3_tree": {"workload": "cfg3", "partition": "tree"},
    "cfg2": {"workload": "cfg2"},
    "cfg4": {"workload": "cfg4"},
    "cfg5": {"workload": "cfg5"},
    "cfg5k": {"workload": "cfg5", "bitstar_knn": True},
}


def sub_args(args, spec):
    """args for one sub-workload: its own defaults (DEFAULTS), the headline's steps / warmup."""
    a = argparse.Namespace(**vars(args))
    a.workload = spec["workload"]
    a.bitstar_knn = spec.get("bitstar_knn", False)
    a.partition = spec.get("partition", "replicated")
    a.scaling = spec.get("scaling", "weak")
    a.tree, a.queries, a.k = DEFAULTS[a.workload]
    a.exact = False
    if a.workload == "cfg4":
        # each PRM* batch grows the roadmap by 8,192 milestones: 2 + 5 batches keep it within 6 % of
        # the configuration's 10^6 vertices (20 + 10 would take it to 1.25 * 10^6)
        a.steps, a.warmup = min(a.steps, 5), min(a.warmup, 2)
    return a


def _sig(x, n=4):
    """x rounded to n significant digits (floats only; the compact line stays short)"""
    if isinstance(x, float) and math.isfinite(x) and x != 0.0:
        return float(f"{x:.{n}g}")
    return x


def _short(s, n):
    s = str(s)
    return s if len(s) <= n else s[: n - 3] + "..."


def _compact_roofline(r, full=True):
    if not r:
        return None
    keys = ("bound", "achieved", "peak", "unit", "frac", "traffic", "kernel", "kernel_ms", "kernel_ms_isolated",
            "frac_isolated") if full else ("frac", "kernel_ms", "traffic", "frac_isolated")
    out = {k: _sig(r.get(k)) for k in keys if k in r}
    if full and r.get("issue"):
        out["issue"] = {k: _sig(v) for k, v in r["issue"].items() if k != "source"}
    return out


def _compact_cpu(c, full=True):
    if not c:
        return None
    if "value" not in c:
        return dict(c)
    if not full:
        return _sig(c["value"])
    out = {k: _sig(c[k]) for k in ("value", "unit", "cores", "kind") if k in c}
    out["sample"] = _short(c.get("sample", ""), 260)
    if isinstance(c.get("single_thread"), dict) and "value" in c["single_thread"]:
        out["single_thread_value"] = _sig(c["single_thread"]["value"])
    return out


def compact_line(line, detail_path):
    """The one JSON line on stdout: the contract's fields, the headline's roofline and cpu_baseline,
    and per sub-workload only value / ms_per_step / workload / roofline {frac, kernel_ms, traffic} /
    cpu_baseline value.  Everything else is in the detail file (`detail`)."""
    keep = ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
            "vs_baseline", "dtype", "data", "rccl_ranks", "nn_queries_per_s", "motion_checks_per_s",
            "motion_valid_fraction", "wall_s")
    out = {k: _sig(line[k]) for k in keep if k in line}
    cfg = dict(line.get("config", {}))
    out["config"] = {k: _sig(v) for k, v in cfg.items() if k != "note"}
    out["phase_ms"] = {k: _sig(v) for k, v in line.get("phase_ms", {}).items() if k != "note"}
    out["roofline"] = _compact_roofline(line.get("roofline"))
    out["cpu_baseline"] = _compact_cpu(line.get("cpu_baseline"))
    ex = {}
    if line.get("single_query"):
        s = line["single_query"]
        ex["single_query_1e6"] = {"queries_per_s": _sig(s["queries_per_s"]), "kernel_us": _sig(s["kernel_us"]),
                                  "hbm_frac": _sig(s["roofline"]["frac"])}
    if line.get("single_query_1e7"):
        s = line["single_query_1e7"]
        ex["single_query_1e7"] = {"queries_per_s": _sig(s["queries_per_s"]), "kernel_us": _sig(s["kernel_us"]),
                                  "hbm_frac": _sig(s["roofline"]["frac"])}
    if line.get("rrt_device"):
        ex["rrt_device_iterations_per_s"] = _sig(line["rrt_device"]["iterations_per_s"])
    if line.get("motion_spheres"):
        ex["motion_spheres_checks_per_s"] = _sig(line["motion_spheres"]["motion_checks_per_s"])
    if line.get("rrt_star_knn"):
        ex["rrt_star_k6169_queries_per_s"] = _sig(line["rrt_star_knn"]["queries_per_s"])
    if line.get("index"):
        ex["index_full_build_ms"] = _sig(line["index"]["full_build_ms"])
    if ex:
        out["extras"] = ex
    subs = {}
    for name, s in line.get("workloads", {}).items():
        e = {"value": _sig(s.get("value")), "unit": s.get("unit"), "ms_per_step": _sig(s.get("ms_per_step")),
             "workload": _short(s.get("config", {}).get("workload", ""), 90),
             "roofline": _compact_roofline(s.get("roofline"), full=False),
             "cpu_baseline": _compact_cpu(s.get("cpu_baseline"), full=False)}
        if "device_only_value" in s:
            e["device_only_value"] = _sig(s["device_only_value"])
        subs[name] = e
    if subs:
        out["workloads"] = subs
    out["detail"] = detail_path
    return out


def write_detail(line, path):
    """the full record (every phase, extra and sub-workload with its roofline and cpu_baseline) in a
    file; returns the path written, or None"""
    if not path:
        return None
    try:
        d = os.path.dirname(os.path.abspath(path))
        os.makedirs(d, exist_ok=True)
        with open(path, "w") as f:
            json.dump(line, f, indent=1)
        return os.path.relpath(os.path.abspath(path), ROOT)
    except OSError as e:
        progress(f"detail file not written: {e}")
        return None


def progress(msg):
    """a progress line on stderr (long default runs stay visibly alive)"""
    print(f"bench [{time.strftime('%H:%M:%S')}] {msg}", file=sys.stderr, flush=True)


def measure(args, torch, dev, local, rank, world, dist, stream, cpu_seconds):
    """Run one workload: warmup, exactly args.steps timed steps bracketed by a barrier +
    synchronize on both sides (max over ranks), then the line's common fields.  Returns
    (line or None on ranks > 0, the Runner, the phase-valid fraction)."""
    if rank == 0:
        progress(f"{args.workload} ({args.partition}, {args.scaling}{', kNN' if args.bitstar_knn else ''}): setup")
    run = Runner(args, torch, dev, local, rank, stream, dist)
    ev = [[torch.cuda.Event(enable_timing=True) for _ in range(4)] for _ in range(args.steps)]
    for _ in range(max(args.warmup, len(run.lanes))):  # every lane warm
        run.step()
    torch.cuda.synchronize(dev)
    if run.tree_mode and args.workload == "cfg3":
        run.owned = torch.zeros((), dtype=torch.int64, device=dev)
    run.profile(True)
    run.kernel_time()
    scr0, fb0 = run.stats()
    rp0 = run.radius_path_stats()
    c0 = run.counters()
    units = 0
    if dist:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    if run.threaded:
        units = run.run_threaded(args.steps, ev)
    else:
        for s in range(args.steps):
            run.step(ev[s])
            units += run.units_per_step()
    torch.cuda.synchronize(dev)
    if dist:
        dist.barrier()
    torch.cuda.synchronize(dev)
    elapsed = time.perf_counter() - t0
    if run.tree_mode and args.workload == "cfg3":  # motion checks of the samples whose nearest state this rank owns
        units += int(run.owned.item())
        run.m = int(run.last_owned.item())
    kern_ms_total, kern_n, kern_name = run.kernel_time()
    kern_ms = kern_ms_total / max(kern_n, 1)
    scr1, fb1 = run.stats()
    rp1 = run.radius_path_stats()
    c1 = run.counters()
    iso_ms = None
    if len(run.lanes) > 1:  # the dominant kernel alone: a few steps on one lane, one at a time
        for _ in range(3):
            run.si = 0
            run.step()
            torch.cuda.synchronize(dev)
        iso_total, iso_n, _ = run.kernel_time()  # (cumulative since profiling started)
        iso_ms = (iso_total - kern_ms_total) / max(iso_n - kern_n, 1)
    run.profile(False)
    run.use_lane(0)
    nn_ms = float(np.mean([e[0].elapsed_time(e[1]) for e in ev]))
    edge_ms = float(np.mean([e[1].elapsed_time(e[2]) for e in ev]))
    mv_ms = float(np.mean([e[2].elapsed_time(e[3]) for e in ev]))
    t = torch.tensor([elapsed, nn_ms, edge_ms, mv_ms, kern_ms], dtype=torch.float64, device=dev)
    u = torch.tensor([units], dtype=torch.float64, device=dev)
    if dist:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dist.all_reduce(u, op=dist.ReduceOp.SUM)
    elapsed, nn_ms, edge_ms, mv_ms, kern_ms = t.tolist()
    total_units = float(u.item())
    if args.workload == "cfg4":  # edge validity of the last batch: row r holds cnt[r] edges
        cols = torch.arange(run.k, device=dev).unsqueeze(0)
        live = cols < run.cnt.unsqueeze(1)
        valid_frac = float(run.evalid[live].float().mean().item()) if bool(live.any()) else None
    elif args.workload != "cfg2":
        valid_frac = float(run.valid[: max(run.m, 1)].float().mean().item())
    else:
        valid_frac = None
    if rank != 0:
        return None, run
    metric, unit = run.metric()
    screen = kern_name.startswith(("knn32", "radius32"))
    line = {
        "metric": metric,
        "value": total_units / elapsed,
        "unit": unit,
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": elapsed * 1e3 / args.steps,
        "higher_is_better": True,
        "scaling": "strong" if (run.tree_mode or run.strong) else "weak",
        "vs_baseline": None,
        "dtype": "f32 screen + f64 certify" if screen else "f64",
        "config": run.config(world),
        "nn_queries_per_s": run.nq * world / (nn_ms * 1e-3),
        "phase_ms": {"nn": nn_ms, "steer_or_edges": edge_ms, "motion": mv_ms},
        "fast_path": {"screened": scr1 - scr0, "exact_reruns": fb1 - fb0},
        "roofline": run.roofline(kern_ms, kern_name, c0, c1, max(args.steps, 1)),
    }
    if iso_ms:  # the kernel's duration without a second step in flight, and the roofline fraction at it
        r = line["roofline"]
        r["kernel_ms_isolated"] = iso_ms
        r["frac_isolated"] = r["frac"] * kern_ms / iso_ms
    if len(run.lanes) > 1:
        line["phase_ms"]["note"] = (f"{len(run.lanes)} steps in flight: a phase's HIP events (on its lane's stream) also "
                                    "span the other lanes' kernels running meanwhile")
    if args.workload == "cfg4":  # one synchronous call per step: kNN, causal scan, edges and insert together
        line["phase_ms"] = {"prm_batch": nn_ms}
        line["edges_checked_per_s"] = run.m * world / (nn_ms * 1e-3)
        line["motion_valid_fraction"] = valid_frac
        line["roadmap_vertices"] = run.nn.size()
    elif args.workload != "cfg2":
        line["motion_checks_per_s"] = run.m * world / (mv_ms * 1e-3)
        line["motion_valid_fraction"] = valid_frac
    if args.workload == "cfg5" and not args.bitstar_knn:  # timed nearestR calls by path
        line["radius_walks"] = {"one_pass": rp1[0] - rp0[0], "overflowed": rp1[1] - rp0[1]}
    return line, run


def attach_cpu_baseline(line, run, args, rank, world, budget):
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        progress(f"{args.workload}: CPU baseline")
        t0 = time.perf_counter()
        line["cpu_baseline"] = cpu_baseline(args.workload, run.sp, run.ck, run.tree, run.q_host, run.k, budget,
                                            run.radius)
        line["cpu_baseline"]["wall_s"] = time.perf_counter() - t0
    else:
        line["cpu_baseline"] = None


def main():
    args = parse()
    env_world = os.environ.get("WORLD_SIZE")
    if env_world is None and args.gpus > 1:
        spawn_ranks(args.gpus)  # does not return
    world = int(env_world or "1")
    if world != args.gpus:
        raise SystemExit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}: launch one rank per GPU")
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    import torch

    visible = torch.cuda.device_count()  # counts devices without initialising them
    if local >= visible:
        raise SystemExit(f"bench.py: rank {rank} needs GPU {local} but only {visible} GPU(s) are visible "
                         f"(--gpus {args.gpus})")
    dist = None
    torch.cuda.set_device(local)
    rccl_ranks = 1
    if world > 1:
        import torch.distributed as dist

        dist.init_process_group(backend="nccl", device_id=torch.device("cuda", local))
        one = torch.ones(1, device=torch.device("cuda", local))
        dist.all_reduce(one)  # ranks as RCCL counts them
        rccl_ranks = int(one.item())
        if rccl_ranks != world:
            raise SystemExit(f"bench.py: RCCL reports {rccl_ranks} ranks, expected {world}")

    dev = torch.device("cuda", local)
    stream = torch.cuda.Stream(dev)  # a real (non-null) stream shared by torch events and the library
    wall0 = time.perf_counter()
    line, run = measure(args, torch, dev, local, rank, world, dist, stream, args.cpu_seconds)

    single = single_large = rrt = spheres = rrt_star = index = None
    if rank == 0 and not args.no_extras:
        progress(f"{args.workload}: extras")
    if rank == 0 and args.workload in ("cfg3", "cfg2") and not args.no_extras:
        index = index_maintenance(torch, run, local)
    if rank == 0 and args.workload == "cfg3" and not args.no_extras:
        spheres = sphere_variant(torch, run, local)
        if args.rrt_star_queries > 0:
            rrt_star = rrt_star_knn(torch, run, args.tree, args.rrt_star_queries)
    if rank == 0 and args.workload == "cfg3" and args.single_query_reps > 0:
        single = single_query_scan(torch, run.nn, dev, args.single_query_reps, args.tree,
                                   "the 28 MB of fp32 rows stay Infinity-Cache resident across back-to-back scans")
        if not args.no_extras:
            single_large = single_query_large(torch, dev, args.single_query_reps)
    if rank == 0:
        attach_cpu_baseline(line, run, args, rank, world, args.cpu_seconds)
    if rank == 0 and args.workload == "cfg3" and args.rrt_iters > 0:
        rrt = rrt_device(torch, run.nn, run.mv, run.sp, dev, args.rrt_iters)
    run.close()
    del run

    subs = {}
    names = [] if args.workloads == "none" else (
        list(SUB_WORKLOADS) if args.workloads == "auto" else [w for w in args.workloads.split(",") if w])
    want_rrt_star = "rrt_star" in names or args.workloads == "auto"
    names = [w for w in names if w != "rrt_star"]
    if args.workload != "cfg3" or args.partition != "replicated":
        names = [] if args.workloads == "auto" else names
    for name in names:
        t0 = time.perf_counter()
        sa = sub_args(args, SUB_WORKLOADS[name])
        sline, srun = measure(sa, torch, dev, local, rank, world, dist, stream, args.sub_cpu_seconds)
        if rank == 0 and sa.workload == args.workload:  # the headline's workload in another partition
            sline["cpu_baseline"] = {"same_as": "the headline line's cpu_baseline (the same samples and tree)"}
        elif rank == 0:
            attach_cpu_baseline(sline, srun, sa, rank, world, args.sub_cpu_seconds)
        if rank == 0:
            sline["wall_s"] = time.perf_counter() - t0
            subs[name] = sline
        srun.close()
        del srun
        torch.cuda.synchronize(dev)

    if (rank == 0 and world == 1 and args.workload == "cfg3" and args.partition == "replicated"
            and want_rrt_star and args.rrt_star_samples > 0):
        t0 = time.perf_counter()
        progress("rrt_star: setup, steps, CPU baseline")
        sub = rrt_star_workload(torch, dev, local, stream, args.steps, args.warmup, ns=args.rrt_star_samples,
                                cpu_seconds=args.sub_cpu_seconds, cpu=not args.no_cpu_baseline)
        sub["wall_s"] = time.perf_counter() - t0
        subs["rrt_star"] = sub
        torch.cuda.synchronize(dev)

    if rank == 0:
        line["rccl_ranks"] = rccl_ranks
        line["data"] = ("synthetic: the reference's RNG streams — RNG::setSeed(42), then a tree sampler and a query "
                        "sampler (allocStateSampler x2); rank r takes queries [r*Q, (r+1)*Q)")
        if index:
            line["index"] = index
        if spheres:
            line["motion_spheres"] = spheres
        if rrt_star:
            line["rrt_star_knn"] = rrt_star
        if single:
            line["single_query"] = single
        if single_large:
            line["single_query_1e7"] = single_large
        if rrt:
            line["rrt_device"] = rrt
        if subs:
            line["workloads"] = subs
        line["wall_s"] = time.perf_counter() - wall0
        detail = write_detail(line, args.detail)
        print(json.dumps(compact_line(line, detail)), flush=True)
    # release every library handle while the HIP runtime (and a profiler attached to it) is up
    torch.cuda.synchronize(dev)
    from ompl_amd import abi
    abi.close_all()
    torch.cuda.synchronize(dev)
    maps = os.environ.get("OMPL_AMD_MAPS")  # library load addresses, to symbolise an exit-time fault
    if maps:
        with open("/proc/self/maps") as fi, open(maps, "w") as fo:
            fo.write(fi.read())
    if dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
