"""GPU probe: kernel time of the kNN scan per path on the BASELINE workloads.

    python tools/knn_probe.py [--quick]

Prints one JSON line per (workload, mode) with the dominant kernel's average time (HIP
events on the launch stream), the culled screen's scanned-tile fraction and the exact
re-run count.  Modes: 0 culled fp32 screen, 1 exact fp64 scan, 2 chunked fp32 screen.
"""
import argparse
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--quick", action="store_true")
    ap.add_argument("--modes", default="0,2,1")
    ap.add_argument("--only", default=None, help="run only this workload")
    args = ap.parse_args()
    import torch

    from ompl_amd import NearestNeighborsGPU
    from ompl_amd import workloads as W
    from ompl_amd.spaces import KinematicChainSpace, RealVectorStateSpace, SE3StateSpace

    dev = torch.device("cuda", 0)
    rng = np.random.default_rng(42)
    work = [
        ("cfg3_se3_1e6_k10", SE3StateSpace(), W.uniform_se3(rng, 1_000_000), W.uniform_se3(rng, 100_000), 10),
        ("cfg3_se3_1e6_k1", None, None, None, 1),
        ("cfg2_r6_1e5_k10", RealVectorStateSpace(6), W.uniform_rv(rng, 100_000, 6), W.uniform_rv(rng, 100_000, 6), 10),
        ("chain12_1e5_k10", KinematicChainSpace(12, 1 / 12), W.uniform_chain(rng, 100_000, 12),
         W.uniform_chain(rng, 20_000, 12), 10),
    ]
    prev = None
    for name, sp, data, q, k in work:
        if sp is None:
            sp, data, q = prev
        prev = (sp, data, q)
        if args.only and name != args.only:
            continue
        nn = NearestNeighborsGPU(sp, 0)
        nn.add(data)
        dq = torch.from_numpy(q).to(dev)
        ids = torch.empty((len(q), k), dtype=torch.int32, device=dev)
        dd = torch.empty((len(q), k), dtype=torch.float64, device=dev)
        modes = [int(m) for m in args.modes.split(",")]
        if name.startswith("chain"):
            modes = [1]
        for mode in modes:
            if mode == 1 and name.startswith("cfg3") and args.quick:
                continue
            nn.set_mode(mode)
            nn.knn_device(dq.data_ptr(), len(q), k, ids.data_ptr(), dd.data_ptr())  # warm (builds sorted copy)
            nn.sync()
            nn.profile(True)
            ms0, n0, _ = nn.kernel_time()
            c0 = nn.cull_stats()
            s0 = nn.stats()
            reps = 3
            t0 = time.perf_counter()
            for _ in range(reps):
                nn.knn_device(dq.data_ptr(), len(q), k, ids.data_ptr(), dd.data_ptr())
            nn.sync()
            wall = (time.perf_counter() - t0) / reps
            ms1, n1, kname = nn.kernel_time()
            c1 = nn.cull_stats()
            s1 = nn.stats()
            nn.profile(False)
            scanned = (c1[0] - c0[0]) / max(c1[1] - c0[1], 1)
            pair_frac = (c1[2] - c0[2]) * 64 / reps / (len(q) * len(data))
            print(json.dumps({"workload": name, "mode": mode, "kernel": kname,
                              "kernel_ms": (ms1 - ms0) / max(n1 - n0, 1), "call_ms": wall * 1e3,
                              "queries_per_s": len(q) / wall, "tiles_scanned_frac": scanned, "pairs_scanned_frac": pair_frac,
                              "exact_reruns": s1[1] - s0[1]}), flush=True)
        del nn


if __name__ == "__main__":
    main()
