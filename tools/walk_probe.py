"""Measurement probe (not product): the batched kNN walk on the headline workload with a probe
build of the library (make -C ompl_amd/csrc probe -> tools/probe_lib/), printing
the walk kernel's time and its event counters per launch.

    OMPL_GPU_LIB=tools/probe_lib/libompl_gpu_probe.so python tools/walk_probe.py [--k 10]
"""
import argparse
import ctypes as C
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--k", type=int, default=10)
    ap.add_argument("--tree", type=int, default=1_000_000)
    ap.add_argument("--queries", type=int, default=100_000)
    ap.add_argument("--space", default="se3")
    ap.add_argument("--reps", type=int, default=3)
    a = ap.parse_args()
    import numpy as np
    import torch

    from ompl_amd import NearestNeighborsGPU, abi
    from ompl_amd import workloads as W
    from ompl_amd.spaces import RealVectorStateSpace, SE3StateSpace

    sp = SE3StateSpace() if a.space == "se3" else RealVectorStateSpace(6)
    tree, q = W.reference_states(sp, (a.tree, a.queries), seed=42)
    nn = NearestNeighborsGPU(sp, 0)
    nn.add(tree)
    dev = torch.device("cuda", 0)
    dq = torch.from_numpy(q).to(dev)
    ids = torch.empty((a.queries, a.k), dtype=torch.int32, device=dev)
    dd = torch.empty((a.queries, a.k), dtype=torch.float64, device=dev)
    nn.knn_device(dq.data_ptr(), a.queries, a.k, ids.data_ptr(), dd.data_ptr())
    nn.sync()
    f = getattr(abi.lib, "ompl_gpu_probe_counters", None)
    cnt = (C.c_uint64 * 23)()

    def counters():
        if f is None:
            return [0] * 23
        f(nn._h, cnt, 23)
        return list(cnt)

    c0 = counters()
    nn.profile(True)
    ms0, n0, _ = nn.kernel_time()
    for _ in range(a.reps):
        nn.knn_device(dq.data_ptr(), a.queries, a.k, ids.data_ptr(), dd.data_ptr())
    nn.sync()
    ms1, n1, name = nn.kernel_time()
    c1 = counters()
    per = [(y - x) / a.reps for x, y in zip(c0, c1)]
    keys = ["tiles", "tiles_bruteforce", "qscans", "radius_tiles", "radius_qscans", "offers", "bulk_merges",
            "insertions", "supertile_masks", "super_rounds", "empty_masks", "recheck_skips", "walk_cycles",
            "prologue_cycles", "mask_cycles", "issue_cycles", "tile_wait_cycles", "scan_cycles",
            "offer_cycles (inside scan)", "next_super_cycles", "loop_tail_cycles", "copy_wait_cycles",
            "timer_overhead_cycles (one per iteration)"]
    out = {"lib": os.path.basename(abi.LIB_PATH), "kernel": name, "kernel_ms": (ms1 - ms0) / max(n1 - n0, 1),
           "per_query": {k: v / a.queries for k, v in zip(keys, per) if v}, "reruns": nn.stats()[1],
           # the timers are per wave (two queries): shader-clock cycles per wave and their shares
           "per_wave_cycles": {k: 2 * v / a.queries for k, v in zip(keys, per) if "_cycles" in k}}
    wc = out["per_wave_cycles"].get("walk_cycles", 0)
    if wc:
        out["cycle_shares"] = {k: v / wc for k, v in out["per_wave_cycles"].items()}
    # spot parity against the exact path on a few queries
    ref = NearestNeighborsGPU(sp, 0)
    ref.set_mode(1)
    ref.add(tree)
    ri, rd, _ = ref.nearestKBatch(q[:200], a.k)
    gi = ids[:200].cpu().numpy().astype(np.int64)
    out["parity_200"] = bool((gi == ri.astype(np.int64)).all())
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
