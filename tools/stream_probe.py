"""GPU probe: single-query fp32 stream (knn_stream32.hip) over a 10^7-state SE(3) store.
Prints the kernel's mean time (HIP events on its stream) and GB/s at 28 B per state for the
library named by OMPL_GPU_LIB (product build by default).   python tools/stream_probe.py [n]"""
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch

    from ompl_amd import NearestNeighborsGPU, workloads as W
    from ompl_amd.spaces import SE3StateSpace

    n = int(sys.argv[1]) if len(sys.argv) > 1 else 10_000_000
    dev = torch.device("cuda", 0)
    nn = NearestNeighborsGPU(SE3StateSpace(), 0)
    nn.add(W.uniform_se3(np.random.default_rng(1234), n))
    reps = 300
    q = torch.from_numpy(W.uniform_se3(np.random.default_rng(99), reps)).to(dev)
    ids = torch.empty(reps, dtype=torch.int32, device=dev)
    dd = torch.empty(reps, dtype=torch.float64, device=dev)
    for i in range(10):
        nn.knn_device(q[i].data_ptr(), 1, 1, ids[i].data_ptr(), dd[i].data_ptr())
    torch.cuda.synchronize()
    nn.profile(True)
    ms0, n0, _ = nn.kernel_time()
    t0 = time.perf_counter()
    for i in range(reps):
        nn.knn_device(q[i].data_ptr(), 1, 1, ids[i].data_ptr(), dd[i].data_ptr())
    torch.cuda.synchronize()
    wall = time.perf_counter() - t0
    ms1, n1, name = nn.kernel_time()
    us = (ms1 - ms0) / max(n1 - n0, 1) * 1e3
    print(json.dumps({"lib": os.path.basename(os.environ.get("OMPL_GPU_LIB", "product")), "kernel": name,
                      "kernel_us": us, "GBps": n * 28 / us / 1e3, "queries_per_s": reps / wall}), flush=True)


if __name__ == "__main__":
    main()
