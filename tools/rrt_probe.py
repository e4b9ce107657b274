"""GPU probe: the device RRT loop (ompl_gpu_rrt_grow_device) on the cfg3 tree (10^6 SE(3) states
from the reference streams, HypercubeBenchmark checker) — iterations/s for the library named by
OMPL_GPU_LIB; the phase-timer build (VARIANT=4) also prints per-iteration phase times.
    python tools/rrt_probe.py [iters] [checker: hypercube|free]"""
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch

    from ompl_amd import NearestNeighborsGPU, workloads as W
    from ompl_amd.checkers import AllValidChecker, HypercubeChecker
    from ompl_amd.motion import DiscreteMotionValidatorGPU
    from ompl_amd.spaces import SE3StateSpace

    iters = int(sys.argv[1]) if len(sys.argv) > 1 else 4000
    ck_name = sys.argv[2] if len(sys.argv) > 2 else "hypercube"
    dev = torch.device("cuda", 0)
    sp = SE3StateSpace(0.0, 1.0)
    ck = HypercubeChecker(3, 0.1) if ck_name == "hypercube" else AllValidChecker()
    nn = NearestNeighborsGPU(sp, 0)
    nn.add(W.uniform_se3(np.random.default_rng(42), 1_000_000))
    mv = DiscreteMotionValidatorGPU(sp, ck, 0)
    s = torch.from_numpy(W.uniform_se3(np.random.default_rng(98), iters)).to(dev)
    near = torch.empty(iters, dtype=torch.int32, device=dev)
    added = torch.empty(iters, dtype=torch.int32, device=dev)
    maxd = 0.2 * sp.getMaximumExtent()
    nn.rrt_grow_device(mv, s.data_ptr(), 8, maxd, near.data_ptr(), added.data_ptr())
    torch.cuda.synchronize()
    n0 = nn.size()
    t0 = time.perf_counter()
    nn.rrt_grow_device(mv, s.data_ptr(), iters, maxd, near.data_ptr(), added.data_ptr())
    wall = time.perf_counter() - t0
    print(json.dumps({"lib": os.path.basename(os.environ.get("OMPL_GPU_LIB", "product")), "checker": ck_name,
                      "iterations_per_s": iters / wall, "us_per_iteration": wall / iters * 1e6,
                      "states_added": nn.size() - n0}), flush=True)


if __name__ == "__main__":
    main()
