"""One store size per process for the single-query (RRT nearest) scan, so that a rocprofv3
--kernel-trace of it gives that size's own kernel time (bench.py's extras run 10^6 and 10^7 in
one process).  usage: python tools/single_query_prof.py <states> [reps]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import json  # noqa: E402

import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402
from ompl_amd import NearestNeighborsGPU, abi  # noqa: E402
from ompl_amd import workloads as W  # noqa: E402
from ompl_amd.spaces import SE3StateSpace  # noqa: E402

n = int(sys.argv[1])
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 200
dev = torch.device("cuda", 0)
nn = NearestNeighborsGPU(SE3StateSpace(), 0)
nn.set_stream(torch.cuda.current_stream(dev).cuda_stream)
nn.add(W.uniform_se3(np.random.default_rng(1234), n))
r = bench.single_query_scan(torch, nn, dev, reps, n, f"{n} states, one process")
print(json.dumps(r))
nn.close()
abi.close_all()
