"""RRT*'s neighbourhood query at the headline tree size (k = 6,169 at 10^6 SE(3) states,
RRTstar.cpp:603-618) through the device-decided large-k path: 1,000 queries x reps, timed with
HIP events on the library's stream; run it under rocprofv3 for the per-kernel split.
usage: python tools/large_k_probe.py [reps]"""
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from ompl_amd import NearestNeighborsGPU, workloads as W  # noqa: E402
from ompl_amd.spaces import SE3StateSpace  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 5
dev = torch.device("cuda", 0)
st = torch.cuda.Stream(dev)
sp = SE3StateSpace(0.0, 1.0)
tree, q = W.reference_states(sp, [1_000_000, 1000], seed=42)
nn = NearestNeighborsGPU(sp, 0)
nn.add(tree)
nn.set_stream(st.cuda_stream)
k = W.rrt_star_k(1_000_000, 6)
dq = torch.from_numpy(q).to(dev)
ids = torch.empty((1000, k), dtype=torch.int32, device=dev)
dd = torch.empty((1000, k), dtype=torch.float64, device=dev)
nn.knn_device(dq.data_ptr(), 1000, k, ids.data_ptr(), dd.data_ptr())
torch.cuda.synchronize()
ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
ev[0].record(st)
for _ in range(reps):
    nn.knn_device(dq.data_ptr(), 1000, k, ids.data_ptr(), dd.data_ptr())
ev[1].record(st)
torch.cuda.synchronize()
print(json.dumps({"k": k, "queries": 1000, "ms_per_batch": ev[0].elapsed_time(ev[1]) / reps}))
nn.close()
