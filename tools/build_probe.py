"""Device k-d build of the sorted store: full build time at 10^6 and 10^7 SE(3) states (HIP
events on the library's stream), then one 10^5-query kNN batch to check the walk still runs.
usage: python tools/build_probe.py [n ...]"""
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from ompl_amd import NearestNeighborsGPU, workloads as W  # noqa: E402
from ompl_amd.spaces import SE3StateSpace  # noqa: E402

dev = torch.device("cuda", 0)
st = torch.cuda.Stream(dev)
out = {}
for n in [int(x) for x in sys.argv[1:]] or [1_000_000, 10_000_000]:
    data = W.uniform_se3(np.random.default_rng(1), n)
    times = []
    for rep in range(2):  # fresh structures: the first also allocates the store and its scratch
        nn = NearestNeighborsGPU(SE3StateSpace(), 0)
        nn.add(data)
        nn.set_stream(st.cuda_stream)
        torch.cuda.synchronize()
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
        ev[0].record(st)
        nn.build_index()
        ev[1].record(st)
        torch.cuda.synchronize()
        times.append(ev[0].elapsed_time(ev[1]))
        if rep == 0:
            nn.close()
    q = torch.from_numpy(W.uniform_se3(np.random.default_rng(2), 100_000)).to(dev)
    ids = torch.empty((100_000, 10), dtype=torch.int32, device=dev)
    dd = torch.empty((100_000, 10), dtype=torch.float64, device=dev)
    nn.profile(True)
    for _ in range(3):
        nn.knn_device(q.data_ptr(), 100_000, 10, ids.data_ptr(), dd.data_ptr())
    torch.cuda.synchronize()
    ms, cnt, name = nn.kernel_time()
    out[n] = {"build_ms": times, "walk_ms": ms / max(cnt, 1), "walk": name, "cull": nn.cull_stats()}
    nn.close()
print(json.dumps(out))
