"""Debug probe: fp32 screen at tiny coordinate scales (underflow) vs the exact path."""
import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "oracle"))
import numpy as np
import pyoracle as O
from ompl_amd import NearestNeighborsGPU
from ompl_amd import workloads as W
from ompl_amd.spaces import RealVectorStateSpace

for scale in (1e-25, 1e-18, 1e-12):
    rng = np.random.default_rng(41)
    sp = RealVectorStateSpace(4)
    data, q = W.uniform_rv(rng, 5000, 4) * scale, W.uniform_rv(rng, 100, 4) * scale
    for mode in (0, 2, 1):
        nn = NearestNeighborsGPU(sp, 0)
        nn.set_mode(mode)
        nn.add(data)
        ids, d, cnt = nn.nearestKBatch(q, 1)
        oi, od, _ = O.knn(sp, data, q, 1)
        bad = np.nonzero(ids[:, 0].astype(np.int64) != oi[:, 0].astype(np.int64))[0]
        print(f"scale {scale} mode {mode}: stats {nn.stats()} rerun_full {nn.rerun_stats()} bad {len(bad)} {bad[:10]}",
              flush=True)
        for b in bad[:3]:
            print("   q", b, "got", ids[b, 0], d[b, 0], "want", oi[b, 0], od[b, 0])
