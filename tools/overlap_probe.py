"""Measurement probe (not product): the headline step (nearestK(k = 10) + steer + checkMotion over
10^5 samples on the 10^6-state SE(3) tree) issued back to back on ONE stream against alternating
over L streams (one NN / validator handle pair per stream, same tree and samples), to measure how
much of the walk's tail and the small kernels around it a second in-flight step hides.
    python tools/overlap_probe.py [--lanes 1,2,3] [--steps 20]"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--lanes", default="1,2,3")
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--queries", type=int, default=100_000)
    a = ap.parse_args()
    import torch

    import bench
    from ompl_amd import DiscreteMotionValidatorGPU, NearestNeighborsGPU
    from ompl_amd.checkers import HypercubeChecker
    from ompl_amd.spaces import SE3StateSpace

    dev = torch.device("cuda", 0)
    sp, ck = SE3StateSpace(0.0, 1.0), HypercubeChecker(3, 0.1)
    tree, q = bench._stream_inputs(sp, 1_000_000, a.queries)
    dq = torch.from_numpy(q).to(dev)
    maxd = 0.2 * sp.getMaximumExtent()
    nq = a.queries
    lanes = []
    for i in range(max(int(x) for x in a.lanes.split(","))):
        st = torch.cuda.Stream(dev)
        nn, mv = NearestNeighborsGPU(sp, 0), DiscreteMotionValidatorGPU(sp, ck, 0)
        nn.add(tree)
        nn.set_stream(st.cuda_stream)
        mv.set_stream(st.cuda_stream)
        bufs = dict(ids=torch.empty((nq, 10), dtype=torch.int32, device=dev),
                    dd=torch.empty((nq, 10), dtype=torch.float64, device=dev),
                    s1=torch.empty((nq, 7), dtype=torch.float64, device=dev),
                    s2=torch.empty((nq, 7), dtype=torch.float64, device=dev),
                    v=torch.empty(nq, dtype=torch.uint8, device=dev))
        lanes.append((st, nn, mv, bufs))

    def step(L):
        st, nn, mv, b = L
        nn.knn_device(dq.data_ptr(), nq, 10, b["ids"].data_ptr(), b["dd"].data_ptr())
        nn.steer_device(dq.data_ptr(), nq, b["ids"].data_ptr(), 10, maxd, b["s1"].data_ptr(), b["s2"].data_ptr())
        mv.check_device(b["s1"].data_ptr(), b["s2"].data_ptr(), nq, b["v"].data_ptr())

    out = {}
    for n in (int(x) for x in a.lanes.split(",")):
        for i in range(3 * n):
            step(lanes[i % n])
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        for i in range(a.steps):
            step(lanes[i % n])
        torch.cuda.synchronize(dev)
        ms = (time.perf_counter() - t0) * 1e3 / a.steps
        out[n] = {"ms_per_step": ms, "units_per_s": 2 * nq / (ms * 1e-3)}
        print(n, out[n], flush=True)
    ref = lanes[0][3]
    for st, nn, mv, b in lanes[1:]:  # every lane answered the same batch identically
        assert torch.equal(b["ids"], ref["ids"]) and torch.equal(b["v"], ref["v"])
    print(json.dumps(out))


if __name__ == "__main__":
    main()
