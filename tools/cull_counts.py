"""Measurement probe (not product): per launch of the culled kNN walk, the tiles it fetched, the
(tile, query) scans and the tiles of a brute-force pass (ompl_gpu_nn_cull_stats), for the
headline (10^6 SE3, k = 10) and cfg5k (10^7 valid SE3 samples, k = 57); with the tile's bytes
(7 fp32 rows x 64 states = 1,792 B) this splits the walk's L2 requests into tile and box reads.
    python tools/cull_counts.py"""
import json
import math
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch

    import bench
    from ompl_amd import NearestNeighborsGPU
    from ompl_amd import workloads as W
    from ompl_amd.checkers import SpheresChecker
    from ompl_amd.motion import DiscreteMotionValidatorGPU
    from ompl_amd.spaces import SE3StateSpace

    dev = torch.device("cuda", 0)
    sp = SE3StateSpace(0.0, 1.0)
    out = {}
    for name, n, nq, k, valid in (("cfg3", 1_000_000, 100_000, 10, None), ("cfg5k", 10_000_000, 100_000, 57, True)):
        ck = None
        if valid:
            c, r = W.sphere_field(32, 0.1, 7)
            mv = DiscreteMotionValidatorGPU(sp, SpheresChecker(c, r), 0)
            tree, q = bench._stream_inputs(sp, n, nq, mv.isValid)
            mv.close()
        else:
            tree, q = bench._stream_inputs(sp, n, nq)
        nn = NearestNeighborsGPU(sp, 0)
        nn.add(tree)
        dq = torch.from_numpy(q).to(dev)
        ids = torch.empty((nq, k), dtype=torch.int32, device=dev)
        dd = torch.empty((nq, k), dtype=torch.float64, device=dev)
        nn.knn_device(dq.data_ptr(), nq, k, ids.data_ptr(), dd.data_ptr())
        nn.sync()
        c0 = nn.cull_stats()
        reps = 3
        for _ in range(reps):
            nn.knn_device(dq.data_ptr(), nq, k, ids.data_ptr(), dd.data_ptr())
        nn.sync()
        c1 = nn.cull_stats()
        tiles, bf, scans = ((b - a) / reps for a, b in zip(c0, c1))
        out[name] = {"tiles_fetched_per_launch": tiles, "tiles_per_wave": tiles / math.ceil(nq / 2),
                     "qscans_per_query": scans / nq, "tile_bytes_per_launch": tiles * 1792,
                     "bruteforce_tiles": bf}
        print(name, out[name], flush=True)
        nn.close()
    print(json.dumps(out))


if __name__ == "__main__":
    main()
