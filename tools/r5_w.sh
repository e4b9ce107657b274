#!/bin/bash
# Round-5 GPU step W: walk event counters (probe build in vlib/) for the headline (10^6, k = 10) and
# BIT*'s kNN (10^7, k = 57), then SQ counters of the cfg5k and cfg3 walks.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
out=gpurun_out/${1:-r5_w}; mkdir -p "$out"
OMPL_GPU_LIB=vlib/libompl_gpu_probe.so timeout -k 10 200 python -u tools/walk_probe.py --k 10 > "$out/probe_cfg3.json" 2> "$out/probe_cfg3.err" || { tail -20 "$out/probe_cfg3.err"; exit 1; }
cat "$out/probe_cfg3.json"
OMPL_GPU_LIB=vlib/libompl_gpu_probe.so timeout -k 10 300 python -u tools/walk_probe.py --k 57 --tree 10000000 > "$out/probe_cfg5k.json" 2> "$out/probe_cfg5k.err" || { tail -20 "$out/probe_cfg5k.err"; exit 1; }
cat "$out/probe_cfg5k.json"
bash tools/sq_counters.sh "$out/sq_cfg5k" --workload cfg5 --bitstar-knn > "$out/sq_cfg5k.log" 2>&1 || { tail -20 "$out/sq_cfg5k.log"; exit 1; }
bash tools/sq_counters.sh "$out/sq_cfg3" > "$out/sq_cfg3.log" 2>&1 || { tail -20 "$out/sq_cfg3.log"; exit 1; }
echo ok
