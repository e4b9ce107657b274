#!/bin/bash
# round-4 first GPU step: the BIT* kNN line (cfg5 --bitstar-knn, k = 57 at 10^7) with its CPU
# baseline, its rocprof trace + FETCH/WRITE passes, then the radius-walk occupancy A/B (var 5 / 6).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
out=gpurun_out/r4a; mkdir -p "$out"
timeout -k 10 600 python -u -m pytest tests/test_gpu_spaces.py tests/test_gpu_large_k.py tests/test_gpu_motion.py tests/test_gpu_prm.py tests/test_gpu_batch.py tests/test_gpu_fullsize.py tests/test_shard_gloo.py -x -q --timeout 120 --timeout-method thread > "$out/spaces.log" 2>&1; rc=$?
tail -3 "$out/spaces.log"; case $rc in 124|134|137|139) exit 1;; esac
s=$(date +%s)
timeout -k 10 400 python -u bench.py --workload cfg5 --bitstar-knn --steps 10 --warmup 2 --cpu-seconds 8 \
  > "$out/cfg5k.json" 2> "$out/cfg5k.err" || { echo "cfg5k rc=$?"; tail -5 "$out/cfg5k.err"; exit 1; }
echo "cfg5k wall $(( $(date +%s) - s )) s"; cut -c1-600 "$out/cfg5k.json"
s=$(date +%s)
timeout -k 10 590 python -u bench.py --steps 20 --warmup 5 > "$out/default.json" 2> "$out/default.err" || { echo "default rc=$?"; tail -5 "$out/default.err"; exit 1; }
echo "default wall $(( $(date +%s) - s )) s"
bash tools/prof_workload.sh cfg5 r4_cfg5k --bitstar-knn || { echo "prof rc=$?"; exit 1; }

