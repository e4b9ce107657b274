#!/bin/bash
# Round-5 GPU step K: cfg4 kernel profile (rocprofv3 --kernel-trace --stats) of the current build.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
out=gpurun_out/${1:-r5_k}; mkdir -p "$out/prof"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$out/prof" -o cfg4 --output-format csv -- python -u bench.py --workload cfg4 --steps 10 --warmup 3 \
    --workloads none --no-extras --no-cpu-baseline > "$out/prof.log" 2>&1 || { tail -20 "$out/prof.log"; exit 1; }
tail -1 "$out/prof.log" | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('cfg4', d['value'], d['ms_per_step'])"
python tools/kstats.py "$(find "$out/prof" -name "*kernel_stats.csv" | head -1)" 6
