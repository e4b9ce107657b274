#!/bin/bash
# The headline walk profiled over the default bench's own step counts (20 timed + 5 warmup), so the
# rocprof average covers the same launches as bench.py's HIP events (short profiles: 3 launches,
# clocks still ramping).  -> gpurun_out/prof_r4_cfg3_long/
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
out=gpurun_out/prof_r4_cfg3_long; mkdir -p "$out"
args="--workload cfg3 --steps 20 --warmup 5 --no-cpu-baseline --single-query-reps 0 --rrt-iters 0 --no-extras --workloads none"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$out" -o trace --output-format csv -- python bench.py $args > "$out/trace.log" 2>&1 || exit $?
grep '^{' "$out/trace.log" | cut -c1-200
