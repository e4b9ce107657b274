#!/bin/bash
# Round-2 measurement pass on the GPU box: the default bench line, then a kernel trace of the
# headline workload alone and one of the extra measurements (index build / appends, RRT* k).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
out=gpurun_out/${1:-r2}
mkdir -p "$out"
timeout -k 10 400 python -u bench.py > "$out/bench.json" 2> "$out/bench.err" || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$out/trace" -o trace --output-format csv -- python bench.py \
    --steps 5 --warmup 2 --no-cpu-baseline --single-query-reps 0 --rrt-iters 0 --no-extras > "$out/trace.log" 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$out/trace_extras" -o trace --output-format csv -- python bench.py \
    --steps 1 --warmup 1 --no-cpu-baseline --single-query-reps 50 --rrt-iters 200 > "$out/trace_extras.log" 2>&1 || exit $?
echo done
