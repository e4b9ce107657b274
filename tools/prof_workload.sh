#!/bin/bash
# rocprofv3 kernel trace + FETCH_SIZE / WRITE_SIZE passes (separate runs) of one bench workload.
# usage (on the GPU box): bash tools/prof_workload.sh <workload> <tag> [extra bench args]
#   -> gpurun_out/prof_<tag>/   (TRACE_STEPS: timed steps of the trace pass, default 20)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
w=$1; tag=$2; shift 2; out=gpurun_out/prof_$tag
mkdir -p "$out"
base="--workload $w --no-cpu-baseline --single-query-reps 0 --rrt-iters 0 --no-extras"
ws=${WORKLOADS:-none}
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$out" -o trace --output-format csv -- python bench.py $base --steps ${TRACE_STEPS:-20} --warmup 5 --workloads $ws "$@" > "$out/trace.log" 2>&1 || exit $?
timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE -d "$out" -o pmc_fetch --output-format csv -- python bench.py $base --steps 2 --warmup 1 --workloads $ws "$@" > "$out/fetch.log" 2>&1 || exit $?
timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE -d "$out" -o pmc_write --output-format csv -- python bench.py $base --steps 2 --warmup 1 --workloads $ws "$@" > "$out/write.log" 2>&1 || exit $?
grep '^{' "$out/trace.log" | cut -c1-300
python tools/kstats.py "$(find "$out" -name "trace_kernel_stats.csv" | head -1)" 4
