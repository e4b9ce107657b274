#!/bin/bash
# Round-4 profiles of the final build (part 1 or 2), each GPU step under its own limit, a failure
# ends the call.  usage: bash tools/r4_prof.sh 1|2
#   1: cfg3 trace + FETCH / WRITE + SQ counters + the walk probe; cfg2; the large-k extras; the
#      single-query scan at 10^6 and at 10^7 (one process each); the k-d build at 10^6 / 10^7
#   2: cfg4, cfg5, cfg5k traces + FETCH / WRITE
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
if [ "${1:-1}" = 1 ]; then
  bash tools/prof_workload.sh cfg3 r4_cfg3 || { echo "prof cfg3 rc=$?"; exit 1; }
  bash tools/sq_counters.sh gpurun_out/r4_sq > gpurun_out/r4_sq.log 2>&1 || { echo "sq rc=$?"; exit 1; }
  if [ -f tools/probe_lib/libompl_gpu_probe0.so ]; then
    OMPL_GPU_LIB=tools/probe_lib/libompl_gpu_probe0.so timeout -k 10 200 python tools/walk_probe.py \
      > gpurun_out/r4_walk_probe.json 2> gpurun_out/r4_walk_probe.err || { echo "probe rc=$?"; exit 1; }
  fi
  bash tools/prof_workload.sh cfg2 r4_cfg2 || { echo "prof cfg2 rc=$?"; exit 1; }
  out=gpurun_out/r4_extras; mkdir -p "$out"
  args="--steps 2 --warmup 1 --no-cpu-baseline --single-query-reps 0 --rrt-iters 2000 --workloads none"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$out" -o trace --output-format csv -- python bench.py $args \
    > "$out/trace.log" 2>&1 || { echo "extras trace rc=$?"; exit 1; }
  timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE -d "$out" -o pmc_fetch --output-format csv -- python bench.py $args \
    > "$out/fetch.log" 2>&1 || { echo "extras fetch rc=$?"; exit 1; }
  timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE -d "$out" -o pmc_write --output-format csv -- python bench.py $args \
    > "$out/write.log" 2>&1 || { echo "extras write rc=$?"; exit 1; }
  for n in 1000000 10000000; do
    o=gpurun_out/r4_single_$n; mkdir -p "$o"
    timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$o" -o trace --output-format csv -- python tools/single_query_prof.py $n \
      > "$o/run.log" 2>&1 || { echo "single $n rc=$?"; exit 1; }
    timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE -d "$o" -o pmc_fetch --output-format csv -- python tools/single_query_prof.py $n \
      > "$o/fetch.log" 2>&1 || { echo "single fetch $n rc=$?"; exit 1; }
  done
  mkdir -p gpurun_out/r4_build
  timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/r4_build -o trace --output-format csv -- \
    python tools/build_probe.py > gpurun_out/r4_build/build.log 2>&1 || { echo "build rc=$?"; exit 1; }
else
  for w in cfg4 cfg5 cfg5k; do
    a="${w%k}"; x=""; [ "$w" = cfg5k ] && x="--bitstar-knn"
    bash tools/prof_workload.sh "$a" "r4_$w" $x || { echo "prof $w rc=$?"; exit 1; }
  done
fi
echo done
