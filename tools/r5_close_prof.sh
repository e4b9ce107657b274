#!/bin/bash
# Round-5 closing profiles of the shipped build: kernel trace (20 timed steps) + FETCH / WRITE passes
# per workload (tools/prof_workload.sh), and for the headline the SQ instruction counters.
# usage: bash tools/r5_close_prof.sh a|b      (a: cfg3 + SQ, cfg2, cfg4; b: cfg5, cfg5k, RRT*)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
case "${1:-a}" in
a)
  bash tools/prof_workload.sh cfg3 r5c_cfg3 || exit 1
  bash tools/sq_counters.sh gpurun_out/prof_r5c_cfg3/sq --workload cfg3 > gpurun_out/prof_r5c_cfg3/sq.log 2>&1 || exit 1
  bash tools/prof_workload.sh cfg2 r5c_cfg2 || exit 1
  bash tools/prof_workload.sh cfg4 r5c_cfg4 || exit 1 ;;
b)
  bash tools/prof_workload.sh cfg5 r5c_cfg5 || exit 1
  bash tools/prof_workload.sh cfg5 r5c_cfg5k --bitstar-knn || exit 1
  WORKLOADS=rrt_star TRACE_STEPS=5 bash tools/prof_workload.sh cfg3 r5c_rrt_star || exit 1 ;;
esac
echo done
