#!/bin/bash
# Round-5 profiles: kernel trace (20 timed steps) + FETCH / WRITE passes per workload.
# usage: bash tools/r5_prof.sh <workload...>   (rrt_star: the cfg3 run with the RRT* workload)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for w in "$@"; do
  echo "== $w"
  if [ "$w" = rrt_star ]; then
    WORKLOADS=rrt_star TRACE_STEPS=5 bash tools/prof_workload.sh cfg3 r5_rrt_star || exit 1
  elif [ "$w" = cfg5k ]; then
    bash tools/prof_workload.sh cfg5 r5_cfg5k --bitstar-knn || exit 1
  else
    bash tools/prof_workload.sh $w r5_$w || exit 1
  fi
done
