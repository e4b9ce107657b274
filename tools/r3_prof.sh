#!/bin/bash
# Round-3 profiles of the final build: for each workload the kernel trace and the FETCH_SIZE /
# WRITE_SIZE passes (tools/prof_workload.sh), the headline's SQ counters, the extras trace
# (single-query stream at 10^6 / 10^7, device RRT, RRT* large k) with its PMC passes, and a
# trace of the k-d build at 10^6 / 10^7.  Every GPU step has its own limit; a failure ends the call.
# usage: bash tools/r3_prof.sh [workloads]   -> gpurun_out/prof_r3f_<w>/, gpurun_out/r3f_*/
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
for w in ${1:-cfg3 cfg2 cfg4 cfg5}; do
  bash tools/prof_workload.sh "$w" "r3f_$w" || { echo "prof $w rc=$?"; exit 1; }
done
bash tools/sq_counters.sh gpurun_out/r3f_sq > gpurun_out/r3f_sq.log 2>&1 || { echo "sq rc=$?"; exit 1; }
bash tools/r3_extras.sh r3f_extras || { echo "extras rc=$?"; exit 1; }
mkdir -p gpurun_out/r3f_build
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/r3f_build -o trace --output-format csv -- \
  python tools/build_probe.py > gpurun_out/r3f_build/build.log 2>&1 || { echo "build rc=$?"; exit 1; }
grep '^{' gpurun_out/r3f_build/build.log
echo done
