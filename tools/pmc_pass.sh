#!/bin/bash
# One rocprofv3 --pmc pass (no other trace domains) over a short bench run of one workload.
# usage (on the GPU box): bash tools/pmc_pass.sh <outdir> "<counters>" [bench args...]
#   e.g. bash tools/pmc_pass.sh gpurun_out/tcc_cfg5k "TCC_HIT_sum TCC_MISS_sum" --workload cfg5 --bitstar-knn
# Counter limits per pass (rocprofv3 does not split): 8 SQ_, 4 TCC_, 4 TCP_, 2 TA_, 2 TD_, 2 GRBM_.
set -u
out=$1; ctrs=$2; shift 2
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p "$out"
timeout -s KILL 150 rocprofv3 --pmc $ctrs -d "$out" -o pmc --output-format csv -- \
    python bench.py --steps 2 --warmup 1 --no-cpu-baseline --single-query-reps 0 --rrt-iters 0 --no-extras \
    --workloads none --detail "" "$@" > "$out/bench.log" 2>&1
