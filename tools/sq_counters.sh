#!/bin/bash
# One rocprofv3 --pmc pass of SQ counters over a short bench run (no other trace domains).
# usage: bash tools/sq_counters.sh <outdir> [bench args...]
set -u
out=$1; shift
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD \
    SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY -d "$out" -o pmc_sq --output-format csv -- \
    python bench.py --steps 2 --warmup 1 --no-cpu-baseline --single-query-reps 0 --rrt-iters 0 --workloads none "$@"
