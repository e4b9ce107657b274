#!/bin/bash
# Run on the GPU box via gpurun: GPU tests, smoke, bench.  Each GPU step has its own time
# limit; after a crash / timeout (exit >= 124 or signal) nothing further touches the GPU.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
step() {  # name timeout cmd...
    local name=$1 to=$2; shift 2
    echo "=== $name: $*"
    timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1
    local rc=$?
    echo "=== $name rc=$rc"
    tail -n 25 "gpurun_out/$name.log"
    if [ $rc -ge 124 ] || [ $rc -gt 1 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
    return 0
}
MODE=${1:-all}
if [ "$MODE" = all ] || [ "$MODE" = test ]; then
    step pytest_gpu 900 python -m pytest tests -m gpu -x -q -p no:cacheprovider
    step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
fi
if [ "$MODE" = all ] || [ "$MODE" = bench ]; then
    step bench 600 python bench.py
fi
if [ "$MODE" = all ] || [ "$MODE" = prof ]; then
    TAG=${2:-r1}
    step prof_trace 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$TAG -o trace --output-format csv -- python bench.py --steps 3 --warmup 1 --no-cpu-baseline
    step prof_fetch 600 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/prof_$TAG -o pmc_fetch --output-format csv -- python bench.py --steps 2 --warmup 1 --no-cpu-baseline
    step prof_write 600 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/prof_$TAG -o pmc_write --output-format csv -- python bench.py --steps 2 --warmup 1 --no-cpu-baseline
fi
