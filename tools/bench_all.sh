#!/bin/bash
# Run bench.py on every workload (GPU box, via gpurun); each run under its own time limit,
# stopping at the first failure.  Output: gpurun_out/bench_<workload>.log
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for w in ${@:-cfg3 cfg2 cfg4 cfg5}; do
    echo "=== $w"
    timeout -k 10 400 python bench.py --workload $w > gpurun_out/bench_$w.log 2>&1
    rc=$?
    tail -c 2500 gpurun_out/bench_$w.log
    [ $rc -ne 0 ] && { echo "stopping after $w (rc=$rc)"; exit $rc; }
done
exit 0
