#!/bin/bash
# Round-3: the extras trace that crashed at exit in round 2 (rrt_persistent_kernel,
# knn_stream32_kernel at 1e6 and 1e7, the large-k select), with the teardown fix, then the
# FETCH_SIZE / WRITE_SIZE passes of the same run.  usage: bash tools/r3_extras.sh <tag>
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
out=gpurun_out/${1:-r3_extras}
mkdir -p "$out"
args="--steps 2 --warmup 1 --no-cpu-baseline --single-query-reps 200 --rrt-iters 2000"
OMPL_AMD_MAPS=$out/maps.txt timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$out" -o trace --output-format csv \
    -- python bench.py $args > "$out/trace.log" 2>&1 || { echo "trace rc=$?"; exit 1; }
timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE -d "$out" -o pmc_fetch --output-format csv -- python bench.py $args \
    > "$out/fetch.log" 2>&1 || { echo "fetch rc=$?"; exit 1; }
timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE -d "$out" -o pmc_write --output-format csv -- python bench.py $args \
    > "$out/write.log" 2>&1 || { echo "write rc=$?"; exit 1; }
grep '^{' "$out/trace.log" | cut -c1-400
echo done
