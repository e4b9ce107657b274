#!/bin/bash
# Round-3 closing GPU run: every -m gpu test, smoke, the default bench line (with its CPU
# baseline), the cfg4 profiles (the chain scan's chunk count changed) and the k-d build trace.
# Each GPU step has its own limit; a failure ends the call.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
out=gpurun_out/r3_final2; mkdir -p "$out"
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread \
    > "$out/pytest.log" 2>&1 || { tail -30 "$out/pytest.log"; exit 1; }
tail -2 "$out/pytest.log"
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$out/smoke.log" 2>&1 || { tail -20 "$out/smoke.log"; exit 1; }
tail -1 "$out/smoke.log"
timeout -k 10 500 python -u bench.py > "$out/bench.json" 2> "$out/bench.err" || { tail -20 "$out/bench.err"; exit 1; }
cut -c1-300 "$out/bench.json"
bash tools/prof_workload.sh cfg4 r3f2_cfg4 || { echo "prof cfg4 rc=$?"; exit 1; }
timeout -k 10 400 python -u bench.py --workload cfg4 --steps 5 --warmup 2 --single-query-reps 0 --rrt-iters 0 > "$out/cfg4.json" 2> "$out/cfg4.err" || { tail -5 "$out/cfg4.err"; exit 1; }
cut -c1-300 "$out/cfg4.json"
mkdir -p gpurun_out/r3f2_build
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/r3f2_build -o trace --output-format csv -- \
  python tools/build_probe.py > gpurun_out/r3f2_build/build.log 2>&1 || { echo "build rc=$?"; exit 1; }
grep '^{' gpurun_out/r3f2_build/build.log
echo done
