#!/bin/bash
# Round-5 closing GPU run: every -m gpu test, smoke, then the default bench line (every config,
# the strong / tree-sharded cfg3 forms and RRT* in its workloads record, with CPU baselines).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
out=gpurun_out/r5_final; mkdir -p "$out"
timeout -k 10 700 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 300 --timeout-method thread \
    > "$out/pytest.log" 2>&1 || { tail -30 "$out/pytest.log"; exit 1; }
tail -2 "$out/pytest.log"
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$out/smoke.log" 2>&1 || { tail -20 "$out/smoke.log"; exit 1; }
tail -1 "$out/smoke.log"
timeout -k 10 420 python -u bench.py --steps 20 --warmup 5 > "$out/bench.json" 2> "$out/bench.err" || { tail -20 "$out/bench.err"; exit 1; }
cut -c1-300 "$out/bench.json"
echo done
