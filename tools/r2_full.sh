#!/bin/bash
# GPU box: every -m gpu test, smoke, the default bench line, then the kernel trace and the
# FETCH_SIZE / WRITE_SIZE passes of the headline workload.  Each GPU step has its own limit and
# nothing further touches the GPU after a failure.
# usage: bash tools/r2_full.sh <tag>   -> gpurun_out/<tag>/
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
tag=${1:-r2_full}; out=gpurun_out/$tag; mkdir -p "$out"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 200 --timeout-method thread \
    > "$out/pytest.log" 2>&1 || { tail -40 "$out/pytest.log"; exit 1; }
tail -3 "$out/pytest.log"
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$out/smoke.log" 2>&1 || { tail -20 "$out/smoke.log"; exit 1; }
tail -1 "$out/smoke.log"
timeout -k 10 500 python -u bench.py > "$out/bench.json" 2> "$out/bench.err" || { tail -20 "$out/bench.err"; exit 1; }
cut -c1-600 "$out/bench.json"
bash tools/prof_workload.sh cfg3 "${tag}_cfg3" || exit $?
echo done
