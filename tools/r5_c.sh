#!/bin/bash
# Round-5 GPU step C: RRT* batch parity, then the whole GPU suite.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
out=gpurun_out/r5_c; mkdir -p "$out"
timeout -k 10 600 python -u -m pytest tests/test_gpu_rrtstar.py -m gpu -v -x -p no:cacheprovider --timeout 300 \
    --timeout-method thread > "$out/rrtstar.log" 2>&1; rc=$?
grep -E "PASS|FAIL|ERROR|passed|failed|^E " "$out/rrtstar.log" | head -40
[ $rc -eq 0 ] || exit $rc
timeout -k 10 1200 python -u -m pytest tests -m gpu -q -x -p no:cacheprovider --timeout 400 --timeout-method thread \
    > "$out/pytest.log" 2>&1; rc=$?
tail -5 "$out/pytest.log"
exit $rc
