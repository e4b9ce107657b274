#!/bin/bash
# Round-5 GPU step E: the whole GPU suite after the source cleanup, then the RRT* / strong / tree
# workload lines (tools/r5_d.sh).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
out=gpurun_out/r5_e; mkdir -p "$out"
timeout -k 10 780 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread > "$out/pytest.log" 2>&1
rc=$?
tail -5 "$out/pytest.log"
[ $rc -eq 0 ] || { grep -n "FAIL\|Error\|error" "$out/pytest.log" | head -30; exit 1; }
bash tools/r5_d.sh
