#!/bin/bash
# Round-5 GPU step V: the whole GPU suite, then the cfg4 kernel profile (tools/r5_k.sh).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
out=gpurun_out/${1:-r5_v}; mkdir -p "$out"
timeout -k 10 800 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > "$out/pytest.log" 2>&1
rc=$?
tail -2 "$out/pytest.log"
[ $rc -eq 0 ] || { grep -n "FAIL\|Error\|error" "$out/pytest.log" | head -30; exit 1; }
bash tools/r5_k.sh "${1:-r5_v}"
