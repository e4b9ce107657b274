#!/bin/bash
# Round-5 GPU step L: chain parity, then the cfg4 kernel profile (tools/r5_k.sh).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
out=gpurun_out/${1:-r5_l}; mkdir -p "$out"
timeout -k 10 700 python -u -m pytest tests/test_gpu_motion.py tests/test_gpu_prm.py tests/test_gpu_chain_boundary.py tests/test_gpu_spaces.py \
    tests/test_gpu_fullsize.py::test_cfg4_prm_batch_1_vs_sequential_loop -m gpu -x -q --timeout 400 --timeout-method thread > "$out/pytest.log" 2>&1
rc=$?
tail -1 "$out/pytest.log"
[ $rc -eq 0 ] || { grep -n "FAIL\|Error\|error" "$out/pytest.log" | head -30; exit 1; }
bash tools/r5_k.sh "${1:-r5_l}"
