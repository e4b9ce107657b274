#!/bin/bash
# Round-5 GPU step A: device libm vs glibc, the new full-size / PRM / SO3 / chain-edge parity tests.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
out=gpurun_out/r5_a; mkdir -p "$out"
timeout -k 10 120 python tools/libm_probe.py 2000000 > "$out/libm.json" 2>&1 || { tail -20 "$out/libm.json"; exit 1; }
cat "$out/libm.json"
timeout -k 10 900 python -u -m pytest tests/test_gpu_chain_boundary.py tests/test_gpu_spaces.py tests/test_gpu_prm.py \
    tests/test_gpu_fullsize.py -m gpu -v -p no:cacheprovider --timeout 400 --timeout-method thread \
    > "$out/pytest.log" 2>&1; rc=$?
grep -E "PASS|FAIL|ERROR|passed|failed" "$out/pytest.log" | tail -60
exit $rc
