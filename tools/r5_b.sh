#!/bin/bash
# Round-5 GPU step B: the glibc sin / cos restatement on the device; chain parity tests; cfg4 bench.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
out=gpurun_out/r5_b; mkdir -p "$out"
timeout -k 10 120 python tools/libm_probe.py 2000000 > "$out/libm.json" 2>&1 || { tail -20 "$out/libm.json"; exit 1; }
cat "$out/libm.json"
timeout -k 10 900 python -u -m pytest tests/test_gpu_chain_boundary.py tests/test_gpu_spaces.py tests/test_gpu_prm.py \
    tests/test_gpu_motion.py tests/test_gpu_fullsize.py -m gpu -q -p no:cacheprovider --timeout 400 --timeout-method thread \
    > "$out/pytest.log" 2>&1; rc=$?
grep -E "FAIL|ERROR|passed|failed" "$out/pytest.log" | tail -30
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --workload cfg4 --steps 10 --warmup 3 --no-cpu-baseline --workloads none \
    > "$out/cfg4.json" 2> "$out/cfg4.err" || { tail -20 "$out/cfg4.err"; exit 1; }
cut -c1-400 "$out/cfg4.json"
