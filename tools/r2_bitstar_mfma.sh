#!/bin/bash
# GPU box: the BIT* batch-sampling tests, then the MFMA brute-force probe (kernel trace) at 10^7 states.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
out=gpurun_out/${1:-r2_bm}; mkdir -p "$out"
timeout -k 10 300 python -u -m pytest tests/test_gpu_bitstar.py -m gpu -x -v -p no:cacheprovider --timeout 120 \
    --timeout-method thread > "$out/pytest.log" 2>&1 || { tail -40 "$out/pytest.log"; exit 1; }
tail -3 "$out/pytest.log"
timeout -k 10 120 ./tools/bin/mfma_probe 10000000 8192 0.1528 > "$out/mfma.json" || exit $?
cat "$out/mfma.json"
timeout -k 10 180 rocprofv3 --kernel-trace --stats -d "$out/mfma_trace" -o trace --output-format csv -- \
    ./tools/bin/mfma_probe 10000000 8192 0.1528 > "$out/mfma_trace.log" 2>&1 || exit $?
echo done
