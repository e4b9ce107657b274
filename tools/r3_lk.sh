#!/bin/bash
# large-k: GPU tests, then the k = 6,169 probe timed and under a kernel trace
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
out=gpurun_out/$1; mkdir -p "$out"
fatal() { case $1 in 124|134|137|139) return 0;; esac; return 1; }
timeout -k 10 400 python -u -m pytest tests/test_gpu_large_k.py tests/test_gpu_nn.py -m gpu -x -q --timeout 200 --timeout-method thread > "$out/pytest.log" 2>&1
rc=$?; tail -2 "$out/pytest.log"; if fatal $rc; then exit 1; fi
timeout -k 10 200 python -u tools/large_k_probe.py 10 > "$out/probe.json" 2> "$out/probe.err"
rc=$?; cat "$out/probe.json"; if fatal $rc; then tail -3 "$out/probe.err"; exit 1; fi
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$out/trace" -o trace --output-format csv -- python tools/large_k_probe.py 5 > "$out/trace.log" 2>&1
rc=$?; echo "trace rc=$rc"; exit $rc
