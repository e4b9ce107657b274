#!/bin/bash
# round-3 GPU step: the new parity tests, then a kernel trace of the k-d build at 10^6 / 10^7.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
out=gpurun_out/$1; mkdir -p "$out"
fatal() { case $1 in 124|134|137|139) return 0;; esac; return 1; }
timeout -k 10 600 python -u -m pytest ${TESTS:-tests} -m gpu -x -v --timeout 300 --timeout-method thread > "$out/pytest.log" 2>&1
rc=$?; grep -E "PASS|FAIL|ERROR|passed|failed" "$out/pytest.log" | tail -15; if fatal $rc; then echo "pytest rc=$rc"; exit 1; fi
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$out/build" -o trace --output-format csv -- python tools/build_probe.py \
    > "$out/build.log" 2>&1
rc=$?; grep '^{' "$out/build.log"; echo "build trace rc=$rc"; exit $rc
