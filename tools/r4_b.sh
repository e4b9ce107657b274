#!/bin/bash
# round-4 walk A/B: parity tests on each variant build (var 7 scan cascade, 8 dynamic tile masks,
# 9 both), then alternating bench runs: cfg3 (headline walk) and cfg5 (radius walk 7/8 waves)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
out=gpurun_out/r4b; mkdir -p "$out"
T="tests/test_gpu_nn.py tests/test_gpu_cull.py"
for v in ${VARS:-7 8 9}; do
  OMPL_GPU_LIB=tools/probe_lib/libompl_gpu_var$v.so timeout -k 10 300 python -u -m pytest $T -m gpu -x -q --timeout 200 \
      --timeout-method thread > "$out/pytest_v$v.log" 2>&1
  rc=$?; echo "var$v: $(tail -1 "$out/pytest_v$v.log")"; if [ $rc != 0 ]; then echo "var$v pytest rc=$rc"; exit 1; fi
done
bash tools/ab_bench.sh "cfg3" "${VARS:-7 8 9}" 3 || exit 1
[ "${RADIUS:-1}" = 1 ] && bash tools/ab_bench.sh "cfg5" "5 6" 2
