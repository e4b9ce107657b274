#!/bin/bash
# round-3 kernel A/B: the walk parity tests on the product library and on each variant build
# (tools/probe_lib/libompl_gpu_var<n>.so), then alternating bench runs (tools/ab_bench.sh).
# usage: bash tools/r3_ab.sh <tag> "<variants>" "<workloads>" [reps]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
out=gpurun_out/$1; mkdir -p "$out"
fatal() { case $1 in 124|134|137|139) return 0;; esac; return 1; }
T=${TESTS:-tests/test_gpu_nn.py tests/test_gpu_cull.py}
timeout -k 10 300 python -u -m pytest $T -m gpu -x -q --timeout 200 --timeout-method thread > "$out/pytest_p.log" 2>&1
rc=$?; tail -2 "$out/pytest_p.log"; if [ $rc != 0 ]; then echo "product pytest rc=$rc"; exit 1; fi
for v in $2; do
  OMPL_GPU_LIB=tools/probe_lib/libompl_gpu_var$v.so timeout -k 10 300 python -u -m pytest $T -m gpu -x -q --timeout 200 \
      --timeout-method thread > "$out/pytest_v$v.log" 2>&1
  rc=$?; tail -2 "$out/pytest_v$v.log"; if [ $rc != 0 ]; then echo "var$v pytest rc=$rc"; exit 1; fi
done
bash tools/ab_bench.sh "$3" "$2" "${4:-3}"
