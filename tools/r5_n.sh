#!/bin/bash
# Round-5 GPU step N: the chain motion kernel at 5 / 6 / 8 waves per SIMD (variant libraries in
# vlib/, OMPL_GPU_LIB), one cfg4 kernel profile each, after the product's.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
for w in ${VARS:-f2 f4 f6}; do
  out=gpurun_out/r5_o/$w; mkdir -p "$out/prof"
  OMPL_GPU_LIB=vlib/libompl_gpu_$w.so timeout -k 10 200 python -u -m pytest tests/test_gpu_motion.py -m gpu -x -q --timeout 150 \
      --timeout-method thread > "$out/pytest.log" 2>&1 || { tail -20 "$out/pytest.log"; exit 1; }
  echo "$w $(tail -1 $out/pytest.log)"
  OMPL_GPU_LIB=vlib/libompl_gpu_$w.so timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$out/prof" -o cfg4 --output-format csv -- \
      python -u bench.py --workload cfg4 --steps 10 --warmup 3 --workloads none --no-extras --no-cpu-baseline > "$out/prof.log" 2>&1 || { tail -20 "$out/prof.log"; exit 1; }
  python tools/kstats.py "$(find "$out/prof" -name "*kernel_stats.csv" | head -1)" 3
done
