#!/bin/bash
# k-d build A/B: median-partition global levels (OMPL_GPU_KD_PART=1, default) against one radix
# sort per level (0): parity tests, the build probe at 10^6 / 10^7 both ways, a kernel trace of
# the probe.  usage: bash tools/r3_part.sh <tag>
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
out=gpurun_out/$1; mkdir -p "$out"
timeout -k 10 500 python -u -m pytest ${TESTS:-tests/test_gpu_index.py tests/test_gpu_nn.py tests/test_gpu_fullsize.py tests/test_gpu_cull.py tests/test_gpu_batch.py} \
    -m gpu -x -q --timeout 300 --timeout-method thread > "$out/pytest.log" 2>&1
rc=$?; tail -2 "$out/pytest.log"; if [ $rc != 0 ]; then echo "pytest rc=$rc"; grep -E "FAIL|Error" "$out/pytest.log" | head; exit 1; fi
for v in 1 0; do
  OMPL_GPU_KD_PART=$v timeout -k 10 200 python -u tools/build_probe.py > "$out/build_part$v.json" 2> "$out/build_part$v.err"
  rc=$?; echo "part=$v $(cat $out/build_part$v.json)"; if [ $rc != 0 ]; then echo "build rc=$rc"; tail -3 "$out/build_part$v.err"; exit 1; fi
done
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$out/prof" -o run --output-format csv -- python3 -u tools/build_probe.py 10000000 > "$out/prof.log" 2>&1
rc=$?; echo "prof rc=$rc"
f=$(find "$out/prof" -name '*kernel_stats.csv' | head -1); [ -n "$f" ] && cp "$f" "$out/trace_kernel_stats.csv"
exit $rc
