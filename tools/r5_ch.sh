#!/bin/bash
# Round-5 GPU step CH: chain parity (product build), then one cfg4 kernel profile per chain-motion
# form: the product (register form, 4 waves per SIMD) and vlib/ variants (rt = the runtime-width
# form with the side pre-test, w2 / w5 = the register form at 2 / 5 waves per SIMD).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
out=gpurun_out/${1:-r5_ch}; mkdir -p "$out"
timeout -k 10 700 python -u -m pytest tests/test_gpu_motion.py tests/test_gpu_prm.py tests/test_gpu_chain_boundary.py tests/test_gpu_spaces.py \
    tests/test_gpu_fullsize.py::test_cfg4_prm_batch_1_vs_sequential_loop tests/test_gpu_fullsize.py::test_cfg4_prm_batch_2_tail_vs_sequential_loop \
    -m gpu -x -q --timeout 400 --timeout-method thread > "$out/pytest.log" 2>&1
rc=$?
tail -1 "$out/pytest.log"
[ $rc -eq 0 ] || { grep -n "FAIL\|Error\|error" "$out/pytest.log" | head -30; exit 1; }
for v in prod ${VARS:-rt w2 w5}; do
  mkdir -p "$out/$v"
  if [ $v = prod ]; then unset OMPL_GPU_LIB; else export OMPL_GPU_LIB=vlib/libompl_gpu_$v.so; fi
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$out/$v" -o cfg4 --output-format csv -- python -u bench.py --workload cfg4 --steps 10 --warmup 3 \
      --workloads none --no-extras --no-cpu-baseline > "$out/$v/prof.log" 2>&1 || { tail -20 "$out/$v/prof.log"; exit 1; }
  echo "== $v $(tail -1 $out/$v/prof.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'])")"
  python tools/kstats.py "$(find "$out/$v" -name "*kernel_stats.csv" | head -1)" 4
done
