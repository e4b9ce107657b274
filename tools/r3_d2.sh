#!/bin/bash
# round-3 GPU step: radius / kNN parity tests on the product and variant libraries, the cfg5
# A/B, then a kernel trace of the cfg4 (causal PRM* on the chain) step.  usage: bash tools/r3_d2.sh <tag> "<variants>"
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
out=gpurun_out/$1; mkdir -p "$out"
TESTS="tests/test_gpu_batch.py tests/test_gpu_fullsize.py tests/test_gpu_bitstar.py tests/test_gpu_index.py tests/test_gpu_nn.py" \
  bash tools/r3_ab.sh "$1" "$2" "cfg5" 2 || exit 1
a="--workload cfg4 --steps 3 --warmup 1 --no-cpu-baseline --no-extras --single-query-reps 0 --rrt-iters 0"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$out/cfg4" -o trace --output-format csv -- python bench.py $a \
  > "$out/cfg4_trace.log" 2>&1 || { echo "cfg4 trace rc=$?"; exit 1; }
python - "$out/cfg4/trace_kernel_stats.csv" <<'PY'
import csv, sys, re
for r in list(csv.DictReader(open(sys.argv[1])))[:16]:
    n = re.sub(r'ompl_amd::|\(anonymous namespace\)::|rocprim::ROCPRIM_400200_NS::detail::', '', r['Name'])[:80]
    print(f"{int(r['Calls']):5d} {float(r['AverageNs'])/1e3:10.1f}us {float(r['Percentage']):6.2f}% {n}")
PY
