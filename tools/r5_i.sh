#!/bin/bash
# Round-5 GPU step I: chain motion parity after a motion-kernel change, then cfg4 (PRM* chain) twice.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
out=gpurun_out/r5_i; mkdir -p "$out"
timeout -k 10 700 python -u -m pytest tests/test_gpu_motion.py tests/test_gpu_prm.py tests/test_gpu_chain_boundary.py tests/test_gpu_spaces.py \
    tests/test_gpu_fullsize.py::test_cfg4_prm_batch_1_vs_sequential_loop tests/test_gpu_fullsize.py::test_cfg4_prm_batch_2_tail_vs_sequential_loop \
    -m gpu -x -q --timeout 400 --timeout-method thread > "$out/pytest.log" 2>&1
rc=$?
tail -3 "$out/pytest.log"
[ $rc -eq 0 ] || { grep -n "FAIL\|Error\|error" "$out/pytest.log" | head -30; exit 1; }
for r in 1 2; do
  timeout -k 10 300 python -u bench.py --workload cfg4 --steps 10 --warmup 3 --workloads none --no-extras --no-cpu-baseline \
      > "$out/cfg4_$r.json" 2> "$out/cfg4_$r.err" || { tail -30 "$out/cfg4_$r.err"; exit 1; }
  python - "$out/cfg4_$r.json" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print("cfg4", d["value"], d["ms_per_step"], json.dumps(d["phase_ms"]), d["roofline"]["kernel_ms"])
PY
done
mkdir -p "$out/prof"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$out/prof" -o cfg4 --output-format csv -- python -u bench.py --workload cfg4 --steps 10 --warmup 3 \
    --workloads none --no-extras --no-cpu-baseline > "$out/prof.log" 2>&1 || { tail -20 "$out/prof.log"; exit 1; }
find "$out/prof" -name "*kernel_stats.csv" | head -1 | xargs -I{} sh -c 'head -8 {}'
timeout -k 10 400 python -u -m pytest tests/test_gpu_rrtstar.py -m gpu -x -q --timeout 240 --timeout-method thread > "$out/pytest_rrtstar.log" 2>&1 || { tail -20 "$out/pytest_rrtstar.log"; exit 1; }
tail -1 "$out/pytest_rrtstar.log"
timeout -k 10 500 python -u bench.py --steps 5 --warmup 2 --workloads rrt_star --no-extras --single-query-reps 0 \
    --rrt-iters 0 --no-cpu-baseline > "$out/rrtstar.json" 2> "$out/rrtstar.err" || { tail -30 "$out/rrtstar.err"; exit 1; }
python - "$out/rrtstar.json" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
w = d["workloads"]["rrt_star"]
print("rrt_star", w["value"], w["ms_per_step"], json.dumps(w["phase_ms"]))
PY
