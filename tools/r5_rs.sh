#!/bin/bash
# Round-5 GPU step RS: RRT* parity tests, then the RRT* workload line (10 timed batches).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
out=gpurun_out/${1:-r5_rs}; mkdir -p "$out"
timeout -k 10 400 python -u -m pytest tests/test_gpu_rrtstar.py tests/test_rrtstar_cost.py -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > "$out/pytest.log" 2>&1
rc=$?; tail -2 "$out/pytest.log"; [ $rc -eq 0 ] || { grep -n "FAIL\|Error" "$out/pytest.log" | head -20; exit 1; }
timeout -k 10 400 python -u bench.py --steps 10 --warmup 5 --workloads rrt_star --no-extras --single-query-reps 0 \
    --rrt-iters 0 --no-cpu-baseline > "$out/bench.json" 2> "$out/bench.err" || { tail -30 "$out/bench.err"; exit 1; }
python - "$out/bench.json" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
w = d["workloads"]["rrt_star"]
print("rrt_star", w["value"], w["ms_per_step"], json.dumps(w["phase_ms"])[:300], json.dumps(w["per_step"]))
PY
