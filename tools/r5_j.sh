#!/bin/bash
# Round-5 GPU step J: RRT* parity and the RRT* workload line (threaded native cost logic).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
out=gpurun_out/r5_j; mkdir -p "$out"
timeout -k 10 400 python -u -m pytest tests/test_gpu_rrtstar.py -m gpu -x -q --timeout 240 --timeout-method thread > "$out/pytest_rrtstar.log" 2>&1 || { tail -20 "$out/pytest_rrtstar.log"; exit 1; }
tail -1 "$out/pytest_rrtstar.log"
timeout -k 10 500 python -u bench.py --steps 5 --warmup 2 --workloads rrt_star --no-extras --single-query-reps 0 \
    --rrt-iters 0 > "$out/rrtstar.json" 2> "$out/rrtstar.err" || { tail -30 "$out/rrtstar.err"; exit 1; }
python - "$out/rrtstar.json" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
w = d["workloads"]["rrt_star"]
print("rrt_star", w["value"], w["ms_per_step"], json.dumps(w["phase_ms"]), json.dumps(w["per_step"]), w["cpu_baseline"]["value"])
PY
