#!/bin/bash
# Round-5 GPU step F: RRT* parity through the native cost logic (pipelined), then the RRT* /
# strong / tree workload lines.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
out=gpurun_out/r5_f; mkdir -p "$out"
timeout -k 10 400 python -u -m pytest tests/test_gpu_rrtstar.py -m gpu -x -v --timeout 240 --timeout-method thread > "$out/pytest.log" 2>&1
rc=$?
tail -5 "$out/pytest.log"
[ $rc -eq 0 ] || { grep -n "FAIL\|Error\|error" "$out/pytest.log" | head -30; exit 1; }
timeout -k 10 500 python -u bench.py --steps 5 --warmup 2 --workloads rrt_star,cfg3_strong,cfg3_tree --no-extras --single-query-reps 0 \
    --rrt-iters 0 > "$out/bench.json" 2> "$out/bench.err" || { tail -30 "$out/bench.err"; exit 1; }
python - "$out/bench.json" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
w = d["workloads"]["rrt_star"]
print("rrt_star", w["value"], w["ms_per_step"], json.dumps(w["phase_ms"]), w["cpu_baseline"]["value"] if w.get("cpu_baseline") else None)
print("headline", d["value"], d["ms_per_step"])
for k in ("cfg3_strong", "cfg3_tree"):
    w = d["workloads"][k]
    print(k, w["value"], w["ms_per_step"], w["scaling"], json.dumps(w["phase_ms"]))
PY
