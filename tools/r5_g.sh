#!/bin/bash
# Round-5 GPU step G: the headline walk's event counters (probe build) and the RRT* line.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
out=gpurun_out/r5_g; mkdir -p "$out"
OMPL_GPU_LIB=tools/probe_lib/libompl_gpu_probe.so timeout -k 10 300 python -u tools/walk_probe.py --k 10 > "$out/walk_probe.json" 2> "$out/walk_probe.err" || { tail -20 "$out/walk_probe.err"; exit 1; }
cat "$out/walk_probe.json"
timeout -k 10 500 python -u bench.py --steps 5 --warmup 2 --workloads rrt_star --no-extras --single-query-reps 0 \
    --rrt-iters 0 > "$out/bench.json" 2> "$out/bench.err" || { tail -30 "$out/bench.err"; exit 1; }
python - "$out/bench.json" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
w = d["workloads"]["rrt_star"]
print("rrt_star", w["value"], w["ms_per_step"], json.dumps(w["phase_ms"]), json.dumps(w["per_step"]))
PY
