#!/bin/bash
# Round-5 GPU step D: the RRT* workload line alone (headline cfg3 without extras), a rocprof trace.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
out=gpurun_out/r5_d; mkdir -p "$out"
timeout -k 10 400 python -u bench.py --steps 5 --warmup 2 --workloads rrt_star,cfg3_strong,cfg3_tree --no-extras --single-query-reps 0 \
    --rrt-iters 0 > "$out/bench.json" 2> "$out/bench.err" || { tail -30 "$out/bench.err"; exit 1; }
python - "$out/bench.json" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(json.dumps(d["workloads"]["rrt_star"], indent=1)[:4000])
print("headline", d["value"], d["ms_per_step"])
for k in ("cfg3_strong", "cfg3_tree"):
    w = d["workloads"][k]
    print(k, w["value"], w["ms_per_step"], w["scaling"])
PY
