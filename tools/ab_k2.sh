#!/bin/bash
# A/B on the GPU box: the product library vs variant builds tools/bin/libompl_gpu_var{5,6}.so
# (make -C ompl_amd/csrc variant VARIANT=n VAR_OUT=../../tools/bin/libompl_gpu_var<n>.so).  Used for
# the walk list length (k+2 product vs k+3 / k+4 variants; results in profiles/r2_ab_k2/).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
out=gpurun_out/ab_k2; mkdir -p "$out"
args="--workload ${WL:-cfg3} --steps 10 --warmup 3 --no-cpu-baseline --no-extras --single-query-reps 0 --rrt-iters 0"
vars=${VARS:-5 6}
for r in 1 2; do
  timeout -k 10 200 python -u bench.py $args > "$out/p_$r.json" 2>/dev/null || exit 1
  for v in $vars; do
    OMPL_GPU_LIB=tools/bin/libompl_gpu_var$v.so timeout -k 10 200 python -u bench.py $args > "$out/v${v}_$r.json" 2>/dev/null || exit 1
  done
done
for f in "$out"/*.json; do
  python - "$f" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(sys.argv[1].split("/")[-1], round(d["value"] / 1e6, 2), "M/s step", round(d["ms_per_step"], 4), "walk", round(d["roofline"]["kernel_ms"], 4), "phases", d["phase_ms"])
PY
done
