#!/bin/bash
# Kernel A/B on the GPU box: the product library and each variant build under
# tools/probe_lib/ (make -C ompl_amd/csrc variant VARIANT=n), alternating, on the given workloads;
# prints each run's walk-kernel time.  usage: bash tools/ab_bench.sh "cfg3 cfg5" "1 2" [reps]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
out=gpurun_out/ab; mkdir -p "$out"
wls=$1; vars=$2; reps=${3:-2}
args="--steps 5 --warmup 2 --no-cpu-baseline --no-extras --single-query-reps 0 --rrt-iters 0"
for r in $(seq "$reps"); do
  for w in $wls; do
    timeout -k 10 200 python -u bench.py --workload "$w" $args > "$out/${w}_p_$r.json" 2>/dev/null || exit 1
    for v in $vars; do
      OMPL_GPU_LIB=tools/probe_lib/libompl_gpu_var$v.so timeout -k 10 200 python -u bench.py --workload "$w" $args \
        > "$out/${w}_v${v}_$r.json" 2>/dev/null || exit 1
    done
  done
done
for f in "$out"/*.json; do
  echo "$(basename "$f") $(grep -o '"kernel_ms": [0-9.]*' "$f") $(grep -o '"ms_per_step": [0-9.]*' "$f")"
done
