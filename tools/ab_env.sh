#!/bin/bash
# A/B of run-time switches and variant libraries on one bench workload, alternating.
# usage: bash tools/ab_env.sh <tag> "<bench args>" <reps> "<setting>" ["<setting>" ...]
#   setting: "-" (product), "VAR=n" (tools/probe_lib/libompl_gpu_var<n>.so), or env assignments
#   ("OMPL_GPU_CHAIN_SHARE=0 OMPL_GPU_QSORT=0").  Prints each run's kernel / step / nn-phase times.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
tag=$1; args=$2; reps=$3; shift 3
out=gpurun_out/ab_$tag; mkdir -p "$out"
base="--steps 10 --warmup 3 --no-cpu-baseline --no-extras --single-query-reps 0 --rrt-iters 0 --workloads none"
for r in $(seq "$reps"); do
  i=0
  for s in "$@"; do
    i=$((i + 1))
    f="$out/s${i}_r$r.json"
    if [ "$s" = "-" ]; then
      timeout -k 10 300 python -u bench.py $args $base > "$f" 2> "$f.err" || { echo "setting $s rc=$?"; tail -3 "$f.err"; exit 1; }
    elif [ "${s#VAR=}" != "$s" ]; then
      OMPL_GPU_LIB=tools/probe_lib/libompl_gpu_var${s#VAR=}.so timeout -k 10 300 python -u bench.py $args $base > "$f" 2> "$f.err" || { echo "setting $s rc=$?"; tail -3 "$f.err"; exit 1; }
    else
      env $s timeout -k 10 300 python -u bench.py $args $base > "$f" 2> "$f.err" || { echo "setting $s rc=$?"; tail -3 "$f.err"; exit 1; }
    fi
  done
done
i=0
for s in "$@"; do
  i=$((i + 1))
  for f in "$out"/s${i}_r*.json; do
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=d['roofline']; print(sys.argv[2].ljust(34), 'value %.4g' % d['value'], 'step_ms %.4f' % d['ms_per_step'], 'kern_ms %.4f' % r['kernel_ms'], r['kernel'], 'phases', {k: round(v, 4) for k, v in d['phase_ms'].items()})" "$f" "$s"
  done
done
