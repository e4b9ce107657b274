#!/bin/bash
# single-query A/B: chunked (0) vs persistent k = 1 stream with 1024 / 2048 / 4096 blocks
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
out=gpurun_out/$1; mkdir -p "$out"
fatal() { case $1 in 124|134|137|139) return 0;; esac; return 1; }
for r in 1 2; do for b in 1024 2048 4096; do
  f="$out/sq$b.$r.json"
  OMPL_GPU_S1_BLOCKS=$b timeout -k 10 300 python -u bench.py --steps 1 --warmup 1 --no-cpu-baseline --rrt-star-queries 0 --rrt-iters 0 --single-query-reps 400 > "$f" 2> "$f.err"
  rc=$?; if fatal $rc; then echo "rc=$rc"; tail -3 "$f.err"; exit 1; fi
  python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); a=d['single_query']; b=d['single_query_1e7']; print(sys.argv[1].split('/')[-1], '1e6', round(a['kernel_us'],2), round(a['queries_per_s']), '1e7', round(b['kernel_us'],2), round(b['roofline']['frac'],3), round(b['queries_per_s']))" "$f"
done; done
