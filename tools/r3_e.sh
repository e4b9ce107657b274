#!/bin/bash
# round-3 GPU step: stream / PRM / kNN parity, then the single-query stream at 10^7 with the
# split form on / off (OMPL_GPU_STREAM_SPLIT).  usage: bash tools/r3_e.sh <tag>
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
out=gpurun_out/$1; mkdir -p "$out"
fatal() { case $1 in 124|134|137|139) return 0;; esac; return 1; }
timeout -k 10 400 python -u -m pytest tests/test_gpu_stream32.py tests/test_gpu_prm.py tests/test_gpu_nn.py -m gpu -x -q \
    --timeout 200 --timeout-method thread > "$out/pytest_p.log" 2>&1
rc=$?; tail -2 "$out/pytest_p.log"; if [ $rc != 0 ]; then echo "pytest rc=$rc"; grep -E "FAIL|Error" "$out/pytest_p.log" | head; exit 1; fi
a="--steps 1 --warmup 1 --no-cpu-baseline --single-query-reps 200 --rrt-iters 0 --rrt-star-queries 0"
for r in 1 2; do for v in 1 0; do
  f="$out/sq_split$v.$r.json"
  OMPL_GPU_SPLIT_MIN=${SPLIT_MIN:-4194304} OMPL_GPU_STREAM_SPLIT=$v timeout -k 10 300 python -u bench.py $a > "$f" 2> "$f.err"
  rc=$?; if fatal $rc; then echo "sq rc=$rc"; tail -3 "$f.err"; exit 1; fi
  python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[1].split('/')[-1], json.dumps(d.get('single_query'))[:200], json.dumps(d.get('single_query_1e7'))[:200])" "$f"
done; done
