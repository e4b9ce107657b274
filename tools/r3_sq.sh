#!/bin/bash
# single-query stream: GPU tests, then the extras bench line (single query at 10^6 / 10^7, RRT device)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
out=gpurun_out/$1; mkdir -p "$out"
fatal() { case $1 in 124|134|137|139) return 0;; esac; return 1; }
timeout -k 10 400 python -u -m pytest tests/test_gpu_stream32.py tests/test_gpu_nn.py tests/test_gpu_rrt_demo.py tests/test_gpu_batch.py -m gpu -x -q --timeout 200 --timeout-method thread > "$out/pytest.log" 2>&1
rc=$?; tail -2 "$out/pytest.log"; if fatal $rc; then exit 1; fi
f="$out/sq.json"
timeout -k 10 300 python -u bench.py --steps 2 --warmup 1 --no-cpu-baseline --rrt-star-queries 0 > "$f" 2> "$f.err"
rc=$?; if fatal $rc; then echo "rc=$rc"; tail -3 "$f.err"; exit 1; fi
python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); [print(k, json.dumps(d.get(k))[:300]) for k in ('single_query','single_query_1e7','rrt_device')]" "$f"
