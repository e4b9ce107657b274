#!/bin/bash
# tree-sharded cfg3 at N=1 (driver-style line), the shard / large-k GPU tests, and the RRT* k line
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
out=gpurun_out/$1; mkdir -p "$out"
fatal() { case $1 in 124|134|137|139) return 0;; esac; return 1; }
timeout -k 10 400 python -u -m pytest tests/test_shard_gloo.py tests/test_gpu_large_k.py -m gpu -x -q --timeout 200 --timeout-method thread > "$out/pytest.log" 2>&1
rc=$?; tail -2 "$out/pytest.log"; if fatal $rc; then exit 1; fi
f="$out/tree.json"
timeout -k 10 300 python -u bench.py --partition tree --steps 5 --warmup 2 --no-cpu-baseline --no-extras --single-query-reps 0 --rrt-iters 0 > "$f" 2> "$f.err"
rc=$?; if fatal $rc; then echo "tree rc=$rc"; tail -5 "$f.err"; exit 1; fi
cut -c1-900 "$f"; tail -2 "$f.err"
f="$out/rrtstar.json"
timeout -k 10 300 python -u bench.py --steps 2 --warmup 1 --no-cpu-baseline --single-query-reps 0 --rrt-iters 0 > "$f" 2> "$f.err"
rc=$?; if fatal $rc; then echo "rrtstar rc=$rc"; tail -3 "$f.err"; exit 1; fi
python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('rrt_star_knn', d.get('rrt_star_knn'))" "$f"
args="--steps 6 --warmup 2 --no-cpu-baseline --no-extras --single-query-reps 0 --rrt-iters 0"
for r in 1 2; do for v in 1 0; do
  f="$out/rc$v.$r.json"
  OMPL_GPU_SUPER_RECHECK=$v timeout -k 10 300 python -u bench.py $args > "$f" 2> "$f.err"
  rc=$?; if fatal $rc; then echo "rc=$rc"; tail -3 "$f.err"; exit 1; fi
  python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=d['roofline']; print(sys.argv[1].split('/')[-1], round(d['value']/1e6,2), 'step_ms', round(d['ms_per_step'],4), 'walk_ms', round(r['kernel_ms'],4), 'pairs', r['algorithmic'][:10])" "$f"
done; done
