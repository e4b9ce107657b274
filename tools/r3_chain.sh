#!/bin/bash
# cfg4 A/B of the chain screen's link order (OMPL_GPU_CHAIN_ORDER 0 / 1), then the PRM* tests.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
out=gpurun_out/$1; mkdir -p "$out"
fatal() { case $1 in 124|134|137|139) return 0;; esac; return 1; }
timeout -k 10 400 python -u -m pytest ${TESTS:-tests/test_gpu_prm.py tests/test_gpu_nn.py tests/test_gpu_large_k.py} -m gpu -x -q --timeout 200 --timeout-method thread > "$out/pytest.log" 2>&1
rc=$?; tail -2 "$out/pytest.log"; if fatal $rc; then exit 1; fi
args="--workload cfg4 --steps 4 --warmup 1 --no-cpu-baseline --no-extras"
for r in 1 2; do for v in ${VARS:-o1w4 o1w1 o0w4}; do
  f="$out/$v.$r.json"
  o=${v:1:1}; wb=${v:3:1}
  OMPL_GPU_CHAIN_ORDER=$o OMPL_GPU_CHAIN_WPB=$wb timeout -k 10 300 python -u bench.py $args > "$f" 2> "$f.err"
  rc=$?; if fatal $rc; then echo "rc=$rc"; tail -3 "$f.err"; exit 1; fi
  python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=d['roofline']; print(sys.argv[1].split('/')[-1], round(d['value']/1e6,3), 'M/s step_ms', round(d['ms_per_step'],3), 'kern_ms', round(r['kernel_ms'],3), r['kernel'], d['phase_ms'])" "$f"
done; done
f="$out/rrtstar.json"
timeout -k 10 300 python -u bench.py --steps 2 --warmup 1 --no-cpu-baseline --single-query-reps 0 --rrt-iters 0 > "$f" 2> "$f.err"
rc=$?; if fatal $rc; then echo "rrtstar rc=$rc"; tail -3 "$f.err"; exit 1; fi
python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('rrt_star_knn', d.get('rrt_star_knn'), 'index', d.get('index'))" "$f"
