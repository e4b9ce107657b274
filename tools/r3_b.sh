#!/bin/bash
# round-3 GPU step: the GPU test suite, the k-d build probe, then one rocprofv3 exit-crash
# isolation run (last: a segfault at exit ends the call).  usage: bash tools/r3_b.sh <tag> <iso>
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
out=gpurun_out/$1; mkdir -p "$out"
fatal() { case $1 in 124|134|137|139) return 0;; esac; return 1; }
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > "$out/pytest.log" 2>&1
rc=$?; tail -3 "$out/pytest.log"; if fatal $rc; then echo "pytest rc=$rc"; exit 1; fi
timeout -k 10 200 python -u tools/build_probe.py > "$out/build.json" 2> "$out/build.err"
rc=$?; cat "$out/build.json"; tail -2 "$out/build.err"; if fatal $rc; then echo "build rc=$rc"; exit 1; fi
args="--steps 6 --warmup 2 --no-cpu-baseline --no-extras --single-query-reps 0 --rrt-iters 0"
for r in 1 2; do
  for v in ${LBV-0 1 2 3}; do
    OMPL_GPU_TILE_LB=$v timeout -k 10 200 python -u bench.py $args > "$out/lb${v}_$r.json" 2>/dev/null
    rc=$?; if fatal $rc; then echo "lb$v rc=$rc"; exit 1; fi
    python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=d['roofline']; print(sys.argv[1].split('/')[-1], round(d['value']/1e6,2), 'walk_ms', round(r['kernel_ms'],4), 'pairs', r['algorithmic'][:10], 'reruns', d['fast_path'])" "$out/lb${v}_$r.json"
  done
done
case ${2:-none} in
rrt) a="--rrt-iters 2000 --single-query-reps 0 --no-extras";;
sq) a="--rrt-iters 0 --single-query-reps 200 --no-extras";;
*) exit 0;;
esac
OMPL_AMD_MAPS=$out/maps.txt timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$out/iso" -o trace --output-format csv \
    -- python bench.py --steps 2 --warmup 1 --no-cpu-baseline $a > "$out/iso.log" 2>&1
rc=$?; echo "iso($2) rc=$rc"; exit $rc
