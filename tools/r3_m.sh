#!/bin/bash
# round-3 measurement step: GPU tests, k-d build probe, then short bench lines (no CPU baseline):
# cfg3 x2, cfg5 radius, cfg5 BIT* kNN.  usage: bash tools/r3_m.sh <tag>
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
out=gpurun_out/$1; mkdir -p "$out"
fatal() { case $1 in 124|134|137|139) return 0;; esac; return 1; }
if [ "${SKIP_TESTS:-0}" != 1 ]; then
  timeout -k 10 600 python -u -m pytest ${TESTS:-tests} -m gpu -x -q --timeout 300 --timeout-method thread > "$out/pytest.log" 2>&1
  rc=$?; tail -4 "$out/pytest.log"; if fatal $rc; then echo "pytest rc=$rc"; exit 1; fi
fi
timeout -k 10 200 python -u tools/build_probe.py > "$out/build.json" 2> "$out/build.err"
rc=$?; cat "$out/build.json"; if fatal $rc; then echo "build rc=$rc"; exit 1; fi
args="--steps 6 --warmup 2 --no-cpu-baseline --no-extras --single-query-reps 0 --rrt-iters 0"
summ() { python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=d['roofline']; print(sys.argv[1].split('/')[-1], round(d['value']/1e6,2), 'M/s step_ms', round(d['ms_per_step'],4), 'walk_ms', round(r['kernel_ms'],4), r['kernel'], 'pairs', r['algorithmic'][:10], d['fast_path'], d['phase_ms'])" "$1"; }
for w in ${WLS:-cfg3 cfg3 cfg5 cfg5k cfg2}; do
  a="--workload ${w%k}"; [ "$w" = cfg5k ] && a="$a --bitstar-knn"
  f="$out/$w.$RANDOM.json"
  timeout -k 10 300 python -u bench.py $a $args > "$f" 2> "$f.err"
  rc=$?; if fatal $rc; then echo "$w rc=$rc"; tail -3 "$f.err"; exit 1; fi
  summ "$f"
done
