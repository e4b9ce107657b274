#!/bin/bash
# round-3 GPU step: every -m gpu test, then short bench lines (no CPU baseline) of the listed
# workloads (cfg5k = cfg5 --bitstar-knn).  usage: bash tools/r3_c.sh <tag> ["cfg3 cfg4 ..."]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
out=gpurun_out/$1; mkdir -p "$out"
fatal() { case $1 in 124|134|137|139) return 0;; esac; return 1; }
if [ "${SKIP_TESTS:-0}" != 1 ]; then
  timeout -k 10 600 python -u -m pytest ${TESTS:-tests} -m gpu -x -q --timeout 300 --timeout-method thread > "$out/pytest.log" 2>&1
  rc=$?; tail -4 "$out/pytest.log"; if [ $rc != 0 ]; then echo "pytest rc=$rc"; grep -E "FAIL|Error" "$out/pytest.log" | head; exit 1; fi
fi
args="--steps 5 --warmup 2 --no-cpu-baseline --no-extras --single-query-reps 0 --rrt-iters 0"
summ() { python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=d['roofline']; print(sys.argv[1].split('/')[-1], round(d['value']/1e6,3), 'M/s step_ms', round(d['ms_per_step'],4), 'kern_ms', round(r['kernel_ms'],4), r['kernel'], d.get('fast_path'), d.get('phase_ms'))" "$1"; }
for w in ${2:-cfg3 cfg4 cfg5}; do
  a="--workload ${w%k}"; [ "$w" = cfg5k ] && a="$a --bitstar-knn"
  f="$out/$w.$RANDOM.json"
  timeout -k 10 300 python -u bench.py $a $args > "$f" 2> "$f.err"
  rc=$?; if fatal $rc; then echo "$w rc=$rc"; tail -3 "$f.err"; exit 1; fi
  [ $rc = 0 ] && summ "$f" || { echo "$w rc=$rc"; tail -3 "$f.err"; }
done
