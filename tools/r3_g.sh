#!/bin/bash
# round-3 GPU step: the k-d build / kNN / stream parity tests, the build probe at 10^6 / 10^7,
# then the cfg2 / cfg4 / cfg5 bench lines with their CPU baselines.  usage: bash tools/r3_g.sh <tag>
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
out=gpurun_out/$1; mkdir -p "$out"
fatal() { case $1 in 124|134|137|139) return 0;; esac; return 1; }
timeout -k 10 500 python -u -m pytest ${TESTS:-tests/test_gpu_index.py tests/test_gpu_nn.py tests/test_gpu_fullsize.py tests/test_gpu_stream32.py tests/test_gpu_cull.py} \
    -m gpu -x -q --timeout 300 --timeout-method thread > "$out/pytest.log" 2>&1
rc=$?; tail -2 "$out/pytest.log"; if [ $rc != 0 ]; then echo "pytest rc=$rc"; grep -E "FAIL|Error" "$out/pytest.log" | head; exit 1; fi
timeout -k 10 200 python -u tools/build_probe.py > "$out/build.json" 2> "$out/build.err"
rc=$?; cat "$out/build.json"; if [ $rc != 0 ]; then echo "build rc=$rc"; exit 1; fi
for w in ${WLS:-cfg4 cfg5 cfg2}; do
  f="$out/$w.json"
  timeout -k 10 400 python -u bench.py --workload $w --steps 5 --warmup 2 --single-query-reps 0 --rrt-iters 0 > "$f" 2> "$f.err"
  rc=$?; if fatal $rc; then echo "$w rc=$rc"; tail -3 "$f.err"; exit 1; fi
  python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[1].split('/')[-1], round(d['value']/1e6,3), 'M/s', round(d['ms_per_step'],3), 'ms', d['roofline']['kernel'], round(d['roofline']['kernel_ms'],3), json.dumps(d.get('cpu_baseline'))[:300])" "$f"
done
