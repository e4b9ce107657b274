#!/bin/bash
# Round-5 GPU step MV: motion parity tests, then the motion-heavy workload lines (cfg5k, cfg5, cfg3)
# without CPU baselines.  usage: bash tools/r5_mv.sh <out> [tests...]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
out=gpurun_out/${1:-r5_mv}; shift || true
mkdir -p "$out"
tests=${*:-tests/test_gpu_motion.py tests/test_gpu_spaces.py tests/test_gpu_batch.py tests/test_gpu_prm.py tests/test_gpu_fullsize.py}
timeout -k 10 600 python -u -m pytest $tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > "$out/pytest.log" 2>&1
rc=$?
tail -2 "$out/pytest.log"
[ $rc -eq 0 ] || { grep -n "FAIL\|Error\|error" "$out/pytest.log" | head -30; exit 1; }
for w in ${WLS:-cfg5k cfg5 cfg4 cfg3}; do
  extra=""; wl=$w
  [ $w = cfg5k ] && { extra="--bitstar-knn"; wl=cfg5; }
  timeout -k 10 300 python -u bench.py --workload $wl $extra --steps 20 --warmup 5 --workloads none --no-extras --single-query-reps 0 \
      --rrt-iters 0 --no-cpu-baseline > "$out/$w.json" 2> "$out/$w.err" || { tail -30 "$out/$w.err"; exit 1; }
  python - "$out/$w.json" "$w" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(sys.argv[2], d["value"], d["ms_per_step"], json.dumps(d["phase_ms"]), d["roofline"]["kernel_ms"], d.get("motion_valid_fraction"))
PY
done
