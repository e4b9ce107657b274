#!/bin/bash
# Round-5 GPU step M: NN parity after a walk change (kNN / radius, full size vs GNAT, appends),
# then the cfg3 / cfg5 / cfg5k lines (no CPU baseline) and their kernel traces.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
out=gpurun_out/${1:-r5_m}; mkdir -p "$out"
timeout -k 10 700 python -u -m pytest tests/test_gpu_nn.py tests/test_gpu_cull.py tests/test_gpu_batch.py tests/test_gpu_index.py \
    tests/test_gpu_fullsize.py::test_cfg3_every_query_vs_gnat tests/test_gpu_fullsize.py::test_cfg2_every_query_vs_gnat \
    tests/test_gpu_fullsize.py::test_cfg5_radius_every_vertex_vs_gnat tests/test_gpu_fullsize.py::test_cfg5_knn_every_vertex_vs_gnat \
    tests/test_gpu_fullsize.py::test_random_access_pattern \
    -m gpu -x -q --timeout 400 --timeout-method thread > "$out/pytest.log" 2>&1
rc=$?
tail -3 "$out/pytest.log"
[ $rc -eq 0 ] || { grep -n "FAIL\|Error\|error" "$out/pytest.log" | head -30; exit 1; }
for w in cfg3 cfg5 cfg5k; do
  extra=""; wl=$w
  [ $w = cfg5k ] && { extra="--bitstar-knn"; wl=cfg5; }
  timeout -k 10 300 python -u bench.py --workload $wl $extra --steps 20 --warmup 5 --workloads none --no-extras --single-query-reps 0 \
      --rrt-iters 0 --no-cpu-baseline > "$out/$w.json" 2> "$out/$w.err" || { tail -30 "$out/$w.err"; exit 1; }
  python - "$out/$w.json" "$w" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(sys.argv[2], d["value"], d["ms_per_step"], json.dumps(d["phase_ms"]), d["roofline"]["kernel_ms"], d["roofline"]["frac"])
PY
done
