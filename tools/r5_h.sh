#!/bin/bash
# Round-5 GPU step H: SE3 kNN parity after a walk change, then the headline (cfg3) alone, twice.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
out=gpurun_out/r5_h; mkdir -p "$out"
timeout -k 10 600 python -u -m pytest tests/test_gpu_nn.py tests/test_gpu_cull.py tests/test_gpu_fullsize.py::test_cfg3_every_query_vs_gnat \
    tests/test_gpu_fullsize.py::test_cfg2_every_query_vs_gnat tests/test_gpu_fullsize.py::test_cfg5_knn_every_vertex_vs_gnat \
    -m gpu -x -q --timeout 300 --timeout-method thread > "$out/pytest.log" 2>&1
rc=$?
tail -3 "$out/pytest.log"
[ $rc -eq 0 ] || { grep -n "FAIL\|Error\|error" "$out/pytest.log" | head -30; exit 1; }
for r in 1 2; do
  timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --workloads none --no-extras --single-query-reps 0 --rrt-iters 0 \
      --no-cpu-baseline > "$out/bench$r.json" 2> "$out/bench$r.err" || { tail -30 "$out/bench$r.err"; exit 1; }
  python - "$out/bench$r.json" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print("headline", d["value"], d["ms_per_step"], json.dumps(d["phase_ms"]), d["roofline"]["kernel_ms"], d["roofline"]["frac"])
PY
done
