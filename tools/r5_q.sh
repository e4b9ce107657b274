#!/bin/bash
# Round-5 GPU step Q: PRM* / RRT* parity after the stored-count kernels, then the RRT* line.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
out=gpurun_out/r5_q; mkdir -p "$out"
timeout -k 10 600 python -u -m pytest tests/test_gpu_prm.py tests/test_gpu_rrtstar.py tests/test_gpu_fullsize.py::test_cfg4_prm_batch_1_vs_sequential_loop \
    -m gpu -x -q --timeout 300 --timeout-method thread > "$out/pytest.log" 2>&1 || { tail -20 "$out/pytest.log"; exit 1; }
tail -1 "$out/pytest.log"
timeout -k 10 500 python -u bench.py --steps 5 --warmup 2 --workloads rrt_star --no-extras --single-query-reps 0 \
    --rrt-iters 0 --no-cpu-baseline > "$out/rrtstar.json" 2> "$out/rrtstar.err" || { tail -30 "$out/rrtstar.err"; exit 1; }
python - "$out/rrtstar.json" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
w = d["workloads"]["rrt_star"]
print("rrt_star", w["value"], w["ms_per_step"], json.dumps(w["phase_ms"]))
PY
