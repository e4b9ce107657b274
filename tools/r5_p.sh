#!/bin/bash
# Round-5 GPU step P: radius tests after the scan fix, then cfg5 (radius) and cfg3 lines.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
out=gpurun_out/r5_p; mkdir -p "$out"
timeout -k 10 500 python -u -m pytest tests/test_gpu_batch.py tests/test_gpu_fullsize.py::test_cfg5_radius_every_vertex_vs_gnat -m gpu -x -q \
    --timeout 300 --timeout-method thread > "$out/pytest.log" 2>&1 || { tail -20 "$out/pytest.log"; exit 1; }
tail -1 "$out/pytest.log"
timeout -k 10 300 python -u bench.py --workload cfg5 --steps 10 --warmup 3 --workloads none --no-extras --no-cpu-baseline > "$out/cfg5.json" 2> "$out/cfg5.err" || { tail -20 "$out/cfg5.err"; exit 1; }
python -c "import json; d=json.loads(open('$out/cfg5.json').read().strip().splitlines()[-1]); print('cfg5', d['value'], d['ms_per_step'], d['phase_ms'], d['radius_walks'])"
