#!/bin/bash
# GPU box: targeted tests, then the default bench line (with extras), each under its own limit.
# usage: bash tools/r2_step.sh <tag> [pytest -k expression]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
out=gpurun_out/${1:-r2}; mkdir -p "$out"
sel=${2:-}
if [ -n "$sel" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread \
      -k "$sel" > "$out/pytest.log" 2>&1 || { tail -40 "$out/pytest.log"; exit 1; }
  tail -3 "$out/pytest.log"
fi
timeout -k 10 400 python -u bench.py --no-cpu-baseline > "$out/bench.json" 2> "$out/bench.err" || { tail -20 "$out/bench.err"; exit 1; }
python - "$out/bench.json" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
for k in ("value", "ms_per_step"):
    print(k, d[k])
print("roofline", {k: d["roofline"][k] for k in ("kernel_ms", "frac")})
for k in ("single_query", "single_query_1e7", "rrt_device", "rrt_star_knn"):
    v = d.get(k)
    if v:
        print(k, {a: b for a, b in v.items() if not isinstance(b, dict)}, v.get("roofline", {}).get("frac"))
PY
