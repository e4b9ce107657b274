#!/bin/bash
# cfg4 A/B of the culled chain scan's chunk count (OMPL_GPU_CHAIN_WPC waves per CU)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
out=gpurun_out/$1; mkdir -p "$out"
a="--workload cfg4 --steps 4 --warmup 1 --no-cpu-baseline --no-extras"
for r in 1 2; do for v in ${WPCS:-24 48 12 96}; do
  f="$out/wpc$v.$r.json"
  OMPL_GPU_CHAIN_WPC=$v timeout -k 10 300 python -u bench.py $a > "$f" 2> "$f.err" || { echo "rc=$?"; tail -3 "$f.err"; exit 1; }
  python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=d['roofline']; print(sys.argv[1].split('/')[-1], round(d['ms_per_step'],3), 'kern', round(r['kernel_ms'],3))" "$f"
done; done
