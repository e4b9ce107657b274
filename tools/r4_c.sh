#!/bin/bash
# round-4: every -m gpu test (no -x: the whole list of failures), then kernel traces of cfg4 / cfg5
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
out=gpurun_out/r4c; mkdir -p "$out"
timeout -k 10 900 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 300 --timeout-method thread \
    > "$out/pytest.log" 2>&1; rc=$?
tail -25 "$out/pytest.log" | grep -E "FAILED|ERROR|passed|failed"
case $rc in 124|134|137|139) echo "pytest rc=$rc"; exit 1;; esac
for w in ${WLS:-cfg4 cfg5 cfg5k}; do
  mkdir -p "$out/tr_$w"
  a="--workload ${w%k}"; [ "$w" = cfg5k ] && a="$a --bitstar-knn"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$out/tr_$w" -o trace --output-format csv -- python bench.py \
    $a --steps 3 --warmup 1 --no-cpu-baseline --workloads none > "$out/tr_$w/trace.log" 2>&1 || { echo "trace $w rc=$?"; exit 1; }
  grep '^{' "$out/tr_$w/trace.log" | cut -c1-200
done
