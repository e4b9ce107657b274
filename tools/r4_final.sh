#!/bin/bash
# Round-4 closing GPU run: every -m gpu test, smoke, the default bench line (all five configs with
# their CPU baselines), then the tree-sharded lines at N = 1 (cfg3, cfg5 radius: the merge kernels on a single shard).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
out=gpurun_out/r4_final; mkdir -p "$out"
timeout -k 10 600 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 300 --timeout-method thread \
    > "$out/pytest.log" 2>&1 || { tail -30 "$out/pytest.log"; exit 1; }
tail -2 "$out/pytest.log"
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$out/smoke.log" 2>&1 || { tail -20 "$out/smoke.log"; exit 1; }
tail -1 "$out/smoke.log"
timeout -k 10 590 python -u bench.py --steps 20 --warmup 5 > "$out/bench.json" 2> "$out/bench.err" || { tail -20 "$out/bench.err"; exit 1; }
cut -c1-300 "$out/bench.json"
for w in cfg3 cfg5; do
  timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 \
    --master-port 29517 bench.py --gpus 1 --workload $w --partition tree --steps 10 --warmup 2 --no-cpu-baseline \
    --no-extras --single-query-reps 0 --rrt-iters 0 --workloads none > "$out/tree_$w.json" 2> "$out/tree_$w.err" \
    || { tail -20 "$out/tree_$w.err"; exit 1; }
  cut -c1-300 "$out/tree_$w.json"
done
echo done
