#!/bin/bash
# GPU box: bench line (with CPU baseline) + kernel trace + FETCH/WRITE passes for cfg2 / cfg4 / cfg5,
# then one SQ-counter pass of the headline workload.  -> gpurun_out/r2_<w>/, gpurun_out/prof_r2_<w>/
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
for w in ${WORKLOADS:-cfg2 cfg4 cfg5}; do
  mkdir -p gpurun_out/r2_$w
  timeout -k 10 400 python -u bench.py --workload $w > gpurun_out/r2_$w/bench.json 2> gpurun_out/r2_$w/bench.err \
      || { tail -20 gpurun_out/r2_$w/bench.err; exit 1; }
  cut -c1-300 gpurun_out/r2_$w/bench.json
  bash tools/prof_workload.sh $w r2_$w || exit $?
done
bash tools/sq_counters.sh gpurun_out/prof_r2_cfg3_sq --no-extras > gpurun_out/sq_cfg3.log 2>&1 || exit $?

# the driver's multi-GPU launch form, at N=1 on this box (RCCL init + barrier + max-over-ranks)
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 \
    --master-port 29511 bench.py --gpus 1 --steps 3 --warmup 1 --no-cpu-baseline --no-extras \
    > gpurun_out/torchrun_n1.json 2> gpurun_out/torchrun_n1.err || { tail -20 gpurun_out/torchrun_n1.err; exit 1; }
cut -c1-400 gpurun_out/torchrun_n1.json
echo done
