#!/bin/bash
# Rehearsal of the multi-GPU bench path on a one-GPU box: N ranks share cuda:0 and move their
# halos through the host-staged transport (RCCL refuses two ranks on one device).  Every GPU step
# is time-limited and the chain stops at the first failure.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for N in ${RANKS:-2 4}; do
  MPH_SLAB_TRANSPORT=host MPH_BENCH_DEVICE=0 timeout -k 10 600 python -m torch.distributed.run \
    --nnodes=1 --nproc-per-node $N --master-addr 127.0.0.1 --master-port $((29500 + N)) \
    bench.py --gpus $N --steps ${STEPS:-10} --warmup 2 --case ${CASE:-d1m} > gpurun_out/rehearsal_${CASE:-d1m}_n$N.log 2>&1 || exit 20
done
