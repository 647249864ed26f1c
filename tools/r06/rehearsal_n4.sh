#!/bin/bash
# The multi-rank bench with four ranks on one GPU (distinct left and right neighbours, unlike two
# ranks): over the host transport, then asking for RCCL, which refuses ranks that share a device --
# every rank must fall back to the host transport and say so in the line.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/${OUT:-rehearsal_n4}
mkdir -p $O
MPH_SLAB_TRANSPORT=host MPH_BENCH_DEVICE=0 timeout -k 10 500 python -m torch.distributed.run \
  --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29504 \
  bench.py --gpus 4 --steps 5 --warmup 2 > $O/host_n4.log 2>&1 || exit 20
MPH_BENCH_DEVICE=0 timeout -k 10 500 python -m torch.distributed.run \
  --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29505 \
  bench.py --gpus 4 --steps 5 --warmup 2 > $O/rccl_fallback_n4.log 2>&1 || exit 21
