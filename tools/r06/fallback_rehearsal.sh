#!/bin/bash
# The multi-rank bench on one GPU: two ranks over the host transport (the rehearsal), then two ranks
# asking for RCCL, which refuses two ranks on one device -- every rank must fall back to the host
# transport and say so in the line (`slab.transport_fallback`).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/${OUT:-fallback}
mkdir -p $O
MPH_SLAB_TRANSPORT=host MPH_BENCH_DEVICE=0 timeout -k 10 600 python -m torch.distributed.run \
  --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29502 \
  bench.py --gpus 2 --steps 5 --warmup 2 > $O/host_n2.log 2>&1 || exit 20
MPH_BENCH_DEVICE=0 timeout -k 10 600 python -m torch.distributed.run \
  --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29503 \
  bench.py --gpus 2 --steps 5 --warmup 2 > $O/rccl_fallback_n2.log 2>&1 || exit 21
