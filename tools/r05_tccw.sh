#!/bin/bash
# round 5: how the search's list writes leave L2, at rest and developed: EA write transactions
# (all / 64-byte), L2 write-backs and evictions, write requests, hits, misses, streaming requests
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r05tccw
mkdir -p $OUT
G1="TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum TCC_NORMAL_WRITEBACK_sum TCC_NORMAL_EVICT_sum"
G2="TCC_WRITE_REQ_sum TCC_HIT_sum TCC_MISS_sum TCC_STREAMING_REQ_sum"
rm -rf gpurun_out/pmc
bash tools/pmc.sh "$G1" "$G2" || exit 11
mv gpurun_out/pmc $OUT/rest
timeout -k 10 120 python3 tools/dev_state.py d1m 2500 $OUT/d1m_dev.gridb > $OUT/dev_state.log 2>&1 || exit 12
BENCH_EXTRA="--state $OUT/d1m_dev.gridb" bash tools/pmc.sh "$G1" "$G2" || exit 13
mv gpurun_out/pmc $OUT/dev
rm -f $OUT/d1m_dev.gridb
