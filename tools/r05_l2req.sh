#!/bin/bash
# round 5: the search's L2 request counts at rest and at t = 1.0 s (writes from the CUs, all
# requests, write sectors) -- is the list-store cost the L2 request rate of scattered 4-byte stores?
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r05l2req
mkdir -p $OUT
G1="TCC_REQ_sum TCC_WRITE_sum TCC_WRITE_SECTORS_sum"
G2="TCP_TCC_WRITE_REQ_sum TCP_TCC_READ_REQ_sum"
rm -rf gpurun_out/pmc
bash tools/pmc.sh "$G1" "$G2" || exit 11
mv gpurun_out/pmc $OUT/rest
timeout -k 10 120 python3 tools/dev_state.py d1m 10000 /tmp/d1m_t1.gridb > $OUT/dev_state.log 2>&1 || exit 12
BENCH_EXTRA="--state /tmp/d1m_t1.gridb" bash tools/pmc.sh "$G1" "$G2" || exit 13
mv gpurun_out/pmc $OUT/t1
rm -f /tmp/d1m_t1.gridb
