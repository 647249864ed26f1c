#!/bin/bash
# round 5: WRITE_SIZE / FETCH_SIZE of the search in the developed flow (list write amplification
# off the lattice)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r05devwrite
mkdir -p $OUT
timeout -k 10 120 python3 tools/dev_state.py d1m 2500 $OUT/d1m_dev.gridb > $OUT/dev_state.log 2>&1 || exit 11
rm -rf gpurun_out/pmc
BENCH_EXTRA="--state $OUT/d1m_dev.gridb" bash tools/pmc.sh WRITE_SIZE FETCH_SIZE || exit 12
mv gpurun_out/pmc $OUT/pmc
rm -f $OUT/d1m_dev.gridb
