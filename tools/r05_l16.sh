#!/bin/bash
# round 5: compact 16-bit lists (MPH_LIST16=1, run-time) against 32-bit ELL rows now that the
# developed flow's list traffic is measured: same-box A/B and developed WRITE_SIZE
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r05l16
mkdir -p $OUT
timeout -k 10 600 env MPH_LIST16=1 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_parity.py -k "(golden or trimmed) and not neighbor_sets" > $OUT/pytest_l16.log 2>&1 || exit 10
OUT=$OUT VARIANTS="MPH_LIST16=1" ROUNDS=2 D16M=1 bash tools/ab_dev.sh || exit 11
timeout -k 10 120 python3 tools/dev_state.py d1m 2500 $OUT/d1m_dev.gridb > $OUT/dev_state.log 2>&1 || exit 12
rm -rf gpurun_out/pmc
MPH_LIST16=1 BENCH_EXTRA="--state $OUT/d1m_dev.gridb" bash tools/pmc.sh WRITE_SIZE || exit 13
mv gpurun_out/pmc $OUT/pmc_dev_l16
rm -f $OUT/d1m_dev.gridb
