#!/bin/bash
# Aligned rows: the jump threshold (d2, d4: jump only when the lanes' rows differ by >= 2 / 4)
# against the build (>= 1), at rest and t = 0.25 s (2 rounds), t = 1.0 s (1 round); then the PMC
# issue groups of the build in the developed state (t = 0.25 s).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/${OUT:-ab_drift}
mkdir -p $O
OUT=$O/t025 VARIANTS="d2 d4" ROUNDS=2 bash tools/ab_dev.sh || exit 17
python3 tools/ab_dev_summary.py $O/t025 > $O/summary_t025.txt 2>&1
OUT=$O/t100 DEV_STEPS=10000 VARIANTS="d2 d4" ROUNDS=1 bash tools/ab_dev.sh || exit 18
python3 tools/ab_dev_summary.py $O/t100 > $O/summary_t100.txt 2>&1
timeout -k 10 120 python3 tools/dev_state.py d1m 2500 /tmp/d1m_dev.gridb > $O/pmc_state.log 2>&1 || exit 19
rm -rf gpurun_out/pmc_base gpurun_out/pmc
BENCH_EXTRA="--state /tmp/d1m_dev.gridb" VARIANTS=base bash tools/pmc_ab.sh || exit 20
cp gpurun_out/pmc_base.txt $O/pmc_dev_t025.txt
rm -rf gpurun_out/pmc gpurun_out/pmc_base /tmp/d1m_dev.gridb
