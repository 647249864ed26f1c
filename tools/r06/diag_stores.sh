#!/bin/bash
# Diagnostic builds of the search (csrc_ab, not product): no list stores (nostore) and the same
# store instructions aimed at the lane's first row (onerow), against the build, at rest, t = 0.25 s
# and t = 1.0 s; only the search's time means anything in the diagnostic builds.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/${OUT:-diag_stores}
mkdir -p $O
OUT=$O/t025 VARIANTS="nostore onerow" ROUNDS=1 bash tools/ab_dev.sh || exit 17
python3 tools/ab_dev_summary.py $O/t025 > $O/summary_t025.txt 2>&1
OUT=$O/t100 DEV_STEPS=10000 VARIANTS="nostore onerow" ROUNDS=1 bash tools/ab_dev.sh || exit 18
python3 tools/ab_dev_summary.py $O/t100 > $O/summary_t100.txt 2>&1
