#!/bin/bash
# A 17-row tile pad against the build's 1 row: D1M rest / t = 0.25 s and D16M, 3 rounds.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/${OUT:-ab_pad17}
mkdir -p $O
OUT=$O D16M=1 VARIANTS="pad17" ROUNDS=3 bash tools/ab_dev.sh || exit 17
python3 tools/ab_dev_summary.py $O > $O/summary.txt 2>&1
