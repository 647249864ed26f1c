#!/bin/bash
# round 6: pass occupancy variants (5 waves per SIMD) -- same-box A/B at rest, t = 0.25 s, t = 1.0 s
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/${RUN:-r06n}
mkdir -p $OUT
OUT=$OUT/ab025 VARIANTS="ua3w5 ub6w5" ROUNDS=2 timeout -k 10 600 bash tools/ab_dev.sh || exit 12
OUT=$OUT/ab100 VARIANTS="ua3w5 ub6w5" ROUNDS=2 DEV_STEPS=10000 timeout -k 10 600 bash tools/ab_dev.sh || exit 13
python tools/ab_dev_summary.py $OUT/ab025 > $OUT/summary025.txt
python tools/ab_dev_summary.py $OUT/ab100 > $OUT/summary100.txt
