#!/bin/bash
# round 6: group-rows A/B at rest and t = 1.0 s only (quick)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/${RUN:-r06m}
mkdir -p $OUT
OUT=$OUT/ab100 VARIANTS="MPH_GROUP_ROWS=0" ROUNDS=2 DEV_STEPS=10000 timeout -k 10 600 bash tools/ab_dev.sh || exit 13
python tools/ab_dev_summary.py $OUT/ab100 > $OUT/summary100.txt
