#!/bin/bash
# round 6: group rows -- bitwise against plain rows, the parity / edge / neighbour-set tests, then
# same-box A/B (MPH_GROUP_ROWS=0 is the plain layout) at rest, t = 0.25 s and t = 1.0 s
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/${RUN:-r06g}
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest -x -q -s --timeout 600 --timeout-method thread \
    tests/test_gpu_parity.py tests/test_gpu_edge.py > $OUT/pytest.log 2>&1 || exit 11
OUT=$OUT/ab025 VARIANTS="MPH_GROUP_ROWS=0" ROUNDS=2 timeout -k 10 600 bash tools/ab_dev.sh || exit 12
OUT=$OUT/ab100 VARIANTS="MPH_GROUP_ROWS=0" ROUNDS=2 DEV_STEPS=10000 timeout -k 10 600 bash tools/ab_dev.sh || exit 13
python tools/ab_dev_summary.py $OUT/ab025 > $OUT/summary025.txt
python tools/ab_dev_summary.py $OUT/ab100 > $OUT/summary100.txt
