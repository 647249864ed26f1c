#!/bin/bash
# round 5: the passes XCD split in block 0 of the next step k_rank_scatter (default) or k_prep (lib_splitp)
# launch after the search (lib_splitk, MPH_SPLIT_IN_PREP=0), same box; then the bitwise XCD-map test
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r05splitprep
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_parity.py -k "xcd or box3d or dam2d" > $OUT/pytest.log 2>&1 || exit 10
OUT=$OUT VARIANTS="splitk splitp" ROUNDS=3 D16M=1 bash tools/ab_dev.sh || exit 11
