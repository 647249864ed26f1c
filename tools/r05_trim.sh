#!/bin/bash
# round 5: lists kept to the passes' largest radius (default) against the reference's whole lists
# (MPH_LIST_FULL=1): the affected GPU tests, then A/B at rest / developed / D16M
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r05trim
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_developed.py tests/test_gpu_fullsize.py -k "neighbor_sets or trimmed or developed or golden or every_step or full_size" > $OUT/pytest.log 2>&1 || exit 11
OUT=$OUT VARIANTS="MPH_LIST_FULL=1" D16M=1 bash tools/ab_dev.sh || exit 12
