#!/bin/bash
# round 6: the slab suite after the probe change
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/r06f
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest -x -v --timeout 600 --timeout-method thread \
    tests/test_gpu_dist.py tests/test_gpu_d16m.py > $OUT/pytest.log 2>&1 || exit 11
