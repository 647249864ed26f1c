#!/bin/bash
# round 6, first GPU call: the long-horizon elastic / FSI parity tests and the FSI probe
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/r06a
mkdir -p $OUT
timeout -k 10 300 python -u tools/fsi_sub_probe.py fsi3d_sub 250 3000 > $OUT/probe_fsi3d_sub.log 2>&1 || exit 11
timeout -k 10 600 python -u -m pytest -x -v -s --timeout 500 --timeout-method thread \
    tests/test_gpu_longrun.py > $OUT/pytest.log 2>&1 || exit 12
