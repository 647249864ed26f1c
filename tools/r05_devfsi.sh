#!/bin/bash
# round 5: the developed-flow parity tests (D1M at t = 0.25 s, FSI at t = 0.2 s)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r05devfsi
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest -x -v -s --timeout 600 --timeout-method thread tests/test_gpu_developed.py > $OUT/pytest.log 2>&1 || exit 11
