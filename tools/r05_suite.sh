#!/bin/bash
# Round 5: the whole GPU test suite on the final build (one process, per-test time limits)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${OUT:-r05suite}
mkdir -p $OUT
timeout -k 10 1050 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
rc=$?
echo "pytest rc=$rc" >> $OUT/pytest_gpu.log
exit $rc
