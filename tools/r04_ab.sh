#!/bin/bash
# GPU session: selected GPU tests (K=<pytest -k expression>, empty: all), then same-box A/B of the
# VARIANTS on CASES (tools/ab.sh), logs under gpurun_out/$OUT.  Time-limited steps; stops at a
# test-runner crash (test failures are recorded and the A/B still runs).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${OUT:-r04ab}
mkdir -p $OUT
if [ "${K-none}" != none ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread ${K:+-k "$K"} \
      > $OUT/pytest_gpu.log 2>&1
  rc=$?
  echo "pytest rc=$rc" >> $OUT/pytest_gpu.log
  case $rc in 0|1|5) ;; *) exit 12;; esac
fi
if [ -n "${VARIANTS+x}" ]; then
  CASES="${CASES:-d1m}" VARIANTS="$VARIANTS" STEPS=${STEPS:-40} bash tools/ab.sh || exit 13
  mkdir -p $OUT/ab && mv gpurun_out/ab_*.log $OUT/ab/
fi
