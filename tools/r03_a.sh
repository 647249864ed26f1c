#!/bin/bash
# Round 3, first box session: every GPU test, then same-box A/B of the fused search + pass A
# against the separate kernels and its tuning variants (tools/ab.sh), then the rocprofv3 kernel
# trace of the default build.  Time-limited steps; stops at the first failure.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r03a
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r03a/smoke.log 2>&1 || exit 11
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread ${PYTEST_ARGS} \
    > gpurun_out/r03a/pytest_gpu.log 2>&1
rc=$?
echo "pytest rc=$rc" >> gpurun_out/r03a/pytest_gpu.log
case $rc in 0|1) ;; *) exit 12;; esac
CASES="${CASES:-d1m}" VARIANTS="${VARIANTS:-MPH_FUSED=0 fcap96 w3fu2 fcap160}" STEPS=40 bash tools/ab.sh || exit 13
mkdir -p gpurun_out/r03a/ab && mv gpurun_out/ab_*.log gpurun_out/r03a/ab/
STEPS=24 bash tools/profile.sh || exit 14
