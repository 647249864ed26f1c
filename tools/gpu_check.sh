#!/bin/bash
# One GPU-box session: smoke, GPU parity tests, a short bench.  Every GPU step is time-limited and
# the chain stops at the first failure (see the gpurun rules in the task description).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
STEPS=${STEPS:-20}
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || exit 11
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread ${PYTEST_ARGS} > gpurun_out/pytest_gpu.log 2>&1
rc=$?
echo "pytest rc=$rc" >> gpurun_out/pytest_gpu.log
case $rc in 0|1) ;; *) exit 12;; esac
timeout -k 10 900 python bench.py --steps $STEPS --warmup 4 ${BENCH_ARGS} > gpurun_out/bench.log 2>&1 || exit 13
