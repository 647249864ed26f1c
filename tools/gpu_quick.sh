#!/bin/bash
# Quick GPU iteration: GPU parity tests (optionally filtered with K=...) then bench lines for the
# cases in CASES (default d1m).  Time-limited steps; stops at the first failure.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/quick
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread ${K:+-k "$K"} \
    > gpurun_out/quick/pytest.log 2>&1 || exit 11
for c in ${CASES:-d1m}; do
  timeout -k 10 300 python bench.py --case $c --steps 20 --warmup 4 --no-cpu-baseline \
      > gpurun_out/quick/bench_$c.json 2> gpurun_out/quick/bench_$c.err || exit 12
done
