#!/bin/bash
# round 5: the developed-flow parity at t = 0.25 s and t = 1.0 s, and the bench's developed
# object at t = 1.0 s (10,000 steps: the reference's whole Dam run)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r05dev10k
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest -x -v -s --timeout 600 --timeout-method thread tests/test_gpu_developed.py > $OUT/pytest.log 2>&1 || exit 11
timeout -k 10 400 python bench.py --developed-steps 10000 --no-cpu-baseline > $OUT/bench_dev10k.json 2> $OUT/bench_dev10k.err || exit 12
