#!/bin/bash
# Aligned rows: the whole GPU suite on the build, then the search's jump placement (pb: at column
# pair boundaries) and tile padding (pad33) against the build and the previous build (r6base).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/${OUT:-ab_rows3}
mkdir -p $O
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || exit 11
OUT=$O/ab VARIANTS="pb pad33 r6base" ROUNDS=2 bash tools/ab_dev.sh || exit 17
python3 tools/ab_dev_summary.py $O/ab > $O/summary.txt 2>&1
