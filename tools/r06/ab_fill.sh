#!/bin/bash
# Gap rows written as zeros at each jump (fill: every list line leaves L2 whole) against the build,
# at rest / t = 0.25 s (2 rounds) and t = 1.0 s (1 round); then D16M in 8 slabs one rank at a time
# (tools/slab_serial.py, graph-timed) on the build.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/${OUT:-ab_fill}
mkdir -p $O
OUT=$O/t025 VARIANTS="fill" ROUNDS=2 bash tools/ab_dev.sh || exit 17
python3 tools/ab_dev_summary.py $O/t025 > $O/summary_t025.txt 2>&1
OUT=$O/t100 DEV_STEPS=10000 VARIANTS="fill" ROUNDS=1 bash tools/ab_dev.sh || exit 18
python3 tools/ab_dev_summary.py $O/t100 > $O/summary_t100.txt 2>&1
timeout -k 10 600 python3 tools/slab_serial.py --case d16m --ranks 8 --steps 4 --warmup 2 > $O/serial_d16m_8.json 2> $O/serial.err || exit 19
