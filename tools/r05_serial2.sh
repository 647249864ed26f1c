#!/bin/bash
# round 5: D16M / 8 slab ranks one at a time, the list kernels also timed as graph replays
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${OUT:-r05serial3}
mkdir -p $OUT
MPH_SLAB_OVERLAP=0 timeout -k 10 600 python tools/slab_serial.py --case d16m --ranks 8 --steps 4 --warmup 2 > $OUT/serial_d16m_8_overlap0.json 2> $OUT/serial0.err || exit 11
