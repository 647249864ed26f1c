#!/bin/bash
# round 5: D16M / 8 slab ranks one at a time (tools/slab_serial.py), pass B in one launch and split
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r05serial
mkdir -p $OUT
MPH_SLAB_OVERLAP=0 timeout -k 10 600 python tools/slab_serial.py --case d16m --ranks 8 --steps 4 --warmup 2 > $OUT/serial_d16m_8_overlap0.json 2> $OUT/serial0.err || exit 11
MPH_SLAB_OVERLAP=1 timeout -k 10 600 python tools/slab_serial.py --case d16m --ranks 8 --steps 4 --warmup 2 > $OUT/serial_d16m_8_overlap1.json 2> $OUT/serial1.err || exit 12
