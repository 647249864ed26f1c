#!/bin/bash
# Round 6 final evidence on the last build (tools/r06/final2.sh's chain), plus D16M in 8 slabs one
# rank at a time with pass B in one launch (MPH_SLAB_OVERLAP=0) and with the overlap (=1).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=${OUT:-r06final3} bash tools/r06/final2.sh || exit $?
O=gpurun_out/${OUT:-r06final3}
for ov in 0 1; do
  MPH_SLAB_OVERLAP=$ov timeout -k 10 600 python3 tools/slab_serial.py --case d16m --ranks 8 --steps 4 --warmup 2 > $O/serial_d16m_8_overlap$ov.json 2> $O/serial_overlap$ov.err || exit 31
done
