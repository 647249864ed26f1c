#!/bin/bash
# Round 3 session f: the elastic overlap (u / P ghost exchanges beside the inner slots, early send
# on elastic ranks): the slab / structure / driver GPU tests, then FSI and Bar in 8 slabs one rank
# at a time (tools/slab_serial.py) with the overlap on and off.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${OUT:-r03f}
K=${K:-"slab or structure or early or driver or dist"}
mkdir -p $OUT
[ -n "$SKIP_TESTS" ] || timeout -k 10 900 python -u -m pytest tests -m gpu -q -k "$K" --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
rc=$?
echo "pytest rc=$rc" >> $OUT/pytest_gpu.log
case $rc in 0|1) ;; *) exit 12;; esac
# fsi3d is 0.12 deep along z: 4 slabs (8 would be thinner than two halo widths)
for cr in ${CASES:-fsi3d:4 bar2d_400k:8 d16m:8}; do
  c=${cr%:*}; r=${cr#*:}
  timeout -k 10 400 python tools/slab_serial.py --case $c --ranks $r --steps 6 --warmup 2 ${REPLAY:+--replay} > $OUT/serial_${c}_$r.json 2>> $OUT/serial.err || exit 13
  MPH_SLAB_OVERLAP=0 timeout -k 10 400 python tools/slab_serial.py --case $c --ranks $r --steps 6 --warmup 2 ${REPLAY:+--replay} > $OUT/serial_${c}_${r}_nooverlap.json 2>> $OUT/serial.err || exit 14
done
# A/B switches on the D16M slabs (VARS: space-separated VAR=VALUE, one run each)
for v in ${VARS}; do
  env $v timeout -k 10 400 python tools/slab_serial.py --case d16m --ranks 8 --steps 6 --warmup 2 ${REPLAY:+--replay} > $OUT/serial_d16m_8_${v}.json 2>> $OUT/serial.err || exit 15
done
