#!/bin/bash
# Round 3 session g: slab / dist tests after the merged pack/unpack/halo launches, the D16M slabs
# one rank at a time (tools/slab_serial.py, overlap on and off), then optional PMC groups of
# VARIANTS (tools/pmc_ab.sh).  Time-limited steps; stops at a test-runner crash.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${OUT:-r03g}
mkdir -p $OUT
if [ "${K:-none}" != none ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -q -k "$K" --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
  rc=$?
  echo "pytest rc=$rc" >> $OUT/pytest_gpu.log
  case $rc in 0|1|5) ;; *) exit 12;; esac
fi
if [ -z "$NO_SERIAL" ]; then
  timeout -k 10 400 python tools/slab_serial.py --case d16m --ranks 8 --steps 6 --warmup 2 > $OUT/serial_d16m_8.json 2>> $OUT/serial.err || exit 13
  MPH_SLAB_OVERLAP=0 timeout -k 10 400 python tools/slab_serial.py --case d16m --ranks 8 --steps 6 --warmup 2 > $OUT/serial_d16m_8_nooverlap.json 2>> $OUT/serial.err || exit 14
fi
for v in $SERIAL_VARIANTS; do   # alternative builds (lib_<name>), one rank at a time without the overlap
  MPH_GPU_LIB=$PWD/particlemethod_fsi_amd/lib_$v/libmph_gpu.so MPH_SLAB_OVERLAP=0 timeout -k 10 400 python tools/slab_serial.py \
      --case d16m --ranks 8 --steps 6 --warmup 2 > $OUT/serial_d16m_8_nooverlap_$v.json 2>> $OUT/serial.err || exit 17
done
if [ -n "$PMC_VARIANTS" ]; then
  VARIANTS="$PMC_VARIANTS" bash tools/pmc_ab.sh || exit 15
  for v in $PMC_VARIANTS; do cp gpurun_out/pmc_$v.txt $OUT/; done
fi
if [ -n "$AB_VARIANTS" ]; then
  CASES="${AB_CASES:-d1m}" VARIANTS="$AB_VARIANTS" STEPS=${STEPS:-40} bash tools/ab.sh || exit 16
  mkdir -p $OUT/ab && mv gpurun_out/ab_*.log $OUT/ab/
fi
