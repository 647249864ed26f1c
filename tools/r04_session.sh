#!/bin/bash
# Round 4 GPU session: every GPU test (K, default all; K=none skips), the same-box A/B of VARIANTS
# on CASES (tools/ab.sh), the D16M / 8 slabs one rank at a time with the replayed exchange
# (tools/slab_serial.py --replay) with and without MPH_SLAB_OVERLAP, and the PMC issue groups of
# the base build (tools/pmc_ab.sh).  Time-limited steps; stops at a test-runner crash.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${OUT:-r04s}
mkdir -p $OUT
if [ "${K-}" != none ]; then
  timeout -k 10 ${PYT_TIMEOUT:-900} python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread ${K:+-k "$K"} \
      > $OUT/pytest_gpu.log 2>&1
  rc=$?
  echo "pytest rc=$rc" >> $OUT/pytest_gpu.log
  case $rc in 0|1|5) ;; *) exit 12;; esac
fi
if [ -n "$PADEBUG" ]; then
  MPH_GPU_LIB=$PWD/particlemethod_fsi_amd/lib_pasd/libmph_gpu.so timeout -k 10 200 python tools/pa_debug.py box3d gate3d d1m \
      > $OUT/pa_debug.log 2>&1 || exit 18
fi
for v in $BITWISE; do   # bit-identical variant builds (lib_<v>) against the base build
  timeout -k 10 300 python tools/lib_bitwise.py run $OUT/bitwise_base.npz > $OUT/bitwise_base.log 2>&1 || exit 16
  MPH_GPU_LIB=$PWD/particlemethod_fsi_amd/lib_$v/libmph_gpu.so timeout -k 10 300 python tools/lib_bitwise.py run \
      $OUT/bitwise_$v.npz > $OUT/bitwise_$v.log 2>&1 || exit 17
  python tools/lib_bitwise.py compare $OUT/bitwise_base.npz $OUT/bitwise_$v.npz >> $OUT/bitwise_$v.log 2>&1
  rm -f $OUT/bitwise_*.npz
done
if [ -n "${VARIANTS+x}" ]; then
  CASES="${CASES:-d1m}" VARIANTS="$VARIANTS" STEPS=${STEPS:-40} bash tools/ab.sh || exit 13
  mkdir -p $OUT/ab && mv gpurun_out/ab_*.log $OUT/ab/
fi
if [ -n "$SERIAL" ]; then
  for ov in 1 0; do
    MPH_SLAB_OVERLAP=$ov timeout -k 10 400 python tools/slab_serial.py --case d16m --ranks 8 --steps 6 --warmup 2 \
        --replay > $OUT/serial_d16m_8_overlap$ov.json 2>> $OUT/serial.err || exit 14
  done
fi
if [ -n "$PMC" ]; then
  VARIANTS="${PMC_VARIANTS:-base}" bash tools/pmc_ab.sh || exit 15
  for v in ${PMC_VARIANTS:-base}; do cp gpurun_out/pmc_$v.txt $OUT/; done
fi
