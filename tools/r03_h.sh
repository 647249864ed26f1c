#!/bin/bash
# Round 3 session h: the work-balanced XCD map of the list kernels.  GPU tests (all, or -k "$K"),
# then A/B benches of the base build against lib_nobal (MPH_XCD_BAL=0) on D1M and D16M, the D16M
# slabs one rank at a time for both, and the per-XCD wave timing (lib_xcd, tools/xcd_diag.py).
# Time-limited steps; stops at a test-runner crash.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${OUT:-r03h}
mkdir -p $OUT
if [ "${K:-all}" != none ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -q ${K:+-k "$K"} --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
  rc=$?
  echo "pytest rc=$rc" >> $OUT/pytest_gpu.log
  case $rc in 0|1|5) ;; *) exit 12;; esac
fi
CASES="${AB_CASES:-d1m d16m}" VARIANTS="${AB_VARIANTS:-nobal}" STEPS=${STEPS:-40} bash tools/ab.sh || exit 16
mkdir -p $OUT/ab && mv gpurun_out/ab_*.log $OUT/ab/
MPH_SLAB_OVERLAP=0 timeout -k 10 400 python tools/slab_serial.py --case d16m --ranks 8 --steps 6 --warmup 2 \
    > $OUT/serial_d16m_8_nooverlap.json 2>> $OUT/serial.err || exit 13
MPH_GPU_LIB=$PWD/particlemethod_fsi_amd/lib_nobal/libmph_gpu.so MPH_SLAB_OVERLAP=0 timeout -k 10 400 \
    python tools/slab_serial.py --case d16m --ranks 8 --steps 6 --warmup 2 > $OUT/serial_d16m_8_nooverlap_nobal.json 2>> $OUT/serial.err || exit 14
if [ -f particlemethod_fsi_amd/lib_xcd/libmph_gpu.so ]; then
  MPH_GPU_LIB=$PWD/particlemethod_fsi_amd/lib_xcd/libmph_gpu.so timeout -k 10 120 python tools/xcd_diag.py --case d1m \
      > $OUT/xcd_d1m.json 2>> $OUT/xcd.err || exit 15
  MPH_GPU_LIB=$PWD/particlemethod_fsi_amd/lib_xcd/libmph_gpu.so MPH_XCD_DIAG=1 MPH_SLAB_OVERLAP=0 timeout -k 10 300 \
      python tools/slab_serial.py --case d16m --ranks 8 --steps 2 --warmup 2 > $OUT/xcd_slab.json 2>> $OUT/xcd.err || exit 15
fi
