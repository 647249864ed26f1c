#!/bin/bash
# round 5, third call: block totals (k_prep, zeroed by the scan) bitwise + A/B, the developed-flow
# diagnostics, then the GPU suite
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r05bsum2
mkdir -p $OUT
timeout -k 10 300 python tools/lib_bitwise.py run $OUT/bw_new.npz box3d box3d_st gate3d seam3d d1m box3d_jit gate2d > $OUT/bw_new.log 2>&1 || exit 11
MPH_GPU_LIB=$PWD/particlemethod_fsi_amd/lib_nobsum/libmph_gpu.so timeout -k 10 300 python tools/lib_bitwise.py run $OUT/bw_old.npz box3d box3d_st gate3d seam3d d1m box3d_jit gate2d > $OUT/bw_old.log 2>&1 || exit 12
python tools/lib_bitwise.py compare $OUT/bw_new.npz $OUT/bw_old.npz > $OUT/bw_compare.log 2>&1
rm -f $OUT/bw_*.npz
for r in 1 2; do
  CASES="d1m d16m" VARIANTS="nobsum" bash tools/ab.sh || exit 13
  for f in gpurun_out/ab_*.log; do mv $f $OUT/$(basename $f .log)_$r.log; done
done
bash tools/r05_diag.sh || exit 14
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
echo "pytest rc=$?" >> $OUT/pytest_gpu.log
