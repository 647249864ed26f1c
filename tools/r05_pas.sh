#!/bin/bash
# round 5: pass A of the interior waves in its own staged kernel (MPH_PA_STAGED=1, lib_pas):
# bitwise against the default build, then A/B at rest / developed / D16M
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r05pas
mkdir -p $OUT
PAS=$PWD/particlemethod_fsi_amd/lib_pas/libmph_gpu.so
MPH_GPU_LIB=$PAS timeout -k 10 300 python tools/lib_bitwise.py run $OUT/bw_new.npz box3d box3d_st gate3d seam3d d1m box3d_jit gate2d > $OUT/bw_new.log 2>&1 || exit 11
timeout -k 10 300 python tools/lib_bitwise.py run $OUT/bw_old.npz box3d box3d_st gate3d seam3d d1m box3d_jit gate2d > $OUT/bw_old.log 2>&1 || exit 12
python tools/lib_bitwise.py compare $OUT/bw_new.npz $OUT/bw_old.npz > $OUT/bw_compare.log 2>&1
rm -f $OUT/bw_*.npz
OUT=$OUT VARIANTS="pas" D16M=1 bash tools/ab_dev.sh || exit 13
