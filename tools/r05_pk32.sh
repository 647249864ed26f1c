#!/bin/bash
# round 5: the search's candidate distances in packed FP32 (MPH_PK32=1, default) against scalar
# FP32 (lib_nopk): bitwise over the 3-D cases, then same-box timing at rest, developed and D16M
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r05pk32
mkdir -p $OUT
CASES="box3d box3d_st gate3d seam3d d1m box3d_jit gate3d_jit rolling3d movwall3d channel3d longz3d"
timeout -k 10 300 python3 tools/lib_bitwise.py run $OUT/a.npz $CASES > $OUT/bw_a.log 2>&1 || exit 10
MPH_GPU_LIB=$PWD/particlemethod_fsi_amd/lib_nopk/libmph_gpu.so timeout -k 10 300 python3 tools/lib_bitwise.py run $OUT/b.npz $CASES > $OUT/bw_b.log 2>&1 || exit 11
python3 tools/lib_bitwise.py compare $OUT/a.npz $OUT/b.npz > $OUT/bw_compare.log 2>&1 || exit 12
rm -f $OUT/a.npz $OUT/b.npz
OUT=$OUT VARIANTS="nopk" ROUNDS=3 D16M=1 bash tools/ab_dev.sh || exit 13
