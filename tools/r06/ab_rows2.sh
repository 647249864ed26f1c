#!/bin/bash
# Aligned list rows, second A/B: the build (base) against the same code without jumps (nj: the
# format's cost alone), without jumps and the old 512-row tiles (nj512: the tile stride's cost) and
# the previous build (r6base); bitwise against r6base first.  Developed states t = 0.25 s and 1.0 s.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/${OUT:-ab_rows2}
mkdir -p $O
L=$PWD/particlemethod_fsi_amd
CASES="box3d box3d_jit gate3d_jit seam3d dam2d gate2d_sub d1m"
MPH_GPU_LIB=$L/lib_r6base/libmph_gpu.so timeout -k 10 240 python3 tools/lib_bitwise.py run $O/base.npz $CASES > $O/bw_base.log 2>&1 || exit 11
MPH_GPU_LIB=$L/lib/libmph_gpu.so timeout -k 10 240 python3 tools/lib_bitwise.py run $O/new.npz $CASES > $O/bw_new.log 2>&1 || exit 12
python3 tools/lib_bitwise.py compare $O/base.npz $O/new.npz > $O/bitwise.txt 2>&1
rm -f $O/base.npz $O/new.npz
OUT=$O/t025 VARIANTS="nj nj512 r6base" ROUNDS=2 bash tools/ab_dev.sh || exit 17
python3 tools/ab_dev_summary.py $O/t025 > $O/summary_t025.txt 2>&1
OUT=$O/t100 DEV_STEPS=10000 VARIANTS="nj r6base" ROUNDS=1 bash tools/ab_dev.sh || exit 18
python3 tools/ab_dev_summary.py $O/t100 > $O/summary_t100.txt 2>&1
