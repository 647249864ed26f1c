#!/bin/bash
# round 6: the cleaned product source (rejected variants removed) -- bitwise against e6081fe on
# every lib_bitwise case plus the D1M developed state, then the whole GPU suite
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/r06d
mkdir -p $OUT
REF=particlemethod_fsi_amd/lib/ref_e6081fe/libmph_gpu.so
CASES="box3d box3d_st gate3d seam3d d1m box3d_jit gate3d_jit dam2d bar2d gate2d_sub channel3d longz3d turek2d rolling3d"
MPH_ABI_ACCEPT=3 MPH_GPU_LIB=$REF timeout -k 10 300 python tools/lib_bitwise.py run $OUT/bw_ref.npz $CASES > $OUT/bw.log 2>&1 || exit 11
timeout -k 10 300 python tools/lib_bitwise.py run $OUT/bw_new.npz $CASES >> $OUT/bw.log 2>&1 || exit 12
python tools/lib_bitwise.py compare $OUT/bw_ref.npz $OUT/bw_new.npz >> $OUT/bw.log 2>&1
rm -f $OUT/bw_*.npz
timeout -k 10 1500 python -u -m pytest -x -v --timeout 600 --timeout-method thread -m gpu tests > $OUT/pytest.log 2>&1 || exit 13
