#!/bin/bash
# round 5: CU-affine tiles of the list kernels (MPH_CU_AFFINE=1, lib_cuaff): bitwise outputs with
# the XCD map forced on small cases, the parity subset on that build, same-box A/B, and the L1 ->
# L2 read requests of the list kernels at rest
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r05cuaff
mkdir -p $OUT
CASES="dam2d box3d_jit gate3d_jit seam3d gate2d"
MPH_XCD_BAL_MIN=0 MPH_GPU_LIB=$PWD/particlemethod_fsi_amd/lib/libmph_gpu.so timeout -k 10 300 python3 tools/lib_bitwise.py run $OUT/base.npz $CASES > $OUT/bw_base.log 2>&1 || exit 11
MPH_XCD_BAL_MIN=0 MPH_GPU_LIB=$PWD/particlemethod_fsi_amd/lib_cuaff/libmph_gpu.so timeout -k 10 300 python3 tools/lib_bitwise.py run $OUT/cuaff.npz $CASES > $OUT/bw_cuaff.log 2>&1 || exit 12
python3 tools/lib_bitwise.py compare $OUT/base.npz $OUT/cuaff.npz > $OUT/bw_compare.log 2>&1 || exit 13
rm -f $OUT/base.npz $OUT/cuaff.npz
MPH_XCD_BAL_MIN=0 MPH_GPU_LIB=$PWD/particlemethod_fsi_amd/lib_cuaff/libmph_gpu.so timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_parity.py -k "neighbor_sets or trimmed or golden or every_step or profile_graphs" > $OUT/pytest_cuaff.log 2>&1 || exit 14
OUT=$OUT VARIANTS="cuaff" ROUNDS=2 D16M=1 bash tools/ab_dev.sh || exit 15
G="TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCP_PENDING_STALL_CYCLES_sum TCP_READ_TAGCONFLICT_STALL_CYCLES_sum GRBM_GUI_ACTIVE"
for v in base cuaff; do
  lib=$PWD/particlemethod_fsi_amd/lib/libmph_gpu.so
  [ $v != base ] && lib=$PWD/particlemethod_fsi_amd/lib_$v/libmph_gpu.so
  rm -rf gpurun_out/pmc
  MPH_GPU_LIB=$lib bash tools/pmc.sh "$G" || exit 16
  python3 tools/pmc_summary.py gpurun_out/pmc > $OUT/pmc_$v.txt
  rm -rf gpurun_out/pmc
done
