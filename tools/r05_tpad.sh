#!/bin/bash
# round 5: list tiles spaced by MPH_TILE_PAD extra rows (lib_tpad1/4/9), so the waves' rows do not
# share L2 sets: bitwise check, same-box A/B, developed WRITE_SIZE
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r05tpad
mkdir -p $OUT
CASES="box3d_jit gate3d_jit dam2d"
MPH_GPU_LIB=$PWD/particlemethod_fsi_amd/lib/libmph_gpu.so timeout -k 10 300 python3 tools/lib_bitwise.py run $OUT/base.npz $CASES > $OUT/bw_base.log 2>&1 || exit 11
MPH_GPU_LIB=$PWD/particlemethod_fsi_amd/lib_tpad9/libmph_gpu.so timeout -k 10 300 python3 tools/lib_bitwise.py run $OUT/tpad9.npz $CASES > $OUT/bw_tpad9.log 2>&1 || exit 12
python3 tools/lib_bitwise.py compare $OUT/base.npz $OUT/tpad9.npz > $OUT/bw_compare.log 2>&1 || exit 13
rm -f $OUT/base.npz $OUT/tpad9.npz
OUT=$OUT VARIANTS="tpad1 tpad4 tpad9" ROUNDS=2 bash tools/ab_dev.sh || exit 14
timeout -k 10 120 python3 tools/dev_state.py d1m 2500 $OUT/d1m_dev.gridb > $OUT/dev_state.log 2>&1 || exit 15
for v in tpad1 tpad9; do
  rm -rf gpurun_out/pmc
  MPH_GPU_LIB=$PWD/particlemethod_fsi_amd/lib_$v/libmph_gpu.so BENCH_EXTRA="--state $OUT/d1m_dev.gridb" bash tools/pmc.sh WRITE_SIZE || exit 16
  mv gpurun_out/pmc $OUT/pmc_dev_$v
done
rm -f $OUT/d1m_dev.gridb
