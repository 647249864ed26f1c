#!/bin/bash
# round 5: proportional list rows (MPH_LIST_SPREAD=1, lib_spread) against plain rows: bitwise outputs,
# the neighbour-set tests on that build, same-box A/B, WRITE_SIZE of the search at rest and developed
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r05spread
mkdir -p $OUT
CASES="dam2d box3d_jit gate3d_jit seam3d gate2d"
MPH_GPU_LIB=$PWD/particlemethod_fsi_amd/lib/libmph_gpu.so timeout -k 10 300 python3 tools/lib_bitwise.py run $OUT/rows.npz $CASES > $OUT/bw_rows.log 2>&1 || exit 11
MPH_GPU_LIB=$PWD/particlemethod_fsi_amd/lib_spread/libmph_gpu.so timeout -k 10 300 python3 tools/lib_bitwise.py run $OUT/spread.npz $CASES > $OUT/bw_spread.log 2>&1 || exit 12
python3 tools/lib_bitwise.py compare $OUT/rows.npz $OUT/spread.npz > $OUT/bw_compare.log 2>&1 || exit 13
rm -f $OUT/rows.npz $OUT/spread.npz
MPH_GPU_LIB=$PWD/particlemethod_fsi_amd/lib_spread/libmph_gpu.so timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_parity.py -k "neighbor_sets or trimmed or golden or every_step or developed" > $OUT/pytest_spread.log 2>&1 || exit 14
OUT=$OUT VARIANTS="spread" ROUNDS=2 D16M=1 bash tools/ab_dev.sh || exit 15
rm -rf gpurun_out/pmc
MPH_GPU_LIB=$PWD/particlemethod_fsi_amd/lib_spread/libmph_gpu.so bash tools/pmc.sh WRITE_SIZE || exit 16
mv gpurun_out/pmc $OUT/pmc_write_spread
timeout -k 10 120 python3 tools/dev_state.py d1m 2500 $OUT/d1m_dev.gridb > $OUT/dev_state.log 2>&1 || exit 17
for v in spread; do
  lib=$PWD/particlemethod_fsi_amd/lib/libmph_gpu.so
  [ $v != base ] && lib=$PWD/particlemethod_fsi_amd/lib_$v/libmph_gpu.so
  rm -rf gpurun_out/pmc
  MPH_GPU_LIB=$lib BENCH_EXTRA="--state $OUT/d1m_dev.gridb" bash tools/pmc.sh WRITE_SIZE || exit 18
  mv gpurun_out/pmc $OUT/pmc_dev_$v
done
rm -f $OUT/d1m_dev.gridb
