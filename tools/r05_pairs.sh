#!/bin/bash
# round 5: neighbour lists in pairs (MPH_LIST_PAIRS=1, lib_pairs) against rows: bitwise outputs,
# the neighbour-set tests on the pairs build, same-box A/B, WRITE_SIZE of the search at rest
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r05pairs
mkdir -p $OUT
CASES="dam2d box3d_jit gate3d_jit seam3d gate2d"
MPH_GPU_LIB=$PWD/particlemethod_fsi_amd/lib/libmph_gpu.so timeout -k 10 300 python3 tools/lib_bitwise.py run $OUT/rows.npz $CASES > $OUT/bw_rows.log 2>&1 || exit 11
MPH_GPU_LIB=$PWD/particlemethod_fsi_amd/lib_pairs/libmph_gpu.so timeout -k 10 300 python3 tools/lib_bitwise.py run $OUT/pairs.npz $CASES > $OUT/bw_pairs.log 2>&1 || exit 12
python3 tools/lib_bitwise.py compare $OUT/rows.npz $OUT/pairs.npz > $OUT/bw_compare.log 2>&1 || exit 13
rm -f $OUT/rows.npz $OUT/pairs.npz
MPH_GPU_LIB=$PWD/particlemethod_fsi_amd/lib_pairs/libmph_gpu.so timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_parity.py -k "neighbor_sets or trimmed" > $OUT/pytest_pairs.log 2>&1 || exit 14
OUT=$OUT VARIANTS="pairs" ROUNDS=2 D16M=1 bash tools/ab_dev.sh || exit 15
rm -rf gpurun_out/pmc
MPH_GPU_LIB=$PWD/particlemethod_fsi_amd/lib_pairs/libmph_gpu.so bash tools/pmc.sh WRITE_SIZE || exit 16
mv gpurun_out/pmc $OUT/pmc_write_pairs
