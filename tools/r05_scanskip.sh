#!/bin/bash
# round 5: the scans skip the cell runs above every particle (MPH_SCAN_SKIP=1, default) against
# the full scans (lib_noskip): bitwise over 3-D and 2-D cases, the parity and slab tests, then
# same-box timing at rest, developed and D16M
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r05scanskip
mkdir -p $OUT
CASES="box3d gate3d seam3d d1m dam2d bar2d gate2d rolling3d movwall3d channel2d channel3d"
timeout -k 10 400 python3 tools/lib_bitwise.py run $OUT/a.npz $CASES > $OUT/bw_a.log 2>&1 || exit 10
MPH_GPU_LIB=$PWD/particlemethod_fsi_amd/lib_noskip/libmph_gpu.so timeout -k 10 400 python3 tools/lib_bitwise.py run $OUT/b.npz $CASES > $OUT/bw_b.log 2>&1 || exit 11
python3 tools/lib_bitwise.py compare $OUT/a.npz $OUT/b.npz > $OUT/bw_compare.log 2>&1 || exit 12
rm -f $OUT/a.npz $OUT/b.npz
timeout -k 10 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_dist.py tests/test_gpu_developed.py -k "not 10000" > $OUT/pytest.log 2>&1 || exit 13
OUT=$OUT VARIANTS="noskip" ROUNDS=2 D16M=1 bash tools/ab_dev.sh || exit 14
