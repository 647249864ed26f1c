#!/bin/bash
# round 5: the short scans (slab class counts, small structure grids) in one launch (k_scan_small,
# default) against scan_reduce + scan_down (lib_oldscan): bitwise over elastic cases, the slab and
# elastic tests, then D16M / 8 per rank one rank at a time (tools/slab_serial.py), both builds
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r05scansmall
mkdir -p $OUT
CASES="bar2d gate2d gate3d_sub box3d dam2d"
timeout -k 10 300 python3 tools/lib_bitwise.py run $OUT/a.npz $CASES > $OUT/bw_a.log 2>&1 || exit 10
MPH_GPU_LIB=$PWD/particlemethod_fsi_amd/lib_oldscan/libmph_gpu.so timeout -k 10 300 python3 tools/lib_bitwise.py run $OUT/b.npz $CASES > $OUT/bw_b.log 2>&1 || exit 11
python3 tools/lib_bitwise.py compare $OUT/a.npz $OUT/b.npz > $OUT/bw_compare.log 2>&1 || exit 12
rm -f $OUT/a.npz $OUT/b.npz
timeout -k 10 700 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_dist.py tests/test_gpu_d16m.py tests/test_gpu_driver.py > $OUT/pytest.log 2>&1 || exit 13
for v in base oldscan; do
  lib=$PWD/particlemethod_fsi_amd/lib/libmph_gpu.so
  [ $v != base ] && lib=$PWD/particlemethod_fsi_amd/lib_$v/libmph_gpu.so
  MPH_GPU_LIB=$lib MPH_SLAB_OVERLAP=0 timeout -k 10 300 python tools/slab_serial.py --case d16m --ranks 8 --steps 4 --warmup 2 > $OUT/serial_$v.json 2> $OUT/serial_$v.err || exit 14
done
