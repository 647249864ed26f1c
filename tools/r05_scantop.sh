#!/bin/bash
# round 5: k_scan_top as one pass of per-thread runs: bitwise (every scan through k_scan_top,
# lib_topalways, against the default) and D16M timing against the previous kernel (lib_oldtop)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r05scantop
mkdir -p $OUT
CASES="box3d gate3d seam3d d1m bar2d gate3d_sub channel3d"
timeout -k 10 300 python3 tools/lib_bitwise.py run $OUT/a.npz $CASES > $OUT/bw_a.log 2>&1 || exit 10
MPH_GPU_LIB=$PWD/particlemethod_fsi_amd/lib_topalways/libmph_gpu.so timeout -k 10 300 python3 tools/lib_bitwise.py run $OUT/b.npz $CASES > $OUT/bw_b.log 2>&1 || exit 11
python3 tools/lib_bitwise.py compare $OUT/a.npz $OUT/b.npz > $OUT/bw_compare.log 2>&1 || exit 12
rm -f $OUT/a.npz $OUT/b.npz
for r in 1 2 3; do
  for v in base oldtop; do
    lib=$PWD/particlemethod_fsi_amd/lib/libmph_gpu.so
    [ $v != base ] && lib=$PWD/particlemethod_fsi_amd/lib_$v/libmph_gpu.so
    MPH_GPU_LIB=$lib timeout -k 10 300 python3 bench.py --case d16m --steps 12 --warmup 4 --no-cpu-baseline > $OUT/d16m_${v}_$r.json 2> $OUT/d16m_$v.err || exit 13
  done
done
