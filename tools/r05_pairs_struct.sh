#!/bin/bash
# round 5: precomputed structure pair records (MPH_STRUCT_PAIRS=1, default) against the per-substep
# gather + struct_pair (lib_nopairs): bitwise over the elastic cases, the elastic GPU tests, then
# same-box timing of Bar 400k and FSI
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r05spairs
mkdir -p $OUT
CASES="bar2d gate2d gate2d_sub gate3d gate3d_sub bar3d turek2d hydro2d gate2d_rolling1 bar2d_ivp fsi3d"
timeout -k 10 300 python3 tools/lib_bitwise.py run $OUT/a.npz $CASES > $OUT/bw_a.log 2>&1 || exit 10
MPH_GPU_LIB=$PWD/particlemethod_fsi_amd/lib_nopairs/libmph_gpu.so timeout -k 10 300 python3 tools/lib_bitwise.py run $OUT/b.npz $CASES > $OUT/bw_b.log 2>&1 || exit 11
python3 tools/lib_bitwise.py compare $OUT/a.npz $OUT/b.npz > $OUT/bw_compare.log 2>&1 || exit 12
rm -f $OUT/a.npz $OUT/b.npz
timeout -k 10 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_parity.py -k "struct or bar or gate or turek or hydro" > $OUT/pytest.log 2>&1 || exit 13
for r in 1 2 3; do
  for v in base nopairs; do
    lib=$PWD/particlemethod_fsi_amd/lib/libmph_gpu.so
    [ $v != base ] && lib=$PWD/particlemethod_fsi_amd/lib_$v/libmph_gpu.so
    for cs in bar2d_400k fsi3d; do
      MPH_GPU_LIB=$lib timeout -k 10 300 python3 bench.py --case $cs --developed-steps 0 --steps 20 --warmup 4 --no-cpu-baseline > $OUT/${cs}_${v}_$r.json 2> $OUT/${cs}_$v.err || exit 14
    done
  done
done
