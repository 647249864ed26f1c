#!/bin/bash
# round 5: pass-B records in planes, pass-A records interleaved (MPH_PLANES=1, MPH_P6_PLANES=0)
# against the round-4 layout (lib_noplanes): bitwise, A/B at rest / developed / D16M, GPU suite
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r05hyb
mkdir -p $OUT
NP=$PWD/particlemethod_fsi_amd/lib_noplanes/libmph_gpu.so
timeout -k 10 300 python tools/lib_bitwise.py run $OUT/bw_new.npz box3d box3d_st gate3d seam3d d1m box3d_jit gate2d > $OUT/bw_new.log 2>&1 || exit 11
MPH_GPU_LIB=$NP timeout -k 10 300 python tools/lib_bitwise.py run $OUT/bw_old.npz box3d box3d_st gate3d seam3d d1m box3d_jit gate2d > $OUT/bw_old.log 2>&1 || exit 12
python tools/lib_bitwise.py compare $OUT/bw_new.npz $OUT/bw_old.npz > $OUT/bw_compare.log 2>&1
rm -f $OUT/bw_*.npz
timeout -k 10 120 python3 tools/dev_state.py d1m 2500 $OUT/d1m_dev.gridb > $OUT/dev_state.log 2>&1 || exit 13
for r in 1 2; do
  for v in hyb noplanes; do
    lib=$PWD/particlemethod_fsi_amd/lib/libmph_gpu.so
    [ $v = noplanes ] && lib=$NP
    MPH_GPU_LIB=$lib timeout -k 10 300 python3 bench.py --developed-steps 0 --steps 20 --warmup 4 --no-cpu-baseline > $OUT/rest_${v}_$r.json 2> $OUT/rest_$v.err || exit 14
    MPH_GPU_LIB=$lib timeout -k 10 300 python3 bench.py --state $OUT/d1m_dev.gridb --steps 20 --warmup 4 --no-cpu-baseline > $OUT/dev_${v}_$r.json 2> $OUT/dev_$v.err || exit 15
    MPH_GPU_LIB=$lib timeout -k 10 300 python3 bench.py --case d16m --steps 12 --warmup 4 --no-cpu-baseline > $OUT/d16m_${v}_$r.json 2> $OUT/d16m_$v.err || exit 16
  done
done
rm -f $OUT/d1m_dev.gridb
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
echo "pytest rc=$?" >> $OUT/pytest_gpu.log
