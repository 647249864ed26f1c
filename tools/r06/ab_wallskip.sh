#!/bin/bash
# Pass B skips a wall's list loop on the steps that do not store Force: bitwise against the build
# before (rev) on cases with walls (every step of lib_bitwise stores at the end of a batch, and the
# 3 + 8 step calls end batches mid-graph), the GPU suite's parity/edge/driver tests, then the A/B.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/${OUT:-ab_wallskip}
mkdir -p $O
L=$PWD/particlemethod_fsi_amd
CASES="box3d box3d_jit gate3d_jit seam3d dam2d box3d_st gate2d_sub movwall3d d1m"
MPH_GPU_LIB=$L/lib_rev/libmph_gpu.so timeout -k 10 240 python3 tools/lib_bitwise.py run $O/base.npz $CASES > $O/bw_base.log 2>&1 || exit 11
MPH_GPU_LIB=$L/lib/libmph_gpu.so timeout -k 10 240 python3 tools/lib_bitwise.py run $O/new.npz $CASES > $O/bw_new.log 2>&1 || exit 12
python3 tools/lib_bitwise.py compare $O/base.npz $O/new.npz > $O/bitwise.txt 2>&1
rm -f $O/base.npz $O/new.npz
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_edge.py tests/test_gpu_driver.py tests/test_gpu_dist.py > $O/pytest.log 2>&1 || exit 16
OUT=$O/t025 VARIANTS="rev" ROUNDS=2 bash tools/ab_dev.sh || exit 17
python3 tools/ab_dev_summary.py $O/t025 > $O/summary_t025.txt 2>&1
for r in 1 2; do
  for v in base rev; do
    lib=$L/lib/libmph_gpu.so; [ $v != base ] && lib=$L/lib_$v/libmph_gpu.so
    MPH_GPU_LIB=$lib timeout -k 10 300 python3 bench.py --case fsi3d_sub --steps 20 --warmup 4 --no-cpu-baseline > $O/fsi3d_sub_${v}_$r.json 2> $O/fsi_$v.err || exit 18
  done
done
