#!/bin/bash
# round 5, fourth call: contiguous-axis cell width (MPH_SA 2/3/4) at rest and in the developed flow;
# the slab + driver GPU tests on the probe fix
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r05sa
mkdir -p $OUT
timeout -k 10 120 python3 tools/dev_state.py d1m 2500 $OUT/d1m_dev.gridb > $OUT/dev_state.log 2>&1 || exit 11
for r in 1 2; do
for v in base sa3 sa4; do
  lib=$PWD/particlemethod_fsi_amd/lib/libmph_gpu.so
  [ $v != base ] && lib=$PWD/particlemethod_fsi_amd/lib_$v/libmph_gpu.so
  MPH_GPU_LIB=$lib timeout -k 10 300 python3 bench.py --state $OUT/d1m_dev.gridb --steps 20 --warmup 4 --no-cpu-baseline > $OUT/dev_${v}_$r.json 2> $OUT/dev_$v.err || exit 12
  MPH_GPU_LIB=$lib timeout -k 10 300 python3 bench.py --developed-steps 0 --steps 20 --warmup 4 --no-cpu-baseline > $OUT/rest_${v}_$r.json 2> $OUT/rest_$v.err || exit 13
done
done
rm -f $OUT/d1m_dev.gridb
timeout -k 10 900 python -u -m pytest tests/test_gpu_dist.py tests/test_gpu_driver.py tests/test_gpu_d16m.py -x -q --timeout 300 --timeout-method thread > $OUT/pytest_dist.log 2>&1
echo "pytest rc=$?" >> $OUT/pytest_dist.log
