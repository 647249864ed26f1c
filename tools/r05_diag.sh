#!/bin/bash
# round 5: where the developed flow's extra time goes -- the diagnostic builds of the search
# (MPH_DIAG_SEARCH=2 set-up only, =1 staging without tests, MPH_DIAG_NOSTORE=1 no list stores) and
# of the passes (MPH_DIAG_GATHER=1 coherent dummy gathers), at rest and from the developed state
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r05diag
mkdir -p $OUT
timeout -k 10 120 python3 tools/dev_state.py d1m 2500 $OUT/d1m_dev.gridb > $OUT/dev_state.log 2>&1 || exit 11
for v in base dsearch2 dsearch1 dnostore dgather r2; do
  lib=$PWD/particlemethod_fsi_amd/lib/libmph_gpu.so
  [ $v != base ] && lib=$PWD/particlemethod_fsi_amd/lib_$v/libmph_gpu.so
  MPH_GPU_LIB=$lib timeout -k 10 300 python3 bench.py --state $OUT/d1m_dev.gridb --steps 20 --warmup 4 --no-cpu-baseline > $OUT/dev_$v.json 2> $OUT/dev_$v.err || exit 12
  MPH_GPU_LIB=$lib timeout -k 10 300 python3 bench.py --developed-steps 0 --steps 20 --warmup 4 --no-cpu-baseline > $OUT/rest_$v.json 2> $OUT/rest_$v.err || exit 13
done
rm -f $OUT/d1m_dev.gridb
