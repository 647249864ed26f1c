#!/bin/bash
# round 5: the search's list write amplification against its occupancy (8 / 6 / 4 waves per SIMD by
# unused dynamic LDS, lib_pad7000 / lib_pad20000): developed-flow WRITE_SIZE and same-box times
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r05occ
mkdir -p $OUT
timeout -k 10 120 python3 tools/dev_state.py d1m 2500 $OUT/d1m_dev.gridb > $OUT/dev_state.log 2>&1 || exit 11
for v in base pad7000 pad20000; do
  lib=$PWD/particlemethod_fsi_amd/lib/libmph_gpu.so
  [ $v != base ] && lib=$PWD/particlemethod_fsi_amd/lib_$v/libmph_gpu.so
  rm -rf gpurun_out/pmc
  MPH_GPU_LIB=$lib BENCH_EXTRA="--state $OUT/d1m_dev.gridb" bash tools/pmc.sh WRITE_SIZE || exit 12
  mv gpurun_out/pmc $OUT/pmc_dev_$v
done
rm -f $OUT/d1m_dev.gridb
OUT=$OUT VARIANTS="pad7000 pad20000" ROUNDS=2 bash tools/ab_dev.sh || exit 13
