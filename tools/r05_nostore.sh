#!/bin/bash
# round 5: the cost of the search's list stores: diagnostic builds without the
# stores (lib_nostore1) and with the same store instructions all aimed at the lane's row 0
# (lib_nostore2: the instructions without the list traffic), same-box A/B at rest and developed,
# then WRITE_SIZE of the search for the default and the row-0 build
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r05nostore
mkdir -p $OUT
OUT=$OUT VARIANTS="nostore1 nostore2" ROUNDS=2 bash tools/ab_dev.sh || exit 11
for v in base nostore2; do
  lib=$PWD/particlemethod_fsi_amd/lib/libmph_gpu.so
  [ $v != base ] && lib=$PWD/particlemethod_fsi_amd/lib_$v/libmph_gpu.so
  rm -rf gpurun_out/pmc
  MPH_GPU_LIB=$lib bash tools/pmc.sh WRITE_SIZE || exit 12
  mv gpurun_out/pmc $OUT/pmc_write_$v
done
