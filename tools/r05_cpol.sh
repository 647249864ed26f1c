#!/bin/bash
# round 5: the search's FP32 record staging loads non-temporal (lib_cpol2: nt, lib_cpol3: sc0 nt),
# so that the staged records leave L2 before the partly written list rows, and the list stores
# non-temporal (lib_scpol2): same-box A/B and the developed flow's WRITE_SIZE / FETCH_SIZE
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r05cpol
mkdir -p $OUT
OUT=$OUT VARIANTS="cpol2 cpol3 scpol2" ROUNDS=2 bash tools/ab_dev.sh || exit 11
timeout -k 10 120 python3 tools/dev_state.py d1m 2500 $OUT/d1m_dev.gridb > $OUT/dev_state.log 2>&1 || exit 12
rm -rf gpurun_out/pmc
MPH_GPU_LIB=$PWD/particlemethod_fsi_amd/lib_cpol2/libmph_gpu.so BENCH_EXTRA="--state $OUT/d1m_dev.gridb" bash tools/pmc.sh WRITE_SIZE FETCH_SIZE || exit 13
mv gpurun_out/pmc $OUT/pmc_dev_cpol2
MPH_GPU_LIB=$PWD/particlemethod_fsi_amd/lib_scpol2/libmph_gpu.so BENCH_EXTRA="--state $OUT/d1m_dev.gridb" bash tools/pmc.sh WRITE_SIZE || exit 14
mv gpurun_out/pmc $OUT/pmc_dev_scpol2
rm -f $OUT/d1m_dev.gridb
