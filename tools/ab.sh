#!/bin/bash
# A/B timing of alternative builds (particlemethod_fsi_amd/lib_<name>/libmph_gpu.so, made with
# `make -C particlemethod_fsi_amd/csrc OUT=../lib_<name> EXTRA=-D...`) on the D1M bench.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for name in base ${VARIANTS}; do
  lib=particlemethod_fsi_amd/lib/libmph_gpu.so
  [ "$name" != base ] && lib=particlemethod_fsi_amd/lib_$name/libmph_gpu.so
  MPH_GPU_LIB=$PWD/$lib timeout -k 10 300 python bench.py --case ${CASE:-d1m} --steps 20 --warmup 4 \
      --no-cpu-baseline > gpurun_out/ab_$name.log 2>&1 || exit 40
done
