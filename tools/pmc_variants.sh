#!/bin/bash
# FETCH_SIZE / WRITE_SIZE passes (tools/pmc.sh) for the product build and alternative builds
# (particlemethod_fsi_amd/lib_<name>/libmph_gpu.so), into gpurun_out/pmc_<name>_{fetch,write}.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for v in base ${VARIANTS}; do
  if [ "$v" = base ]; then lib=particlemethod_fsi_amd/lib/libmph_gpu.so; else lib=particlemethod_fsi_amd/lib_$v/libmph_gpu.so; fi
  for c in FETCH_SIZE WRITE_SIZE; do
    MPH_GPU_LIB=$PWD/$lib bash tools/pmc.sh "$c" || exit 30
    rm -rf gpurun_out/pmc_${v}_$c; mv gpurun_out/pmc gpurun_out/pmc_${v}_$c
  done
done
