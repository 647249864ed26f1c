#!/bin/bash
# L2 (TCC) behaviour of the D1M kernels for the product build ("base") and alternative builds
# (lib_<name>): hits, misses, EA read requests and their outstanding level (level / requests = mean
# cycles an L2 miss waits for its fill) -> gpurun_out/pmc_tcc_<name>.txt (tools/pmc_summary.py).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
G3="TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_LEVEL_sum GRBM_GUI_ACTIVE SQ_WAVES"
for v in ${VARIANTS:-base}; do
  lib=particlemethod_fsi_amd/lib/libmph_gpu.so
  [ "$v" != base ] && lib=particlemethod_fsi_amd/lib_$v/libmph_gpu.so
  export MPH_GPU_LIB=$PWD/$lib
  rm -rf gpurun_out/pmc gpurun_out/pmc_tcc_$v
  mkdir -p gpurun_out/pmc_tcc_$v
  bash tools/pmc.sh "$G3" || exit 30
  mv gpurun_out/pmc/* gpurun_out/pmc_tcc_$v/
  python tools/pmc_summary.py gpurun_out/pmc_tcc_$v > gpurun_out/pmc_tcc_$v.txt
done
