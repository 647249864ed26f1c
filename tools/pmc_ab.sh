#!/bin/bash
# Diagnostic PMC groups (issue, waits, LDS, L1/TA) of the D1M bench for the product build ("base")
# and alternative builds (lib_<name>) or run-time settings (VAR=VALUE): gpurun_out/pmc_<name>.txt, per kernel (tools/pmc_summary.py).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
G1="SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_WAIT_INST_ANY"
G2="SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM SQ_WAIT_ANY TA_BUSY_avr TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum GRBM_GUI_ACTIVE"
for v in ${VARIANTS:-base}; do
  lib=particlemethod_fsi_amd/lib/libmph_gpu.so
  envv=()
  if [[ "$v" == *=* ]]; then envv=("$v")   # a run-time setting on the base library
  elif [ "$v" != base ]; then lib=particlemethod_fsi_amd/lib_$v/libmph_gpu.so; fi
  export MPH_GPU_LIB=$PWD/$lib
  rm -rf gpurun_out/pmc gpurun_out/pmc_$v
  mkdir -p gpurun_out/pmc_$v
  env "${envv[@]}" bash tools/pmc.sh "$G1" "$G2" || exit 30
  mv gpurun_out/pmc/* gpurun_out/pmc_$v/
  python tools/pmc_summary.py gpurun_out/pmc_$v > gpurun_out/pmc_$v.txt
done
