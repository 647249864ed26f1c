#!/bin/bash
# round 5: the gather path of pass A with 48-byte interleaved records (default) and three 16-byte
# planes (lib_p6planes): L1 tag-RAM requests per bank, tag-conflict / pending / return stalls,
# UTCL1 (address translation), TA stalls, latencies -- one rocprofv3 pass per group, D1M at rest
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r05gpath
mkdir -p $OUT
G1="TCP_READ_TAGCONFLICT_STALL_CYCLES_sum TCP_PENDING_STALL_CYCLES_sum TCP_TCR_TCP_STALL_CYCLES_sum TCP_TCP_TA_DATA_STALL_CYCLES_sum GRBM_GUI_ACTIVE"
G2="TCP_TAGRAM0_REQ_sum TCP_TAGRAM1_REQ_sum TCP_TAGRAM2_REQ_sum TCP_TAGRAM3_REQ_sum GRBM_GUI_ACTIVE"
G3="TCP_UTCL1_REQUEST_sum TCP_UTCL1_STALL_MULTI_MISS_sum TCP_UTCL1_THRASHING_STALL_sum TCP_TCP_LATENCY_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum TA_DATA_STALLED_BY_TC_CYCLES_sum GRBM_GUI_ACTIVE"
G4="TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCP_TCC_READ_REQ_LATENCY_sum TCP_TOTAL_READ_sum GRBM_GUI_ACTIVE"
for v in base p6planes; do
  lib=$PWD/particlemethod_fsi_amd/lib/libmph_gpu.so
  [ $v != base ] && lib=$PWD/particlemethod_fsi_amd/lib_$v/libmph_gpu.so
  rm -rf gpurun_out/pmc
  MPH_GPU_LIB=$lib bash tools/pmc.sh "$G1" "$G2" "$G3" "$G4" || exit 11
  python3 tools/pmc_summary.py gpurun_out/pmc > $OUT/$v.txt
  mv gpurun_out/pmc $OUT/pmc_$v
done
