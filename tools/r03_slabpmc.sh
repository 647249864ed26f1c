#!/bin/bash
# One PMC pass over the D16M slabs (tools/slab_serial.py, one rank at a time): per-dispatch
# counters of pass B, split (overlap: the interior and the face launches) and unsplit
# (MPH_SLAB_OVERLAP=0), summarised by tools/slab_pmc_summary.py.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${OUT:-r03spmc}
mkdir -p $OUT
G="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE"
for mode in 1 0; do
  MPH_SLAB_OVERLAP=$mode timeout -s KILL 400 rocprofv3 --pmc $G --kernel-include-regex "k_pass_b" \
      --output-format csv -d $OUT/ov$mode -o ov$mode -- \
      python3 tools/slab_serial.py --case ${CASE:-d16m} --ranks ${RANKS:-8} --steps 2 --warmup 1 \
      > $OUT/ov$mode.log 2>&1 || exit 20
done
python3 tools/slab_pmc_summary.py $OUT > $OUT/summary.txt || exit 21
