#!/bin/bash
# round 5: rocprofv3 kernel stats + PMC issue groups of D1M in the developed flow (t = 0.25 s,
# tools/dev_state.py), beside the same at rest
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r05dev
mkdir -p $OUT
timeout -k 10 120 python3 tools/dev_state.py d1m 2500 $OUT/d1m_dev.gridb > $OUT/dev_state.log 2>&1 || exit 11
timeout -k 10 300 python3 bench.py --state $OUT/d1m_dev.gridb --warmup 5 --steps 20 --no-cpu-baseline > $OUT/bench_dev.json 2> $OUT/bench_dev.err || exit 12
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kt -o kt -- \
    python3 bench.py --state $OUT/d1m_dev.gridb --steps 24 --warmup 8 --no-cpu-baseline > $OUT/bench_under_kt.log 2>&1 || exit 13
G1="SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_WAIT_INST_ANY"
G2="SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM SQ_WAIT_ANY TA_BUSY_avr TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum GRBM_GUI_ACTIVE"
rm -rf gpurun_out/pmc
BENCH_EXTRA="--state $OUT/d1m_dev.gridb" bash tools/pmc.sh "$G1" "$G2" || exit 14
mv gpurun_out/pmc $OUT/pmc_dev
python3 tools/pmc_summary.py $OUT/pmc_dev > $OUT/pmc_dev.txt
python3 tools/pmc_issue.py $OUT/pmc_dev.txt d1m_dev > $OUT/pmc_issue_dev.json
rm -f $OUT/d1m_dev.gridb
