#!/bin/bash
# Round 6 final evidence on the aligned-rows build: smoke, the D1M bench line (default flags:
# developed, run_average and the CPU baseline), the driver's command, the other single-GPU configs,
# the rocprofv3 kernel-trace + FETCH/WRITE passes of D1M at rest (tools/profile.sh) and of the
# developed states t = 0.25 s and t = 1.0 s (FETCH/WRITE), the PMC issue groups and the FP64
# counter.  Every GPU step is time-limited; the chain stops at the first failure.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
OUT=gpurun_out/${OUT:-r06final2}
mkdir -p $OUT
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || exit 11
timeout -k 10 500 python bench.py > $OUT/bench_d1m.json 2> $OUT/bench_d1m.err || exit 12
timeout -k 10 400 python bench.py --warmup 5 --steps 20 --no-cpu-baseline > $OUT/bench_driver_cmd.json 2> $OUT/bench_driver_cmd.err || exit 13
for c in fsi3d_sub bar2d_400k fsi3d d16m; do
  extra=""
  [ "$c" = d16m ] && extra="--no-cpu-baseline"
  timeout -k 10 600 python bench.py --case $c --steps 20 --warmup 4 $extra > $OUT/bench_$c.json 2> $OUT/bench_$c.err || exit 14
done
rm -rf gpurun_out/prof
bash tools/profile.sh || exit 15
mkdir -p $OUT/prof && cp -r gpurun_out/prof/kt gpurun_out/prof/fetch gpurun_out/prof/write $OUT/prof/ && cp gpurun_out/prof/*.log $OUT/prof/
for st in 2500 10000; do
  timeout -k 10 200 python3 tools/dev_state.py d1m $st /tmp/d1m_$st.gridb > $OUT/dev_state_$st.log 2>&1 || exit 18
  export BENCH_EXTRA="--state /tmp/d1m_$st.gridb"
  timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/dev$st/fetch -o fetch -- \
      python3 bench.py --steps 8 --warmup 8 --profile-steps 8 --no-cpu-baseline --developed-steps 0 --run-average-end 0 $BENCH_EXTRA > $OUT/dev$st.fetch.log 2>&1 || exit 19
  timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/dev$st/write -o write -- \
      python3 bench.py --steps 8 --warmup 8 --profile-steps 8 --no-cpu-baseline --developed-steps 0 --run-average-end 0 $BENCH_EXTRA > $OUT/dev$st.write.log 2>&1 || exit 20
  unset BENCH_EXTRA
  rm -f /tmp/d1m_$st.gridb
done
rm -rf gpurun_out/pmc_base gpurun_out/pmc
VARIANTS=base bash tools/pmc_ab.sh || exit 16
cp gpurun_out/pmc_base.txt $OUT/pmc_issue_groups.txt
rm -rf gpurun_out/pmc
bash tools/pmc.sh "SQ_INSTS_VALU_FLOPS_FP64 SQ_WAVES" || exit 17
mkdir -p $OUT/pmc_fp64 && cp -r gpurun_out/pmc/g1 $OUT/pmc_fp64/
