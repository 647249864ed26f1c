#!/bin/bash
# Round 6 final evidence on the final build: smoke, the D1M bench line (default flags: developed,
# run_average and the CPU baseline), the driver's command, the other single-GPU configs (fsi3d_sub
# the stable FSI workload, fsi3d the survey's ElasticDt = Dt configuration), the rocprofv3
# kernel-trace + FETCH/WRITE passes of D1M (tools/profile.sh), the PMC issue groups and the FP64
# FLOP counter.  Every GPU step is time-limited; the chain stops at the first failure.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
OUT=gpurun_out/${OUT:-r06final}
mkdir -p $OUT
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || exit 11
timeout -k 10 500 python bench.py > $OUT/bench_d1m.json 2> $OUT/bench_d1m.err || exit 12
timeout -k 10 400 python bench.py --warmup 5 --steps 20 --no-cpu-baseline > $OUT/bench_driver_cmd.json 2> $OUT/bench_driver_cmd.err || exit 13
for c in fsi3d_sub bar2d_400k fsi3d d16m; do
  extra=""
  [ "$c" = d16m ] && extra="--no-cpu-baseline"
  timeout -k 10 600 python bench.py --case $c --steps 20 --warmup 4 $extra > $OUT/bench_$c.json 2> $OUT/bench_$c.err || exit 14
done
bash tools/profile.sh || exit 15
mkdir -p $OUT/prof && cp -r gpurun_out/prof/kt gpurun_out/prof/fetch gpurun_out/prof/write $OUT/prof/ && cp gpurun_out/prof/*.log $OUT/prof/
rm -rf gpurun_out/pmc_base gpurun_out/pmc
VARIANTS=base bash tools/pmc_ab.sh || exit 16
cp gpurun_out/pmc_base.txt $OUT/pmc_issue_groups.txt
rm -rf gpurun_out/pmc
bash tools/pmc.sh "SQ_INSTS_VALU_FLOPS_FP64 SQ_WAVES" || exit 17
mkdir -p $OUT/pmc_fp64 && cp -r gpurun_out/pmc/g1 $OUT/pmc_fp64/
