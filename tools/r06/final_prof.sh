#!/bin/bash
# Round 6 final evidence, profiles only (the bench lines of tools/r06/final.sh are in
# gpurun_out/r06final): rocprofv3 kernel trace + FETCH/WRITE passes of D1M, PMC issue groups, FP64.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
OUT=gpurun_out/${OUT:-r06final}
mkdir -p $OUT
rm -rf gpurun_out/prof
bash tools/profile.sh || exit 15
mkdir -p $OUT/prof && cp -r gpurun_out/prof/kt gpurun_out/prof/fetch gpurun_out/prof/write $OUT/prof/ && cp gpurun_out/prof/*.log $OUT/prof/
rm -rf gpurun_out/pmc_base gpurun_out/pmc
VARIANTS=base bash tools/pmc_ab.sh || exit 16
cp gpurun_out/pmc_base.txt $OUT/pmc_issue_groups.txt
rm -rf gpurun_out/pmc
bash tools/pmc.sh "SQ_INSTS_VALU_FLOPS_FP64 SQ_WAVES" || exit 17
mkdir -p $OUT/pmc_fp64 && cp -r gpurun_out/pmc/g1 $OUT/pmc_fp64/
