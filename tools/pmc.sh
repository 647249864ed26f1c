#!/bin/bash
# Diagnostic PMC passes (one rocprofv3 --pmc run per counter group) on a short bench, in the
# timed region's store pattern (8-step batches; tools/pmc_fp64.py drops the init launch).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/pmc
mkdir -p $OUT
CASE=${CASE:-d1m}
timeout -k 10 120 rocprofv3 -L > $OUT/counters_list.txt 2>&1 || true
i=0
for grp in "$@"; do
  i=$((i+1))
  timeout -k 10 600 rocprofv3 --pmc $grp --output-format csv -d $OUT/g$i -o g$i -- \
      python3 bench.py --case $CASE --steps 8 --warmup 8 --no-cpu-baseline --developed-steps 0 --run-average-end 0 $BENCH_EXTRA --profile-steps 8 > $OUT/g$i.log 2>&1 || exit 30
done
