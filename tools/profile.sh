#!/bin/bash
# rocprofv3 evidence for profiles/: one kernel-trace + stats pass, then one PMC pass per TCC
# counter (FETCH_SIZE and WRITE_SIZE do not fit one pass on gfx950; MI355X_MICROARCH.md PMC slots).
# The PMC passes replay the same store pattern as the timed region: 8-step graphs (the first 7
# steps skip the output-only stores) and an 8-step profiled batch; tools/pmc_traffic.py drops each
# kernel's first launch (the initialisation sums of mph_create).
# Every GPU step is time-limited; the chain stops at the first failure.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/prof
mkdir -p $OUT
CASE=${CASE:-d1m}
ARGS="--case $CASE --steps ${STEPS:-24} --warmup 8 --no-cpu-baseline --developed-steps 0 --run-average-end 0 $BENCH_EXTRA"
PMC_ARGS="--case $CASE --steps 8 --warmup 8 --profile-steps 8 --no-cpu-baseline --developed-steps 0 --run-average-end 0 $BENCH_EXTRA"
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kt -o kt -- \
    python3 bench.py $ARGS > $OUT/bench_under_kt.log 2>&1 || exit 21
timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/fetch -o fetch -- \
    python3 bench.py $PMC_ARGS > $OUT/fetch.log 2>&1 || exit 22
timeout -k 10 600 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/write -o write -- \
    python3 bench.py $PMC_ARGS > $OUT/write.log 2>&1 || exit 23
