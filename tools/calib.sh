#!/bin/bash
# FETCH_SIZE / WRITE_SIZE calibration on kernels of known bytes (tools/pmc_calib.hip): one run for
# the byte counts, then one --pmc pass per counter.  Time-limited; stops at the first failure.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/calib
mkdir -p $OUT
timeout -k 10 120 ./tools/_build/pmc_calib > $OUT/known.json || exit 31
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/fetch -o fetch -- \
    ./tools/_build/pmc_calib > $OUT/fetch.log 2>&1 || exit 32
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/write -o write -- \
    ./tools/_build/pmc_calib > $OUT/write.log 2>&1 || exit 33
