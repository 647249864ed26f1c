#!/bin/bash
# round 5: the search's list-store cost at t = 1.0 s (10,000 steps): no stores (lib_nostore1) and
# the same store instructions on the lane's row 0 (lib_nostore2), same box
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r05nostore_t1
mkdir -p $OUT
OUT=$OUT DEV_STEPS=10000 VARIANTS="nostore1 nostore2" ROUNDS=2 bash tools/ab_dev.sh || exit 11
