#!/bin/bash
# round 5: confirmation A/B of one padded row between list tiles (lib_tpad1), three rounds + D16M
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r05tpad1
mkdir -p $OUT
OUT=$OUT VARIANTS="tpad1" ROUNDS=3 D16M=1 bash tools/ab_dev.sh || exit 11
