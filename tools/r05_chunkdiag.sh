#!/bin/bash
# round 5: the search with 4- or 8-entry LDS chunks written as 16- or 32-byte stores (diagnostic builds lib_chunk, lib_chunk8,
# MPH_DIAG_CHUNK=1: the passes read nothing valid, so only the search time counts), same box, at
# rest, t = 0.25 s and t = 1.0 s
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r05chunk8
mkdir -p $OUT/t025 $OUT/t1
OUT=$OUT/t025 DEV_STEPS=2500 VARIANTS="chunk8" ROUNDS=2 bash tools/ab_dev.sh || exit 11
OUT=$OUT/t1 DEV_STEPS=10000 VARIANTS="chunk8" ROUNDS=2 bash tools/ab_dev.sh || exit 12
