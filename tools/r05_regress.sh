#!/bin/bash
# round 5: D16M search regression check: the build before the chunked-search plumbing (lib_old,
# commit ed5f8f6) against the current one with that plumbing compiled out (MPH_CHUNK_BUILD=0)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r05regress
mkdir -p $OUT
OUT=$OUT VARIANTS="old" ROUNDS=2 D16M=1 bash tools/ab_dev.sh || exit 11
