#!/bin/bash
# round 5: the (y, x, z) cell order (MPH_SLAB_PERM=5) against the default (x, y, z), same box
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r05perm5
mkdir -p $OUT
OUT=$OUT VARIANTS="MPH_SLAB_PERM=5" ROUNDS=2 D16M=1 bash tools/ab_dev.sh || exit 11
