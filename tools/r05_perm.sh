#!/bin/bash
# round 5: the cell orders (MPH_SLAB_PERM=1..4 force an axis order on a 3-D context) at rest and in
# the developed flow
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r05perm
mkdir -p $OUT
OUT=$OUT VARIANTS="MPH_SLAB_PERM=1 MPH_SLAB_PERM=2 MPH_SLAB_PERM=3 MPH_SLAB_PERM=4" ROUNDS=1 bash tools/ab_dev.sh || exit 11
