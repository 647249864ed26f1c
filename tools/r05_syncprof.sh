#!/bin/bash
# round 5: kernel traces of the unbatched call pattern, with and without the output-only stores
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r05syncprof
mkdir -p $OUT
for cs in bar2d_400k d1m; do
  timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $OUT/${cs}_store -o run -- python3 tools/sync_loop.py $cs 50 > $OUT/${cs}_store.log 2>&1 || exit 11
  MPH_DIAG_SYNC_NOSTORE=1 timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $OUT/${cs}_nostore -o run -- python3 tools/sync_loop.py $cs 50 > $OUT/${cs}_nostore.log 2>&1 || exit 12
done
