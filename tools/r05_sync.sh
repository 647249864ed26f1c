#!/bin/bash
# round 5: the unbatched drop-in call pattern (step1.sync): polling wait on pinned flags (default)
# against the blocking wait (MPH_SYNC_WAIT=block), and without the output-only stores (diagnostic)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r05sync
mkdir -p $OUT
for r in 1 2; do
  for v in poll MPH_SYNC_WAIT=block MPH_DIAG_SYNC_NOSTORE=1; do
    envset=(); [[ "$v" == *=* ]] && envset=("$v")
    tag=${v//=/-}
    for cs in d1m bar2d_400k; do
      env "${envset[@]}" timeout -k 10 200 python3 bench.py --case $cs --developed-steps 0 --steps 100 --warmup 8 --no-cpu-baseline > $OUT/${cs}_${tag}_$r.json 2> $OUT/${cs}_$tag.err || exit 11
    done
  done
done
