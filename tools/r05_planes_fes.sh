#!/bin/bash
# round 5: F, E, S in element planes -- the whole GPU suite, then the unbatched call pattern's
# kernel trace and the bench's step1 lines for Bar and FSI
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r05fes
mkdir -p $OUT
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || exit 11
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/bar_sync -o run -- python3 tools/sync_loop.py bar2d_400k 50 > $OUT/bar_sync.log 2>&1 || exit 12
for cs in bar2d_400k fsi3d; do
  timeout -k 10 200 python3 bench.py --case $cs --developed-steps 0 --steps 100 --warmup 8 --no-cpu-baseline > $OUT/${cs}.json 2> $OUT/${cs}.err || exit 13
done
