#!/bin/bash
# round 5: smoke and the bench lines on the last build (k_scan_top in one pass): D1M default, the
# driver's command and D16M
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r05final7
mkdir -p $OUT
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || exit 11
timeout -k 10 400 python bench.py > $OUT/bench_d1m.json 2> $OUT/bench_d1m.err || exit 12
timeout -k 10 400 python bench.py --warmup 5 --steps 20 --no-cpu-baseline > $OUT/bench_driver_cmd.json 2> $OUT/bench_driver_cmd.err || exit 13
timeout -k 10 600 python bench.py --case d16m --steps 20 --warmup 4 --no-cpu-baseline > $OUT/bench_d16m.json 2> $OUT/bench_d16m.err || exit 14
