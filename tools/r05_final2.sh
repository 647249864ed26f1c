#!/bin/bash
# Round 5 final evidence, call B: the D1M bench line and the rocprofv3 kernel trace after the
# profiled launches moved to dispatch-packet timestamps (hipExtLaunchKernelGGL), then the developed
# flow's kernel trace and PMC issue groups (tools/r05_devprof.sh).  Chain stops at the first failure.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${OUT:-r05final2}
mkdir -p $OUT
timeout -k 10 400 python bench.py > $OUT/bench_d1m.json 2> $OUT/bench_d1m.err || exit 12
timeout -k 10 400 python bench.py --warmup 5 --steps 20 --no-cpu-baseline > $OUT/bench_driver_cmd.json 2> $OUT/bench_driver_cmd.err || exit 13
rm -rf gpurun_out/prof
bash tools/profile.sh || exit 15
mkdir -p $OUT/prof && cp -r gpurun_out/prof/kt gpurun_out/prof/fetch gpurun_out/prof/write $OUT/prof/ && cp gpurun_out/prof/*.log $OUT/prof/
bash tools/r05_devprof.sh || exit 16
