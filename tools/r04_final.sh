#!/bin/bash
# Round 4 final evidence (one gpurun call): smoke, the D1M bench line (default flags), the other
# single-GPU BASELINE configs, the rocprofv3 kernel-trace + FETCH/WRITE passes of D1M
# (tools/profile.sh), and D16M in 8 slabs one rank at a time with the exchange replayed, in the
# default configuration.  Every GPU step is time-limited; the chain stops at the first failure.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${OUT:-r04final}
mkdir -p $OUT
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || exit 11
timeout -k 10 400 python bench.py > $OUT/bench_d1m.json 2> $OUT/bench_d1m.err || exit 12
for c in ${CASES:-bar2d_400k fsi3d d16m}; do
  extra=""
  [ "$c" = d16m ] && extra="--no-cpu-baseline"
  timeout -k 10 600 python bench.py --case $c --steps 20 --warmup 4 $extra > $OUT/bench_$c.json 2> $OUT/bench_$c.err || exit 13
done
bash tools/profile.sh || exit 14
mkdir -p $OUT/prof && cp -r gpurun_out/prof/kt $OUT/prof/ && cp -r gpurun_out/prof/fetch gpurun_out/prof/write $OUT/prof/ \
    && cp gpurun_out/prof/*.log $OUT/prof/
if [ -n "$SERIAL" ]; then
  timeout -k 10 400 python tools/slab_serial.py --case d16m --ranks 8 --steps 6 --warmup 2 --replay \
      > $OUT/serial_d16m_8.json 2> $OUT/serial.err || exit 15
fi
