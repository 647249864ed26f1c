#!/bin/bash
# Bench lines for every single-GPU BASELINE config (bench.py --case): Bar (configs[2]), FSI
# (configs[3]) and D16M on one GPU (the per-GPU share of configs[4] is D1M-sized; this is the
# whole 16M tank on one card).  Every GPU step is time-limited; the chain stops at the first failure.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/configs
for c in ${CASES:-bar2d_400k fsi3d d16m}; do
  extra=""
  [ "$c" = d16m ] && extra="--no-cpu-baseline"
  timeout -k 10 600 python bench.py --case $c --steps ${STEPS:-20} --warmup 4 $extra \
      > gpurun_out/configs/bench_$c.json 2> gpurun_out/configs/bench_$c.err || exit 30
done
