#!/bin/bash
# Full GPU evidence of the current tree: smoke, every GPU test, the D1M bench line, rocprofv3
# kernel stats + FETCH/WRITE PMC (timed store pattern), FP64 FLOP PMC, and the other configs.
# Each step time-limited; stops at the first failure.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/rc/smoke.log 2>&1 || exit 11
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 600 --timeout-method thread > gpurun_out/rc/pytest_gpu.log 2>&1 || exit 12
timeout -k 10 300 python bench.py > gpurun_out/rc/bench_d1m.json 2> gpurun_out/rc/bench_d1m.err || exit 13
STEPS=24 bash tools/profile.sh || exit 14
timeout -k 10 300 bash tools/pmc.sh SQ_INSTS_VALU_FLOPS_FP64 || exit 15
for c in ${CASES:-bar2d_400k fsi3d d16m}; do
  timeout -k 10 300 python bench.py --case $c --steps 24 --warmup 8 > gpurun_out/rc/bench_$c.json 2> gpurun_out/rc/bench_$c.err || exit 16
done
