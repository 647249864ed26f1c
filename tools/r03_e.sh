#!/bin/bash
# Round 3 session: all GPU tests; D16M / 8 slabs one rank at a time (tools/slab_serial.py, with
# and without the pass-B overlap); D1M bench; PMC of the fused search + pass A (MPH_FUSED=1).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${OUT:-r03e}
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
rc=$?
echo "pytest rc=$rc" >> $OUT/pytest_gpu.log
case $rc in 0|1) ;; *) exit 12;; esac
timeout -k 10 600 python tools/slab_serial.py --case d16m --ranks 8 --steps 4 --warmup 2 > $OUT/serial_d16m_8.json 2> $OUT/serial.err || exit 13
MPH_SLAB_OVERLAP=0 timeout -k 10 600 python tools/slab_serial.py --case d16m --ranks 8 --steps 4 --warmup 2 > $OUT/serial_d16m_8_nooverlap.json 2>> $OUT/serial.err || exit 14
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $OUT/bench_d1m.json 2> $OUT/bench.err || exit 15
MPH_FUSED=1 VARIANTS=base bash tools/pmc_ab.sh || exit 16
cp gpurun_out/pmc_base.txt $OUT/pmc_fused.txt
