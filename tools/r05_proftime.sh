#!/bin/bash
# round 5: the list kernels timed as graph replays (mph_profile_graphs) against the rocprofv3
# kernel trace of the same command; D16M / 8 slab ranks one at a time
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r05proftime
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_parity.py -k "profile_graphs" > $OUT/pytest.log 2>&1 || exit 10
timeout -k 10 300 python3 bench.py --steps 24 --warmup 8 --no-cpu-baseline --developed-steps 0 > $OUT/bench.json 2> $OUT/bench.err || exit 11
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kt -o kt -- \
    python3 bench.py --steps 24 --warmup 8 --no-cpu-baseline --developed-steps 0 > $OUT/bench_under_kt.log 2>&1 || exit 12
MPH_SLAB_OVERLAP=0 timeout -k 10 600 python tools/slab_serial.py --case d16m --ranks 8 --steps 4 --warmup 2 > $OUT/serial_d16m_8_overlap0.json 2> $OUT/serial0.err || exit 13
