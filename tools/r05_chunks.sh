#!/bin/bash
# round 5: chunked search + pass A on two streams (MPH_CHUNKS): bitwise tests, a kernel trace that
# shows whether the pieces overlap, then same-box A/B at rest / developed / D16M
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r05chunks
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_parity.py -k "chunked" > $OUT/pytest.log 2>&1 || exit 11
MPH_CHUNKS=4 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kt4 -o kt -- \
    python3 bench.py --steps 16 --warmup 8 --no-cpu-baseline --developed-steps 0 > $OUT/bench_kt4.log 2>&1 || exit 12
OUT=$OUT VARIANTS="MPH_CHUNKS=2 MPH_CHUNKS=4" D16M=1 bash tools/ab_dev.sh || exit 13
