#!/bin/bash
# Pass A timed in sequence after the search (mph_profile_graphs) against rocprofv3's kernel trace
# of the same bench command.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
O=gpurun_out/${OUT:-check_seq}
mkdir -p $O
timeout -k 10 300 python3 bench.py --steps 24 --warmup 8 --no-cpu-baseline --developed-steps 0 --run-average-end 0 > $O/bench.json 2> $O/bench.err || exit 11
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o kt -- \
    python3 bench.py --steps 24 --warmup 8 --no-cpu-baseline --developed-steps 0 --run-average-end 0 > $O/bench_under_kt.json 2>&1 || exit 12
