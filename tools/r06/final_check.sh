#!/bin/bash
# The round's last tree: the whole GPU suite and smoke (as the driver runs them), then the default
# bench line.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/${OUT:-final_check}
mkdir -p $O
OUT=${O#gpurun_out/} bash tools/r06/full_suite.sh || exit 11
timeout -k 10 600 python3 bench.py > $O/bench.json 2> $O/bench.err || exit 12
