#!/bin/bash
# Tile padding of the 640-row list tiles (MPH_TILE_PAD rows between tiles; the build: 1) at rest and
# t = 0.25 s, 2 rounds.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/${OUT:-ab_pad}
mkdir -p $O
OUT=$O VARIANTS="pad3 pad9 pad17 pad65" ROUNDS=2 bash tools/ab_dev.sh || exit 17
python3 tools/ab_dev_summary.py $O > $O/summary.txt 2>&1
