#!/bin/bash
# Pass A taking each XCD's range from its far end (the list tiles the search wrote last first,
# while the Infinity Cache holds them) against the forward order (norev): bitwise, parity, then
# D1M rest / t = 0.25 s (2 rounds), t = 1.0 s and D16M (1 round).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/${OUT:-ab_rev}
mkdir -p $O
L=$PWD/particlemethod_fsi_amd
CASES="box3d box3d_jit gate3d_jit d1m"
MPH_GPU_LIB=$L/lib_norev/libmph_gpu.so timeout -k 10 240 python3 tools/lib_bitwise.py run $O/base.npz $CASES > $O/bw_base.log 2>&1 || exit 11
MPH_GPU_LIB=$L/lib/libmph_gpu.so timeout -k 10 240 python3 tools/lib_bitwise.py run $O/new.npz $CASES > $O/bw_new.log 2>&1 || exit 12
python3 tools/lib_bitwise.py compare $O/base.npz $O/new.npz > $O/bitwise.txt 2>&1
rm -f $O/base.npz $O/new.npz
OUT=$O/t025 VARIANTS="norev" ROUNDS=2 bash tools/ab_dev.sh || exit 17
python3 tools/ab_dev_summary.py $O/t025 > $O/summary_t025.txt 2>&1
OUT=$O/t100 DEV_STEPS=10000 D16M=1 VARIANTS="norev" ROUNDS=1 bash tools/ab_dev.sh || exit 18
python3 tools/ab_dev_summary.py $O/t100 > $O/summary_t100.txt 2>&1
