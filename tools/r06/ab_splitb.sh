#!/bin/bash
# Pass B's own XCD split on the steps without Force output (waves of walls count their fixed cost
# only) against the build before (prev): bitwise, parity/edge, then D1M rest / t = 0.25 s (3 rounds)
# and D16M, fsi3d_sub (1 round).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/${OUT:-ab_splitb}
mkdir -p $O
L=$PWD/particlemethod_fsi_amd
CASES="box3d box3d_jit gate3d_jit d1m"
MPH_GPU_LIB=$L/lib_prev/libmph_gpu.so timeout -k 10 240 python3 tools/lib_bitwise.py run $O/base.npz $CASES > $O/bw_base.log 2>&1 || exit 11
MPH_GPU_LIB=$L/lib/libmph_gpu.so timeout -k 10 240 python3 tools/lib_bitwise.py run $O/new.npz $CASES > $O/bw_new.log 2>&1 || exit 12
python3 tools/lib_bitwise.py compare $O/base.npz $O/new.npz > $O/bitwise.txt 2>&1
rm -f $O/base.npz $O/new.npz
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_edge.py > $O/pytest.log 2>&1 || exit 16
OUT=$O/ab VARIANTS="prev" ROUNDS=3 bash tools/ab_dev.sh || exit 17
python3 tools/ab_dev_summary.py $O/ab > $O/summary.txt 2>&1
OUT=$O/d16 D16M=1 VARIANTS="prev" ROUNDS=1 bash tools/ab_dev.sh || exit 18
python3 tools/ab_dev_summary.py $O/d16 > $O/summary_d16m.txt 2>&1
