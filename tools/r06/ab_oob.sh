#!/bin/bash
# List passes gathering through sized buffer descriptors, rows without an entry masked by an
# out-of-range offset (no cache lookup): bitwise and parity against the committed aligned rows
# (rows1), then same-box A/B with rows1 and the build before aligned rows (r6base).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/${OUT:-ab_oob}
mkdir -p $O
L=$PWD/particlemethod_fsi_amd
CASES="box3d box3d_jit gate3d_jit seam3d dam2d box3d_st gate2d_sub d1m"
MPH_GPU_LIB=$L/lib_rows1/libmph_gpu.so timeout -k 10 240 python3 tools/lib_bitwise.py run $O/base.npz $CASES > $O/bw_base.log 2>&1 || exit 11
MPH_GPU_LIB=$L/lib/libmph_gpu.so timeout -k 10 240 python3 tools/lib_bitwise.py run $O/new.npz $CASES > $O/bw_new.log 2>&1 || exit 12
python3 tools/lib_bitwise.py compare $O/base.npz $O/new.npz > $O/bitwise.txt 2>&1
rm -f $O/base.npz $O/new.npz
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_edge.py tests/test_gpu_developed.py > $O/pytest.log 2>&1 || exit 16
OUT=$O/t025 VARIANTS="rows1 r6base" ROUNDS=2 bash tools/ab_dev.sh || exit 17
python3 tools/ab_dev_summary.py $O/t025 > $O/summary_t025.txt 2>&1
OUT=$O/t100 DEV_STEPS=10000 VARIANTS="rows1" ROUNDS=1 bash tools/ab_dev.sh || exit 18
python3 tools/ab_dev_summary.py $O/t100 > $O/summary_t100.txt 2>&1
