#!/bin/bash
# Aligned list rows (row jumps at stencil group ends): bitwise against the previous build (lib_r6base)
# on the lattice and jittered cases and from the developed D1M state (t = 0.25 s), the list parity
# tests, then a same-box A/B at rest and in the developed flow.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/${OUT:-ab_rows}
mkdir -p $O
L=$PWD/particlemethod_fsi_amd
CASES="box3d box3d_jit gate3d_jit seam3d dam2d gate2d d1m"
MPH_GPU_LIB=$L/lib_r6base/libmph_gpu.so timeout -k 10 240 python3 tools/lib_bitwise.py run $O/base.npz $CASES > $O/bw_base.log 2>&1 || exit 11
MPH_GPU_LIB=$L/lib/libmph_gpu.so timeout -k 10 240 python3 tools/lib_bitwise.py run $O/new.npz $CASES > $O/bw_new.log 2>&1 || exit 12
python3 tools/lib_bitwise.py compare $O/base.npz $O/new.npz > $O/bitwise.txt 2>&1
rm -f $O/base.npz $O/new.npz
MPH_GPU_LIB=$L/lib_r6base/libmph_gpu.so timeout -k 10 200 python3 tools/dev_state.py d1m ${DEV_STEPS:-2500} $O/d1m_dev.gridb > $O/dev_state.log 2>&1 || exit 13
MPH_GPU_LIB=$L/lib_r6base/libmph_gpu.so timeout -k 10 120 python3 tools/r06/bw_state.py $O/d1m_dev.gridb $O/dbase.npz > $O/bws_base.log 2>&1 || exit 14
MPH_GPU_LIB=$L/lib/libmph_gpu.so timeout -k 10 120 python3 tools/r06/bw_state.py $O/d1m_dev.gridb $O/dnew.npz > $O/bws_new.log 2>&1 || exit 15
python3 tools/lib_bitwise.py compare $O/dbase.npz $O/dnew.npz > $O/bitwise_dev.txt 2>&1
rm -f $O/dbase.npz $O/dnew.npz $O/d1m_dev.gridb
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_edge.py > $O/pytest.log 2>&1 || exit 16
OUT=$O VARIANTS="${VARIANTS:-r6base}" ROUNDS=${ROUNDS:-2} bash tools/ab_dev.sh || exit 17
python3 tools/ab_dev_summary.py $O > $O/summary.txt 2>&1
