#!/bin/bash
# Search inner loop (list entry in the FP32 record, one induction variable): bitwise against the
# base build, then a same-box A/B of base / round-5 final (e608, ABI 3) / the new search (srch).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/ab_srch
mkdir -p $O
L=$PWD/particlemethod_fsi_amd
MPH_GPU_LIB=$L/lib/libmph_gpu.so timeout -k 10 240 python3 tools/lib_bitwise.py run $O/base.npz > $O/bw_base.log 2>&1 || exit 11
MPH_GPU_LIB=$L/lib_srch/libmph_gpu.so timeout -k 10 240 python3 tools/lib_bitwise.py run $O/srch.npz > $O/bw_srch.log 2>&1 || exit 12
python3 tools/lib_bitwise.py compare $O/base.npz $O/srch.npz > $O/bitwise.txt 2>&1 || exit 13
rm -f $O/base.npz $O/srch.npz
export MPH_ABI_ACCEPT=3
OUT=$O VARIANTS="${VARIANTS:-e608 srch}" ROUNDS=${ROUNDS:-3} bash tools/ab_dev.sh || exit 14
python3 tools/ab_dev_summary.py $O > $O/summary.txt 2>&1
