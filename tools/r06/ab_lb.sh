#!/bin/bash
# The list kernels' block size (MPH_LB, 256 in the build: the search, pass A and pass B) at 128 and
# 512 threads; bitwise against the build on the small cases, then D1M rest / t = 0.25 s, 2 rounds.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/${OUT:-ab_lb}
mkdir -p $O
V="lb128 lb512"
L=particlemethod_fsi_amd
MPH_GPU_LIB=$PWD/$L/lib/libmph_gpu.so timeout -k 10 300 python3 tools/lib_bitwise.py run $O/bw_base.npz > $O/bw.log 2>&1 || exit 11
for v in $V; do
  MPH_GPU_LIB=$PWD/$L/lib_$v/libmph_gpu.so timeout -k 10 300 python3 tools/lib_bitwise.py run $O/bw_$v.npz >> $O/bw.log 2>&1 || exit 12
  python3 tools/lib_bitwise.py compare $O/bw_base.npz $O/bw_$v.npz > $O/bw_cmp_$v.txt 2>&1; echo "$v $?" >> $O/bw.log
done
rm -f $O/bw_*.npz
OUT=$O VARIANTS="$V" ROUNDS=2 bash tools/ab_dev.sh || exit 17
python3 tools/ab_dev_summary.py $O > $O/summary.txt 2>&1
