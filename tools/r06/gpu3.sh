#!/bin/bash
# round 6: the 512-neighbour fix (edge test, parity suite, bitwise against e6081fe), the bench line
# with run_average, and the fsi3d_sub bench line
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/r06c
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
    tests/test_gpu_edge.py tests/test_gpu_parity.py > $OUT/pytest.log 2>&1 || exit 11
MPH_GPU_LIB=particlemethod_fsi_amd/lib/ref_e6081fe/libmph_gpu.so timeout -k 10 300 python tools/lib_bitwise.py run $OUT/bw_ref.npz > $OUT/bw.log 2>&1 || exit 12
timeout -k 10 300 python tools/lib_bitwise.py run $OUT/bw_new.npz >> $OUT/bw.log 2>&1 || exit 13
python tools/lib_bitwise.py compare $OUT/bw_ref.npz $OUT/bw_new.npz >> $OUT/bw.log 2>&1
rm -f $OUT/bw_*.npz
timeout -k 10 500 python bench.py > $OUT/bench_d1m.json 2> $OUT/bench_d1m.err || exit 14
timeout -k 10 400 python bench.py --case fsi3d_sub --steps 20 --warmup 4 > $OUT/bench_fsi3d_sub.json 2> $OUT/bench_fsi3d_sub.err || exit 15
