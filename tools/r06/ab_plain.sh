#!/bin/bash
# Plain-row shortcut (waves without jumps skip the row mask) and no jumps in 2-D, against the
# committed masked-gather build (oob): D1M rest / t = 0.25 s, Bar 400k (2-D), FSI sub, 2 rounds.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/${OUT:-ab_plain}
mkdir -p $O
L=$PWD/particlemethod_fsi_amd
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_edge.py > $O/pytest.log 2>&1 || exit 16
OUT=$O/t025 VARIANTS="oob" ROUNDS=2 bash tools/ab_dev.sh || exit 17
python3 tools/ab_dev_summary.py $O/t025 > $O/summary_t025.txt 2>&1
for r in 1 2; do
  for v in base oob; do
    lib=$L/lib/libmph_gpu.so; [ $v != base ] && lib=$L/lib_$v/libmph_gpu.so
    for c in bar2d_400k fsi3d_sub; do
      MPH_GPU_LIB=$lib timeout -k 10 300 python3 bench.py --case $c --steps 20 --warmup 4 --no-cpu-baseline > $O/${c}_${v}_$r.json 2> $O/${c}_$v.err || exit 18
    done
  done
done
