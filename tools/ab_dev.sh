#!/bin/bash
# Same-box A/B of library builds (particlemethod_fsi_amd/lib_<name>; "base" = lib/) at rest (D1M),
# in the developed flow (D1M from t = 0.25 s, or DEV_STEPS steps; tools/dev_state.py) and, with D16M=1, on D16M;
# ROUNDS alternating rounds.  Output: $OUT/{rest,dev,d16m}_<name>_<round>.json (tools/ab_dev_summary.py)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=${OUT:-gpurun_out/abdev}
mkdir -p $OUT
trap 'rm -f $OUT/d1m_dev.gridb' EXIT   # the state is ~72 MB: never left for gpurun to copy back
timeout -k 10 120 python3 tools/dev_state.py d1m ${DEV_STEPS:-2500} $OUT/d1m_dev.gridb > $OUT/dev_state.log 2>&1 || exit 21
for r in $(seq 1 ${ROUNDS:-2}); do
  for v in base ${VARIANTS}; do
    lib=$PWD/particlemethod_fsi_amd/lib/libmph_gpu.so
    envset=()
    if [[ "$v" == *=* ]]; then envset=("$v")   # VAR=VALUE: a run-time setting on the base library
    elif [ $v != base ]; then lib=$PWD/particlemethod_fsi_amd/lib_$v/libmph_gpu.so; fi
    tag=${v//=/-}
    env "${envset[@]}" MPH_GPU_LIB=$lib timeout -k 10 300 python3 bench.py --developed-steps 0 --run-average-end 0 --steps 20 --warmup 4 --no-cpu-baseline > $OUT/rest_${tag}_$r.json 2> $OUT/rest_$tag.err || exit 22
    env "${envset[@]}" MPH_GPU_LIB=$lib timeout -k 10 300 python3 bench.py --state $OUT/d1m_dev.gridb --run-average-end 0 --steps 20 --warmup 4 --no-cpu-baseline > $OUT/dev_${tag}_$r.json 2> $OUT/dev_$tag.err || exit 23
    if [ "${D16M:-0}" = 1 ]; then
      env "${envset[@]}" MPH_GPU_LIB=$lib timeout -k 10 300 python3 bench.py --case d16m --run-average-end 0 --steps 12 --warmup 4 --no-cpu-baseline > $OUT/d16m_${tag}_$r.json 2> $OUT/d16m_$tag.err || exit 24
    fi
  done
done
rm -f $OUT/d1m_dev.gridb
