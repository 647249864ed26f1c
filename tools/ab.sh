#!/bin/bash
# A/B timing of alternative builds (particlemethod_fsi_amd/lib_<name>/libmph_gpu.so, made with
# `make -C particlemethod_fsi_amd/csrc OUT=../lib_<name> EXTRA=-D...`) or run-time settings (a
# variant VAR=VALUE runs the base library with that environment variable) on the bench of CASE
# (default d1m); one log per variant: gpurun_out/ab_<case>_<name>.log (tools/ab_summary.py).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for case in ${CASES:-${CASE:-d1m}}; do
  for name in base ${VARIANTS}; do
    lib=$PWD/particlemethod_fsi_amd/lib/libmph_gpu.so
    envset=()
    if [[ "$name" == *@* ]]; then   # <build>@VAR=VALUE: an alternative build with a run-time setting
      lib=$PWD/particlemethod_fsi_amd/lib_${name%%@*}/libmph_gpu.so; envset=("${name#*@}")
    elif [[ "$name" == *=* ]]; then IFS=, read -ra envset <<< "$name"   # VAR=VALUE[,VAR2=VALUE2]
    elif [ "$name" != base ]; then lib=$PWD/particlemethod_fsi_amd/lib_$name/libmph_gpu.so; fi
    env "${envset[@]}" MPH_GPU_LIB=$lib timeout -k 10 300 python bench.py --case $case --steps ${STEPS:-20} \
        --warmup 4 --no-cpu-baseline > "gpurun_out/ab_${case}_${name}.log" 2>&1 || exit 40
  done
done
