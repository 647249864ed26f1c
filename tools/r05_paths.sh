#!/bin/bash
# round 5: the search's column paths and a simulated LDS row ring at rest, t = 0.25 s and t = 1.0 s
# (diagnostic build lib_paths; the developed states from the default build)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r05paths
mkdir -p $OUT
DL=$PWD/particlemethod_fsi_amd/lib_paths/libmph_gpu.so
MPH_GPU_LIB=$DL timeout -k 10 120 python -u tools/search_paths.py --at 1 > $OUT/paths.jsonl 2> $OUT/paths.err || exit 11
for st in 2500 10000; do
  timeout -k 10 120 python3 tools/dev_state.py d1m $st /tmp/d1m_$st.gridb >> $OUT/paths.err 2>&1 || exit 12
  MPH_GPU_LIB=$DL timeout -k 10 120 python -u tools/search_paths.py --state /tmp/d1m_$st.gridb --at 1 >> $OUT/paths.jsonl 2>> $OUT/paths.err || exit 13
  rm -f /tmp/d1m_$st.gridb
done
