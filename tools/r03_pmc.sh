#!/bin/bash
# GPU session: selected GPU tests (K), then the diagnostic PMC groups (tools/pmc_ab.sh) of the
# VARIANTS, summaries copied to gpurun_out/$OUT.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${OUT:-r03pmc}
mkdir -p $OUT
if [ "${K:-none}" != none ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread ${K:+-k "$K"} \
      > $OUT/pytest_gpu.log 2>&1
  rc=$?
  echo "pytest rc=$rc" >> $OUT/pytest_gpu.log
  case $rc in 0|1|5) ;; *) exit 12;; esac
fi
VARIANTS="${VARIANTS:-base}" bash tools/pmc_ab.sh || exit 14
for v in ${VARIANTS:-base}; do cp gpurun_out/pmc_$v.txt $OUT/; done
