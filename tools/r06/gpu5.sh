#!/bin/bash
# round 6: multi-GPU readiness -- the developed 8-slab test, the slab suite (probe on scratch
# buffers), and a 2-rank bench rehearsal (host transport, one GPU) for the per-rank output
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/r06e
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest -x -v -s --timeout 800 --timeout-method thread \
    tests/test_gpu_developed.py -k slab8 tests/test_gpu_dist.py > $OUT/pytest.log 2>&1 || exit 11
RANKS=2 STEPS=10 timeout -k 10 400 bash tools/gpu_dist_rehearsal.sh || exit 12
cp gpurun_out/rehearsal_d1m_n2.log $OUT/
