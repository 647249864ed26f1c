#!/bin/bash
# round 5, first GPU call: the new parity tests (off-lattice goldens, neighbour sets, developed
# D1M against the oracle) and the bench line with its `developed` object
set -o pipefail
OUT=gpurun_out/r05a
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest -x -v --timeout 600 --timeout-method thread \
    tests/test_gpu_developed.py tests/test_gpu_parity.py -k "jit or neighbor_sets or developed" \
    > $OUT/pytest.log 2>&1 &&
timeout -k 10 300 python bench.py --warmup 5 --steps 20 > $OUT/bench.json 2> $OUT/bench.err
