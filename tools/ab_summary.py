#!/usr/bin/env python3
"""One line per A/B log (gpurun_out/ab_<case>_<name>.log, tools/ab.sh): rate, ms/step, mean
neighbour count and the per-kernel HIP-event averages.  Arguments: case names (default d1m)."""
import glob
import json
import os
import sys

root = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "gpurun_out")
for case in sys.argv[1:] or ["d1m"]:
    for p in sorted(glob.glob(os.path.join(root, "ab_%s_*.log" % case))):
        name = os.path.basename(p)[len("ab_%s_" % case):-4]
        try:
            d = json.loads(open(p).read().strip().splitlines()[-1])
        except (OSError, ValueError, IndexError):
            print(case, name, "missing")
            continue
        print(case, name, "%.4g" % d["value"], "%.4f ms" % d["ms_per_step"], "nb %.2f" % d["neighbors"]["mean"],
              {k: round(v, 4) for k, v in d["kernels_ms"].items()})
