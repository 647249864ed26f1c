#!/usr/bin/env python3
"""Summary of tools/ab_dev.sh: per variant and workload the mean ms/step over rounds and the list
kernels' HIP-event times.   python tools/ab_dev_summary.py gpurun_out/abdev"""
import collections
import glob
import json
import os
import sys

d = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/abdev"
acc = collections.defaultdict(list)
for f in sorted(glob.glob(os.path.join(d, "*_*_*.json"))):
    w, v, r = os.path.basename(f)[:-5].rsplit("_", 2)[0].split("_", 1)[0], None, None
    parts = os.path.basename(f)[:-5].split("_")
    w, r, v = parts[0], parts[-1], "_".join(parts[1:-1])
    try:
        j = json.load(open(f))
    except ValueError:
        continue
    acc[(w, v)].append(j)
for (w, v), js in sorted(acc.items()):
    ms = sum(j["ms_per_step"] for j in js) / len(js)
    k = {x: round(sum(j["kernels_ms"].get(x, 0) for j in js) / len(js), 4)
         for x in ("neighbors", "pass_a", "pass_b", "rank_scatter", "prep")}
    print("%-5s %-14s %8.4f ms  %s" % (w, v, ms, k))
