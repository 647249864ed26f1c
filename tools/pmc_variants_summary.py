"""Per-kernel FETCH_SIZE (x2, gfx950 read correction) and WRITE_SIZE MB per launch of the
builds measured by tools/pmc_variants.sh.  usage: python tools/pmc_variants_summary.py base ell"""
import collections
import csv
import glob
import sys


def per_kernel(d):
    acc = collections.defaultdict(list)
    for p in glob.glob(d + "/g1/*counter_collection.csv"):
        for r in csv.DictReader(open(p)):
            k = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("mph::", "").split("<")[0]
            acc[k].append(float(r["Counter_Value"]))
    return {k: sum(v[1:]) / max(len(v) - 1, 1) * 1024 / 1e6 for k, v in acc.items()}   # drop the init launch


for v in sys.argv[1:]:
    f = per_kernel("gpurun_out/pmc_%s_FETCH_SIZE" % v)
    w = per_kernel("gpurun_out/pmc_%s_WRITE_SIZE" % v)
    print(v)
    for k in ("k_neighbors", "k_pass_a", "k_pass_b"):
        print("  %-12s read %8.1f MB  write %8.1f MB" % (k, 2 * f.get(k, 0), w.get(k, 0)))
