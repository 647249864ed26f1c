"""Summarise rocprofv3 --pmc CSVs (gpurun_out/pmc/g*/...) per kernel: mean counter value."""
import collections
import csv
import glob
import sys

root = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/pmc"
vals = collections.defaultdict(lambda: collections.defaultdict(list))
for path in sorted(glob.glob(root + "/g*/*counter_collection.csv")):
    for r in csv.DictReader(open(path)):
        k = r["Kernel_Name"].split("(")[0].replace("void ", "")
        vals[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, d in vals.items():
    if not k.startswith("mph::"):
        continue
    print(k)
    for c, v in sorted(d.items()):
        print("   %-32s %14.4g" % (c, sum(v) / len(v)))
