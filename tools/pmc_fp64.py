"""FP64 work per kernel launch from a rocprofv3 --pmc pass of SQ_INSTS_VALU_FLOPS_FP64
(tools/pmc.sh) -> profiles/pmc_fp64.json, read by bench.py for its "fp64" object.

SQ_INSTS_VALU_FLOPS_FP64 counts FLOPs per wavefront instruction: on D1M it equals
ADD_F64 + MUL_F64 + 2 FMA_F64 + TRANS_F64 instructions for every kernel (pass A 1.367e8 =
2.296e7 + 4.591e7 + 2 x 3.308e7 + 1.68e6), and pass A's VALU count / SQ_WAVES (~6500 per wave)
is the per-wavefront instruction count.  The lane FLOPs of a launch are therefore 64x the
counter -- an upper bound, since lanes masked off by divergence are counted too.

usage: python tools/pmc_fp64.py gpurun_out/pmc profiles/pmc_fp64.json [tag]
"""
import collections
import csv
import glob
import json
import os
import sys


def main():
    src = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/pmc"
    dst = sys.argv[2] if len(sys.argv) > 2 else "profiles/pmc_fp64.json"
    tag = sys.argv[3] if len(sys.argv) > 3 else ""
    acc = collections.defaultdict(lambda: collections.defaultdict(list))
    for path in glob.glob(src + "/g*/*counter_collection.csv"):
        for r in csv.DictReader(open(path)):
            name = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("mph::", "").split("<")[0]
            acc[name][r["Counter_Name"]].append((int(r["Dispatch_Id"]), float(r["Counter_Value"])))
    out = {"_note": "lane FP64 FLOPs per launch = 64 x SQ_INSTS_VALU_FLOPS_FP64, averaged over "
                    "launches (upper bound: masked lanes count); " + tag,
           "case": os.environ.get("MPH_PMC_CASE", "d1m")}
    for name, d in sorted(acc.items()):
        vals = [v for _, v in sorted(d.get("SQ_INSTS_VALU_FLOPS_FP64", []))]
        if len(vals) % 8 == 1 and len(vals) > 1:
            vals = vals[1:]   # mph_create's initialisation launch (runs step in batches of 8)
        if not sum(vals):
            continue
        f = sum(vals) / len(vals)
        out[name.replace("k_", "", 1)] = {"wave_flops": f, "lane_flops_per_launch": 64.0 * f}
    with open(dst, "w") as fh:
        json.dump(out, fh, indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
