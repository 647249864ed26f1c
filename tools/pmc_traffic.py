"""Turn the rocprofv3 FETCH_SIZE / WRITE_SIZE passes of tools/profile.sh into per-kernel HBM bytes
per launch (profiles/pmc_traffic.json, read by bench.py for roofline.traffic).

Correction (MI355X_MICROARCH.md, HBM section): on gfx950 FETCH_SIZE (KiB) reports half the bytes
of wide coalesced streaming reads, so reads are counted as 2 x FETCH_SIZE; WRITE_SIZE (KiB) is
taken as is.  Both are averaged over the launches of each kernel.

usage: python tools/pmc_traffic.py gpurun_out/prof profiles/pmc_traffic.json [tag]
"""
import collections
import csv
import glob
import json
import os
import sys


def per_kernel(path_glob):
    acc = collections.defaultdict(list)
    for path in glob.glob(path_glob):
        for r in csv.DictReader(open(path)):
            name = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("mph::", "")
            name = name.split("<")[0]
            acc[name].append(float(r["Counter_Value"]))
    return {k: sum(v) / len(v) for k, v in acc.items()}


def main():
    src = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/prof"
    dst = sys.argv[2] if len(sys.argv) > 2 else "profiles/pmc_traffic.json"
    tag = sys.argv[3] if len(sys.argv) > 3 else ""
    fetch = per_kernel(src + "/fetch/*counter_collection.csv")
    write = per_kernel(src + "/write/*counter_collection.csv")
    names = {"k_neighbors": "neighbors", "k_pass_a": "pass_a", "k_pass_b": "pass_b", "k_prep": "prep",
             "k_rank_scatter": "rank_scatter", "k_scan_down": "scan_down", "k_scan_reduce": "scan_reduce",
             "k_place": "place"}
    out = {"_note": "HBM bytes per launch = (2*FETCH_SIZE + WRITE_SIZE) * 1024 (gfx950 FETCH_SIZE "
                    "correction, MI355X_MICROARCH.md); averaged over launches; " + tag,
           "case": os.environ.get("MPH_PMC_CASE", "d1m")}
    for k, short in names.items():
        if k in fetch or k in write:
            f, w = fetch.get(k, 0.0), write.get(k, 0.0)
            out[short] = {"fetch_kib": f, "write_kib": w, "hbm_bytes_per_launch": (2 * f + w) * 1024}
    with open(dst, "w") as fh:
        json.dump(out, fh, indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
