"""Turn the rocprofv3 FETCH_SIZE / WRITE_SIZE passes of tools/profile.sh into per-kernel HBM bytes
per launch (profiles/pmc_traffic.json, read by bench.py for roofline.traffic).

Correction (MI355X_MICROARCH.md, HBM section, and our own calibration profiles/pmc_calib.json,
tools/pmc_calib.hip): on gfx950 FETCH_SIZE (KiB) counts one 64-B unit per 128-B fabric request --
exactly half of a coalesced 16-B/lane stream, and one unit per random 8-B or 16-B gather, and
1.25 units per random 48-B record (the share of records that straddle a 128-B line) -- so reads
are 2 x FETCH_SIZE for every pattern of these kernels; WRITE_SIZE (KiB) is exact for coalesced
stores (and reads 1.09x the bytes of an ELL-row 4-B store pattern).  Per kernel the counters are
averaged over its launches; a first launch that belongs to mph_create's initialisation sums
(kernels with 8k + 1 launches: the profiled runs step in batches of 8) is dropped, so the
averages follow the timed region's store pattern (7 trimmed steps + 1 full step per 8).

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
            acc[name].append((int(r["Dispatch_Id"]), float(r["Counter_Value"])))
    out = {}
    for k, v in acc.items():
        v.sort()
        vals = [x for _, x in v]
        if len(vals) % 8 == 1 and len(vals) > 1:
            vals = vals[1:]   # mph_create's initialisation launch
        out[k] = sum(vals) / len(vals)
    return out


def main():
    src = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/prof"
    dst = sys.argv[2] if len(sys.argv) > 2 else "profiles/pmc_traffic.json"
    tag = sys.argv[3] if len(sys.argv) > 3 else ""
    fetch = per_kernel(src + "/fetch/*counter_collection.csv")
    write = per_kernel(src + "/write/*counter_collection.csv")
    names = {"k_neighbors": "neighbors", "k_neighbors_redo": "neighbors_redo", "k_pass_a": "pass_a", "k_pass_b": "pass_b", "k_prep": "prep",
             "k_rank_scatter": "rank_scatter", "k_scan_down": "scan_down", "k_scan_reduce": "scan_reduce",
             "k_scan_top": "scan_top", "k_place": "place"}
    out = {"_note": "HBM bytes per launch = (2*FETCH_SIZE + WRITE_SIZE) * 1024 (gfx950 FETCH_SIZE "
                    "correction, MI355X_MICROARCH.md); averaged over launches; " + tag,
           "case": os.environ.get("MPH_PMC_CASE", "d1m")}
    total = 0.0
    for k, short in names.items():
        if k in fetch or k in write:
            f, w = fetch.get(k, 0.0), write.get(k, 0.0)
            out[short] = {"fetch_kib": f, "write_kib": w, "hbm_bytes_per_launch": (2 * f + w) * 1024}
            total += (2 * f + w) * 1024   # every kernel runs once per step
    out["hbm_bytes_per_step"] = total
    with open(dst, "w") as fh:
        json.dump(out, fh, indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
