"""Calibration of FETCH_SIZE / WRITE_SIZE (rocprofv3, gfx950) on kernels of known bytes
(tools/pmc_calib.hip), for the access patterns of the MPH hot path.

usage: python tools/pmc_calib.py gpurun_out/calib profiles/pmc_calib.json
  expects <dir>/known.json (the program's stdout), <dir>/fetch/*counter_collection.csv and
  <dir>/write/*counter_collection.csv (one rocprofv3 --pmc pass each).
The result gives, per pattern, counter bytes / requested bytes and counter bytes / 64-B lines:
tools/pmc_traffic.py uses the factor of the matching pattern to turn counters into bytes.
"""
import collections
import csv
import glob
import json
import sys


def per_kernel(path_glob):
    acc = collections.defaultdict(list)
    for path in glob.glob(path_glob):
        for r in csv.DictReader(open(path)):
            name = r["Kernel_Name"].split("(")[0].replace("void ", "").split("<")[0]
            acc[name.replace("k_", "", 1)].append(float(r["Counter_Value"]))
    return {k: sum(v) / len(v) for k, v in acc.items()}


def main():
    src = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/calib"
    dst = sys.argv[2] if len(sys.argv) > 2 else "profiles/pmc_calib.json"
    known = json.load(open(src + "/known.json"))
    fetch = per_kernel(src + "/fetch/*counter_collection.csv")
    write = per_kernel(src + "/write/*counter_collection.csv")
    out = {"_note": "counter KiB x 1024 against the bytes each kernel requests (tools/pmc_calib.hip); "
                    "arrays of 4 GiB, beyond the 256 MiB Infinity Cache; averaged over 2 launches"}
    for k, v in known.items():
        cnt = write.get(k, 0.0) if "write" in k or "scatter" in k else fetch.get(k, 0.0)
        b = cnt * 1024.0
        lines = v.get("lines64", v.get("lines64_min"))
        out[k] = {"counter": "WRITE_SIZE" if ("write" in k or "scatter" in k) else "FETCH_SIZE",
                  "counter_bytes": b, "requested_bytes": v["bytes"],
                  "counter_over_requested": b / v["bytes"] if v["bytes"] else None,
                  "counter_over_lines64": b / (64.0 * lines) if lines else None,
                  "fetch_bytes": fetch.get(k, 0.0) * 1024.0, "write_bytes": write.get(k, 0.0) * 1024.0}
    with open(dst, "w") as fh:
        json.dump(out, fh, indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
