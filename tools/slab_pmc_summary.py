"""Per-dispatch pass-B counters of the round-3 slab PMC runs (tag r05-variants, tools/r03_slabpmc.sh): with the overlap every step of a rank
launches pass B twice (interior waves, face waves) -- told apart by their VALU counts (the
interior launch does most of the work); without it once.  Prints the mean per launch kind."""
import collections
import csv
import glob
import sys

root = sys.argv[1]
for mode in ("ov1", "ov0"):
    disp = collections.defaultdict(dict)
    for path in glob.glob("%s/%s/**/*counter_collection.csv" % (root, mode), recursive=True):
        for r in csv.DictReader(open(path)):
            key = (r["Process_Id"], r.get("Thread_Id", ""), r["Dispatch_Id"])
            d = disp[key]
            d[r["Counter_Name"]] = d.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
            d["dur_us"] = (float(r["End_Timestamp"]) - float(r["Start_Timestamp"])) / 1e3
            d["grid"] = int(r["Grid_Size"])
            d["vgpr"] = r.get("VGPR_Count", r.get("Arch_VGPR_Count", ""))
    rows = [d for d in disp.values() if d.get("SQ_INSTS_VALU", 0) > 0]
    if not rows:
        print(mode, "no dispatches")
        continue
    rows.sort(key=lambda d: d["SQ_INSTS_VALU"])
    groups = {"all": rows}
    if mode == "ov1":
        med = rows[len(rows) // 2]["SQ_INSTS_VALU"]
        lo = [d for d in rows if d["SQ_INSTS_VALU"] < 0.6 * med]
        hi = [d for d in rows if d["SQ_INSTS_VALU"] >= 0.6 * med]
        groups = {"face (smaller VALU)": lo, "interior": hi}
    for name, g in groups.items():
        if not g:
            continue
        keys = sorted(k for k in g[0] if k not in ("vgpr",))
        mean = {k: sum(d.get(k, 0.0) for d in g) / len(g) for k in keys}
        print("%s %s: %d dispatches, vgpr %s" % (mode, name, len(g), g[0]["vgpr"]))
        for k in keys:
            print("   %-20s %14.5g" % (k, mean[k]))
        if mean.get("SQ_WAVES"):
            print("   %-20s %14.5g" % ("wave_cycles/wave", mean["SQ_WAVE_CYCLES"] / mean["SQ_WAVES"]))
            print("   %-20s %14.5g" % ("valu/wave", mean["SQ_INSTS_VALU"] / mean["SQ_WAVES"]))
