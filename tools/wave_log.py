#!/usr/bin/env python3
"""Per-wave timing of the search (diagnostic build `make -C particlemethod_fsi_amd/csrc
OUT=../lib_xcd EXTRA=-DMPH_DIAG_XCD=2`, run with MPH_GPU_LIB=.../lib_xcd/libmph_gpu.so): every
wave of k_neighbors records its start, end (wall_clock64, 100 MHz) and XCC_ID; this prints the
distribution of wave durations, the kernel span, and how much of the span runs below full
residency (the launch's tail), per XCD.

usage: MPH_GPU_LIB=... python tools/wave_log.py [--case d1m] > out.json
"""
import argparse
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402

TICK_US = 0.01   # 100 MHz


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--case", default="d1m")
    ap.add_argument("--warmup", type=int, default=8)
    args = ap.parse_args()
    from particlemethod_fsi_amd import MphSolver, cases
    cfg, parts = cases.get(args.case).build()
    with MphSolver(cfg, parts) as s:
        fn = s._L.mph_diag_waves
        fn.restype = ctypes.c_int
        fn.argtypes = [ctypes.c_void_p, ctypes.POINTER(ctypes.c_ulonglong), ctypes.c_int]
        nmax = (((parts.n + 255) // 256) * 5 // 4 + 16) * 4
        buf = (ctypes.c_ulonglong * (3 * nmax))()
        fn(s._h, buf, nmax)          # allocates the log
        s.step(args.warmup)
        s.step(1)                    # the logged launch (a 1-step graph)
        k = fn(s._h, buf, nmax)
    a = np.frombuffer(buf, dtype=np.uint64, count=3 * k).reshape(k, 3).astype(np.int64)
    a = a[a[:, 1] > 0]
    idle = int(((a[:, 1] - a[:, 0]) * TICK_US < 2.0).sum())   # waves of a slack grid that found no tile
    a = a[(a[:, 1] - a[:, 0]) * TICK_US >= 2.0]
    t0, t1, x = a[:, 0], a[:, 1], a[:, 2]
    base = t0.min()
    dur = (t1 - t0) * TICK_US
    span = (t1.max() - base) * TICK_US
    out = {"case": args.case, "waves": int(len(a)), "idle_waves": idle, "span_us": round(span, 2),
           "wave_us": {p: round(float(np.percentile(dur, q)), 2) for p, q in
                       (("p10", 10), ("p50", 50), ("p90", 90), ("p99", 99), ("max", 100))},
           "wave_us_mean": round(float(dur.mean()), 2)}
    # residency over time: waves alive per 1 us bin, and the span after the last wave started
    bins = np.arange(0, span + 1.0, 1.0)
    alive = np.zeros(len(bins))
    s0 = (t0 - base) * TICK_US
    s1 = (t1 - base) * TICK_US
    for lo, hi in zip(s0, s1):
        alive[int(lo):int(hi) + 1] += 1
    peak = float(np.percentile(alive[alive > 0], 90))
    out["alive_peak_p90"] = peak
    out["last_start_us"] = round(float(s0.max()), 2)
    out["tail_us"] = round(span - float(s0.max()), 2)
    out["time_below_half_peak_us"] = round(float((alive < 0.5 * peak).sum()), 1)
    per = {}
    for xc in range(8):
        m = x == xc
        if m.any():
            per[xc] = {"waves": int(m.sum()), "end_us": round(float(s1[m].max()), 2),
                       "last_start_us": round(float(s0[m].max()), 2),
                       "mean_wave_us": round(float(dur[m].mean()), 2)}
    out["per_xcd"] = per
    # the hardware's block -> XCD assignment: per logical XCD j = block & 7, the XCC_IDs its waves ran on
    slots = np.nonzero((np.frombuffer(buf, dtype=np.uint64, count=3 * k).reshape(k, 3)[:, 1] > 0))[0]
    raw = np.frombuffer(buf, dtype=np.uint64, count=3 * k).reshape(k, 3)[slots]
    logical = (slots // 4) % 8
    out["logical_to_xcc"] = {int(j): sorted({int(v) for v in raw[logical == j, 2]}) for j in range(8)}
    # the slowest waves: their slot (block * 4 + wave) and duration
    order = np.argsort(-dur)[:20]
    out["slowest"] = [[int(i), round(float(dur[i]), 2), round(float(s0[i]), 2)] for i in order]
    json.dump(out, sys.stdout, indent=1)
    print()


if __name__ == "__main__":
    main()
