"""Per-XCD wave timing of the three list kernels (search, pass A, pass B) over one step.

Needs the diagnostic build (`make -C particlemethod_fsi_amd/csrc OUT=../lib_xcd
EXTRA=-DMPH_DIAG_XCD=1`, run with MPH_GPU_LIB=.../lib_xcd/libmph_gpu.so): each wave records its
start and end (wall_clock64, 100 MHz) per XCC_ID into the context's DevState (XcdProbe in
mph_kernels.hip).  Per kernel this prints each XCD's span (first wave start to last wave end,
relative to the kernel's first start), its summed wave time and its wave count: an XCD that
finishes late while the others idle is the imbalance a work-balanced block map would remove.

usage: MPH_GPU_LIB=... python tools/xcd_diag.py [--case d1m] [--warmup 4]
"""
from __future__ import annotations

import argparse
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

KERNELS = ("neighbors", "pass_a", "pass_b")
TICK_MS = 1e-5   # wall_clock64 runs at 100 MHz


def xcd_read(s, reset=True):
    """The diagnostic words of solver s as {kernel: {...}}, then restart them (reset)."""
    fn = s._L.mph_diag_xcd
    fn.restype = ctypes.c_int
    fn.argtypes = [ctypes.c_void_p, ctypes.POINTER(ctypes.c_ulonglong), ctypes.c_int]
    buf = (ctypes.c_ulonglong * 96)()
    rc = fn(s._h, buf, 1 if reset else 0)
    if rc != 0:
        raise RuntimeError("mph_diag_xcd: %d" % rc)
    out = {}
    for k, name in enumerate(KERNELS):
        w = [buf[k * 32 + j] for j in range(32)]
        t0s, t1s, busy, waves = w[0:8], w[8:16], w[16:24], w[24:32]
        live = [x for x in range(8) if waves[x]]
        if not live:
            continue
        base = min(t0s[x] for x in live)
        end = max(t1s[x] for x in live)
        out[name] = {
            "span_ms": round((end - base) * TICK_MS, 5),
            "xcd_end_ms": [round((t1s[x] - base) * TICK_MS, 5) if waves[x] else None for x in range(8)],
            "xcd_wave_ms_sum": [round(busy[x] * TICK_MS, 4) for x in range(8)],
            "xcd_waves": waves,
        }
        ends = [t1s[x] - base for x in live]
        out[name]["end_spread"] = round((max(ends) - min(ends)) / max(ends), 4)
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--case", default="d1m")
    ap.add_argument("--warmup", type=int, default=4)
    ap.add_argument("--repeat", type=int, default=3)
    args = ap.parse_args()
    from particlemethod_fsi_amd import MphSolver, cases
    case = cases.get(args.case)
    cfg, parts = case.build()
    s = MphSolver(cfg, parts, device=0)
    s.step(args.warmup)
    xcd_read(s, reset=True)
    runs = []
    for _ in range(args.repeat):
        s.step(1)
        runs.append(xcd_read(s, reset=True))
    print(json.dumps({"case": args.case, "runs": runs}))
    s.close()


if __name__ == "__main__":
    main()
