"""Which path the search takes per wave and stencil column, along the developed D1M flow.

Needs the diagnostic build (`make -C particlemethod_fsi_amd/csrc OUT=../lib_paths
EXTRA=-DMPH_DIAG_PATHS=1`, run with MPH_GPU_LIB=.../lib_paths/libmph_gpu.so): every wave-column
of the search counts its path (one FP32 window, two FP32 runs, FP64 staged, per-lane global
loads), its lanes' candidates and its window's records (scan_candidates_lds).  At each checkpoint
the counters of one step are printed as one JSON line.

usage: MPH_GPU_LIB=... python tools/search_paths.py [--case d1m] [--at 1,2500,10000]
"""
from __future__ import annotations

import argparse
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

PATHS = ("f32_one", "f32_two", "f64_staged", "global")


def read(s, reset=True):
    fn = s._L.mph_diag_paths
    fn.restype = ctypes.c_int
    fn.argtypes = [ctypes.c_void_p, ctypes.POINTER(ctypes.c_ulonglong), ctypes.c_int]
    buf = (ctypes.c_ulonglong * 48)()
    rc = fn(s._h, buf, 1 if reset else 0)
    if rc != 0:
        raise RuntimeError("mph_diag_paths: %d" % rc)
    return [int(x) for x in buf]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--case", default="d1m")
    ap.add_argument("--at", default="1,2500,10000")
    ap.add_argument("--state", default=None, help="start from a tools/dev_state.py grid (--at counts on)")
    a = ap.parse_args()
    from particlemethod_fsi_amd import MphSolver, cases
    case = cases.get(a.case)
    cfg, parts = case.build()
    if a.state:
        import tempfile
        from particlemethod_fsi_amd.solver import read_case_files
        d = tempfile.mkdtemp(prefix="mphstate_")
        with open(os.path.join(d, "c.data"), "w") as fh:
            fh.write(cases.data_text(case.data()))
        scfg, parts = read_case_files(os.path.join(d, "c.data"), a.state, case.dim, case.module)
        cfg.time = scfg.time
    with MphSolver(cfg, parts) as s:
        done = 0
        for at in [int(x) for x in a.at.split(",")]:
            if at - 1 > done:
                s.step(at - 1 - done)
            read(s)
            s.step(1)
            w = read(s)
            done = at
            cols = sum(w[0:4])
            out = {"case": a.case, "step": at, "time_s": s.time, "waves": w[15], "columns": cols,
                   "split": {"no_gap": w[12], "too_wide": w[13], "two": w[14]}}
            for k, name in enumerate(PATHS):
                out[name] = {"columns": w[k], "col_frac": w[k] / max(cols, 1), "candidates": w[4 + k],
                             "records": w[8 + k],
                             "cand_per_col": w[4 + k] / max(w[k], 1), "rec_per_col": w[8 + k] / max(w[k], 1)}
            tot = max(w[32], 1)
            out["stored"] = w[32]
            out["ring"] = {"rule%d_R%d" % (r, 4 << ri): {"ahead": w[16 + (r * 4 + ri) * 2] / tot,
                                                          "behind": w[17 + (r * 4 + ri) * 2] / tot}
                           for r in range(2) for ri in range(4)}
            out["ring_rows_flushed_r1_R16"] = w[33]
            out["rows"] = {"aligned_per_column": w[40], "aligned_per_group": w[41], "today": w[42],
                           "lane_fill_today": w[32] / max(64 * w[42], 1),
                           "lane_fill_per_column": w[32] / max(64 * w[40], 1),
                           "lane_fill_per_group": w[32] / max(64 * w[41], 1)}
            out["store_segments"] = {"instructions": w[46], "entries": w[47],
                                     "segments_lanes_in_order": w[44], "segments_lanes_by_prev_count": w[45],
                                     "entries_per_segment_in_order": w[47] / max(w[44], 1),
                                     "entries_per_segment_sorted": w[47] / max(w[45], 1)}
            out["span_hist"] = dict(zip(("64-96", "96-128", "128-160", "160-192", "192-256", ">256"),
                                        [x / max(cols, 1) for x in w[34:40]]))
            print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
