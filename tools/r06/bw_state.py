#!/usr/bin/env python3
"""Bitwise A/B from a saved state (tools/dev_state.py): the library of MPH_GPU_LIB steps the D1M
developed state `steps` steps and saves every per-particle field (compare with
tools/lib_bitwise.py compare), plus the list's row statistics.

  MPH_GPU_LIB=... python tools/r06/bw_state.py STATE.gridb OUT.npz [steps]
"""
import os
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))

import numpy as np  # noqa: E402

from lib_bitwise import FIELDS  # noqa: E402


def main():
    state, out = sys.argv[1], sys.argv[2]
    steps = int(sys.argv[3]) if len(sys.argv) > 3 else 10
    from particlemethod_fsi_amd import MphSolver, cases
    from particlemethod_fsi_amd.solver import read_case_files
    case = cases.get("d1m")
    cfg, parts = case.build()
    d = tempfile.mkdtemp(prefix="mphbw_")
    with open(os.path.join(d, "c.data"), "w") as fh:
        fh.write(cases.data_text(case.data()))
    scfg, sparts = read_case_files(os.path.join(d, "c.data"), state, case.dim, case.module)
    cfg.time = scfg.time
    res = {}
    with MphSolver(cfg, sparts) as s:
        s.step(steps)
        for f in FIELDS:
            if f in ("DeformGradient", "Strain", "Stress"):
                continue
            res["dev/%s" % f] = s.get(f)
        mean, mx = s.list_stats()
        nmean, nmx = s.neighbor_stats()
        print("list entries mean %.4f max %d; NeighborCount mean %.4f max %d" % (mean, mx, nmean, nmx))
    np.savez(out, **res)


if __name__ == "__main__":
    main()
