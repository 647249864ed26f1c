#!/usr/bin/env python3
"""Diagnostic run of the staged pass A (a lib_pasd build: -DMPH_PA_STAGED=1 -DMPH_DIAG_PA=1):
creates each case and steps it once; the library reports an entry outside its column window or
entries left over as an error."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from particlemethod_fsi_amd import MphSolver, cases  # noqa: E402

for name in sys.argv[1:] or ["box3d", "d1m"]:
    cfg, parts = cases.get(name).build()
    try:
        with MphSolver(cfg, parts) as s:
            s.step(1)
            print(name, "ok", float(s.get("DensityA").max()))
    except Exception as e:  # the diagnostic status
        print(name, "ERROR", e)
