"""Diagnostic: per-field max |diff| of a case on one GPU context against the CPU oracle at a few
step counts (how far reassociation roundoff grows in that case), to size slab-test tolerances.

usage: python tools/slab_diag.py CASE [steps...]
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

from particlemethod_fsi_amd import MphSolver, cases  # noqa: E402
from oracle_bindings import OracleSolver  # noqa: E402

FIELDS = ["Position", "Velocity", "PressureP", "Force", "VolStrainP", "DivergenceP", "DensityA",
          "DeformGradient", "Strain", "Stress"]


def main():
    case = sys.argv[1]
    steps = [int(a) for a in sys.argv[2:]] or [1, 10, 30]
    cfg, parts = cases.get(case).build()
    o = OracleSolver(cfg, parts)
    o.init()
    with MphSolver(cfg, parts) as s:
        done = 0
        for k in steps:
            s.step(k - done)
            o.step(k - done)
            done = k
            row = []
            for f in FIELDS:
                a, b = s.get(f), o.get(f)
                sc = float(np.max(np.abs(b))) or 1.0
                row.append("%s %.1e" % (f, float(np.max(np.abs(a - b))) / sc))
            print("step %d rel: %s" % (k, ", ".join(row)), flush=True)


if __name__ == "__main__":
    main()
