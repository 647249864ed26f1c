#!/usr/bin/env python3
"""Bitwise A/B of two builds (e.g. the round-6 cleanup against e6081fe): run each case for a
few steps with the library of MPH_GPU_LIB and save every per-particle field, or compare two saved
runs.

  MPH_GPU_LIB=.../libmph_gpu.so python tools/lib_bitwise.py run OUT.npz [cases...]
  python tools/lib_bitwise.py compare A.npz B.npz        (exit 1 on any difference)
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402

FIELDS = ["Position", "Velocity", "PressureP", "PressureA", "NeighborCount", "Force", "Acceleration",
          "DensityA", "VolStrainP", "DivergenceP", "GravityCenter", "DeformGradient", "Strain", "Stress"]


def run(out, names):
    from particlemethod_fsi_amd import MphSolver, cases
    res = {}
    for name in names:
        cfg, parts = cases.get(name).build()
        with MphSolver(cfg, parts) as s:
            s.step(3)
            s.step(8)
            for f in FIELDS:
                res["%s/%s" % (name, f)] = s.get(f)
    np.savez(out, **res)


def compare(a, b):
    A, B = np.load(a), np.load(b)
    bad = 0
    for k in sorted(A.files):
        same = np.array_equal(A[k], B[k])
        if not same:
            bad += 1
            print("DIFF", k, float(np.max(np.abs(A[k].astype(float) - B[k].astype(float)))))
    print("compared %d arrays: %s" % (len(A.files), "bit-identical" if not bad else "%d differ" % bad))
    return 1 if bad else 0


if __name__ == "__main__":
    if sys.argv[1] == "run":
        run(sys.argv[2], sys.argv[3:] or ["box3d", "box3d_st", "gate3d", "seam3d", "d1m"])
    else:
        sys.exit(compare(sys.argv[2], sys.argv[3]))
