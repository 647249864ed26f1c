#!/usr/bin/env python3
"""Roundoff sensitivity of the reference's own algorithm (the bit-identical CPU oracle): the case
run twice, once as given and once with every position perturbed by one ulp, compared after each
checkpoint -- how far one ulp of input noise carries after k steps.  The GPU path reassociates its
sums (a few ulp per step), so its distance from the oracle is judged against this growth (the
elastic FSI gate amplifies it).

  python tools/ulp_study.py fsi3d 1 10 29 52 > tests/golden/ulp_fsi3d.json
  python tools/ulp_study.py bar2d_400k 1 10 50 100 > tests/golden/ulp_bar2d_400k.json
"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

import numpy as np  # noqa: E402

from oracle_bindings import OracleSolver  # noqa: E402
from particlemethod_fsi_amd import cases  # noqa: E402

FIELDS = ["Position", "Velocity", "PressureP", "VolStrainP", "DivergenceP", "Force"]
SOLID_FIELDS = ["DeformGradient", "Stress"]   # elastic tensors: compared on the structure particles


def main():
    name = sys.argv[1]
    checks = [int(x) for x in sys.argv[2:]] or [1, 10, 29, 52]
    OracleSolver.set_threads(os.cpu_count() or 1)
    cfg, parts = cases.get(name).build()
    solid = (parts.property >= 2) & (parts.property < 4)
    a = OracleSolver(cfg, parts)
    import dataclasses
    b_parts = dataclasses.replace(parts, position=np.nextafter(parts.position, np.inf))
    b = OracleSolver(cfg, b_parts)
    a.init()
    b.init()
    out = {"case": name, "perturbation": "every Position component moved by one ulp (nextafter)",
           "source": "oracle/mph_oracle.c, tools/ulp_study.py", "checkpoints": {}}
    done, t0 = 0, time.time()
    for k in checks:
        a.step(k - done)
        b.step(k - done)
        done = k
        res = {}
        for f in FIELDS + (SOLID_FIELDS if solid.any() else []):
            x, y = a.get(f), b.get(f)
            if f in SOLID_FIELDS:
                x, y = x[solid], y[solid]
                res[f] = {"max_abs": float(np.max(np.abs(x - y))), "scale": float(np.max(np.abs(x)))}
                continue
            res[f] = {"max_abs": float(np.max(np.abs(x - y))),
                      "max_abs_solid": float(np.max(np.abs(x[solid] - y[solid]))) if solid.any() else 0.0,
                      "max_abs_fluid": float(np.max(np.abs(x[~solid] - y[~solid]))) if (~solid).any() else 0.0,
                      "scale": float(np.max(np.abs(x)))}
        out["checkpoints"][str(k)] = res
        print("step %d %.0f s" % (k, time.time() - t0), file=sys.stderr, flush=True)
    json.dump(out, sys.stdout, indent=1)
    print()


if __name__ == "__main__":
    main()
