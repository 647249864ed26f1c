#!/usr/bin/env python3
"""How the FSI cases evolve on the GPU: fluid front, gate displacement and max|F - I| every K
steps (finite check included), to choose the hand-off time of test_gpu_longrun.py.

  python tools/fsi_sub_probe.py fsi3d_sub 250 3000
"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402

from particlemethod_fsi_amd import MphSolver, cases  # noqa: E402


def main():
    name, every, total = sys.argv[1], int(sys.argv[2]), int(sys.argv[3])
    cfg, parts = cases.get(name).build()
    solid = (parts.property >= 2) & (parts.property < 4)
    fluid = parts.property < 2
    print("%s n=%d solid=%d gate face %.4f" % (name, parts.n, int(solid.sum()),
                                               float(parts.position[solid, 0].min())), flush=True)
    with MphSolver(cfg, parts) as s:
        t0 = time.time()
        for k in range(every, total + 1, every):
            s.step(every)
            pos = s.get("Position")
            F = s.get("DeformGradient")[solid]
            d = pos[solid] - parts.position[solid]
            print("step %5d t=%.4f front %.4f gate max|u| %.3e max ux %.3e max|F-I| %.3e finite %s  %.1f s"
                  % (k, s.time, float(pos[fluid, 0].max()), float(np.abs(d).max()), float(d[:, 0].max()),
                     float(np.abs(F - np.eye(3)).max()), bool(np.isfinite(pos).all()), time.time() - t0),
                  flush=True)


if __name__ == "__main__":
    main()
