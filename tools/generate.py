#!/usr/bin/env python3
"""In-repo particle generator: the reference generator's Cuboid algorithm
(generator.cpp:128-184 readCuboid, 654-677 genparticle, 839-862 writefile) restated in
particlemethod_fsi_amd/mphio.py, from a .boid file or a registered case.

  python tools/generate.py --boid dam.boid out.grid            # the generator's ASCII .grid
  python tools/generate.py --case d16m out.gridb --binary      # binary grid (mph_write_grid_binary)
  python tools/generate.py --case bar2d out.grid --data out.data   # + the case's .data file

The ASCII output is the generator's text (positions rounded through %e exactly as the solver
reads them back); the binary grid holds the same values and is read by the same entry points
(mph_read_grid_*, mph_explicit) without text parsing.
"""
import argparse
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from particlemethod_fsi_amd import cases, mphio, solver  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    src = ap.add_mutually_exclusive_group(required=True)
    src.add_argument("--boid")
    src.add_argument("--case")
    ap.add_argument("out")
    ap.add_argument("--binary", action="store_true")
    ap.add_argument("--data", help="also write the case's .data file (--case only)")
    a = ap.parse_args()
    t0 = time.time()
    if a.boid:
        spacing, lower, upper, cubs = mphio.parse_boid(open(a.boid).read())
        dim = 2 if all(abs(c.upper[2] - c.lower[2]) <= 1.01 * c.space for c in cubs) else 3
    else:
        c = cases.get(a.case)
        spacing, lower, upper, cubs, dim = c.spacing, c.lower, c.upper, c.cuboids, c.dim
        if a.data:
            with open(a.data, "w") as fh:
                fh.write(cases.data_text(c.data()))
    parts = mphio.generate(cubs)
    if a.binary:
        cfg = mphio.config_default(dim, "bar")
        cfg.time = 0.0
        cfg.particle_spacing = spacing
        for d in range(3):
            cfg.domain_min[d] = lower[d]
            cfg.domain_max[d] = upper[d]
        solver.write_grid_binary(a.out, cfg, parts)
    else:
        with open(a.out, "w") as fh:
            fh.write(mphio.format_grid(parts, spacing, lower, upper))
    print("%d particles -> %s (%d bytes, %.1f s)" % (parts.n, a.out, os.path.getsize(a.out), time.time() - t0))


if __name__ == "__main__":
    main()
