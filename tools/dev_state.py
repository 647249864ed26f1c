#!/usr/bin/env python3
"""Write the developed state of a case -- the GPU run to a given step count from the generator's
lattice -- as a binary grid (mph_write_grid_binary: Time, x, x0, v; what a .prof restart holds,
main.cpp:957-982), so that profiles and A/B runs can start from it (bench.py --state).

  python tools/dev_state.py d1m 2500 gpurun_out/d1m_dev.gridb
"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from particlemethod_fsi_amd import MphSolver, cases, mphio, solver  # noqa: E402


def main():
    name, steps, out = sys.argv[1], int(sys.argv[2]), sys.argv[3]
    cfg, parts = cases.get(name).build()
    t0 = time.time()
    with MphSolver(cfg, parts) as s:
        s.step(steps)
        pos, vel, t = s.get("Position"), s.get("Velocity"), s.time
    c = cfg.copy()
    c.time = t
    solver.write_grid_binary(out, c, mphio.Particles(parts.property, pos, parts.initial_position, vel))
    print("%s: %d steps (t = %.6f s) -> %s in %.1f s" % (name, steps, t, out, time.time() - t0))


if __name__ == "__main__":
    main()
