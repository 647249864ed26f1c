"""GPU parity in the DEVELOPED 3-D dam break.

The full-size tests of test_gpu_fullsize.py stop at 52 steps, where D1M's fluid has moved ~0.01 dx
and every neighbour set is still the initial lattice's.  The reference's own Dam run is 10,001
steps (main.cpp:581; results/Dam/dam.data EndTime 1.0 at Dt 1e-4).  Here the GPU runs D1M
(BASELINE configs[1], 1,397,200 particles) to t = 0.25 s (2,500 steps) and to t = 1.0 s (10,000
steps, the end of the reference's run): the column has collapsed
along the floor, particles are off the lattice and the neighbour sets have changed.  That exact
state (Position, Velocity, Time -- everything the step carries; walls are static in this case) is
handed to the CPU oracle, bit-identical to the reference, as the reference's own restart from a
.prof file would read it (main.cpp:788-955), and both advance 1 and 10 more steps:

  * NeighborCount exact; the neighbour SETS of sample ranges (mph_neighbor_rows of a context built
    from the state with the reference's whole lists) equal to the oracle's lists (main.cpp:1764-1772);
  * Position 1e-12 m, Velocity 1e-9 m/s, PressureP / VolStrainP / DivergenceP / Force within 1e-8 of
    their largest magnitude plus the roundoff floors of test_gpu_parity.py;
  * the state did leave the lattice: NeighborCount differs from the creation's for >= 1 % of the
    particles, and the fluid front moved by more than 10 dx.
"""
import os

import numpy as np
import pytest

from particlemethod_fsi_amd import MphSolver, cases, mphio

pytestmark = pytest.mark.gpu

FLOOR = {"PressureP": 1e-9, "Force": 1e-15, "VolStrainP": 1e-13, "DivergenceP": 1e-12}
DEVELOPED_STEPS = 2500           # t = 0.25 s at Dt = 1e-4
SAMPLE_ROWS = [(0, 4000), (485000, 4000), (966000, 4000), (1200000, 4000)]   # fluid (3) and wall


@pytest.mark.parametrize("steps", [DEVELOPED_STEPS, 10000])   # t = 0.25 s, and t = 1.0 s: the reference's whole Dam run
def test_d1m_developed_matches_oracle(steps):
    from oracle_bindings import OracleSolver
    OracleSolver.set_threads(min(16, os.cpu_count() or 1))
    cfg, parts = cases.get("d1m").build()
    fluid = parts.property < 2
    with MphSolver(cfg, parts) as s:
        nc0 = s.get("NeighborCount")
        s.step(steps)
        pos, vel = s.get("Position"), s.get("Velocity")
        nc_dev = s.get("NeighborCount")
        changed = float((nc_dev != nc0).mean())
        front0 = float(parts.position[fluid, 0].max())
        front = float(pos[fluid, 0].max())
        print("developed: t=%.4f changed=%.3f front %.4f -> %.4f m, max|v| %.3f m/s"
              % (s.time, changed, front0, front, float(np.abs(vel).max())))
        assert changed >= 0.01, changed
        assert front - front0 > 10 * cfg.particle_spacing, (front0, front)
        # restart of the reference from that state (a .prof holds Time, x, x0, v)
        rcfg = cfg.copy()
        rcfg.time = s.time
        state = mphio.Particles(parts.property, pos, parts.initial_position, vel)
        o = OracleSolver(rcfg, state)
        o.init()
        # the neighbour SETS of sample ranges at the restart (main.cpp:1764-1772): a context built
        # from that state with the reference's whole lists (MPH_LIST_FULL=1) against the oracle's
        os.environ["MPH_LIST_FULL"] = "1"
        try:
            with MphSolver(rcfg, state) as full:
                for first, count in SAMPLE_ROWS:
                    counts, offsets, ids = full.neighbor_rows(first, count)
                    for i in range(count):
                        assert np.array_equal(ids[offsets[i]:offsets[i + 1]], np.sort(o.neighbors(first + i))), first + i
        finally:
            del os.environ["MPH_LIST_FULL"]
        done = 0
        for k in (1, 10):
            s.step(k - done)
            o.step(k - done)
            done = k
            assert np.array_equal(s.get("NeighborCount"), o.get("NeighborCount")), k
            for f in ["Position", "Velocity", "PressureP", "VolStrainP", "DivergenceP", "Force"]:
                a, b = s.get(f), o.get(f)
                scale = float(np.max(np.abs(b)))
                t = {"Position": 1e-12, "Velocity": 1e-9}.get(f, 1e-8 * scale + FLOOR.get(f, 1e-12))
                err = float(np.max(np.abs(a - b)))
                assert err <= t, (k, f, err, t)
        assert s.time == o.time
