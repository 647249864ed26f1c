"""GPU parity at the BASELINE.json configuration sizes, against the CPU oracle.

The oracle is bit-identical to the reference (tests/test_oracle.py), so it stands in for the
reference at sizes whose golden files would be too large to commit:

  d1m         3-D dam break, 1,397,200 particles            (configs[1], the bench workload)
  fsi3d       3-D dam onto an elastic gate, 2,259,700       (configs[3])
  bar2d_400k  2-D elastic cantilever, 400,000 structure     (configs[2])

Compared over the bench's horizon: D1M and FSI after steps 1, 10, 29 and 52 (bench.py's default
warmup 8 + 40 timed + 4 profiled steps = 52; the driver's bench run 5 + 20 + 4 = 29), Bar 400k
after steps 1, 10, 50 and 100 (the oracle needs about a second per D1M step on 16 host cores);
sums of the elastic cases at 1e-7 relative, the solid bound of the other parity tests.  Same
tolerances as
test_gpu_parity.py: NeighborCount exact, positions 1e-12 m, velocities 1e-9 m/s, sums 1e-8
relative + roundoff floor.  Where the reference itself is that sensitive -- the elastic gate
after 29 and 52 steps -- a field passes within 4x the difference between two oracle runs whose
start positions differ by one ulp (tests/golden/ulp_<case>.json, tools/ulp_study.py).  Plus
size-independent properties of the full D1M run: a rerun is bitwise identical and the time
advances by exactly Dt per step.
"""
import os

import numpy as np
import pytest

from particlemethod_fsi_amd import MphSolver, cases

pytestmark = pytest.mark.gpu

FLOOR = {"PressureP": 1e-9, "PressureA": 1e-9, "Force": 1e-15, "Acceleration": 1e-12,
         "VolStrainP": 1e-13, "DivergenceP": 1e-12, "DensityA": 1e-13, "GravityCenter": 1e-16,
         "DeformGradient": 1e-13, "Strain": 1e-13, "Stress": 1e-8}


def _oracle_threads():
    from oracle_bindings import OracleSolver
    OracleSolver.set_threads(min(16, os.cpu_count() or 1))


CHECKPOINTS = {"d1m": (1, 10, 29, 52), "fsi3d": (1, 10, 29, 52), "bar2d_400k": (1, 10, 50, 100)}
# The reference's own roundoff sensitivity (tools/ulp_study.py: the CPU oracle, bit-identical to
# the reference, run once as given and once with every position moved by one ulp; the max
# difference per field after each checkpoint).  The elastic FSI gate amplifies roundoff ~10x per
# 10 steps, so after 29 / 52 steps two runs of the reference itself differ by more than the
# fixed bounds; a field then passes within ULP_FACTOR x that growth.  The GPU's reassociated sums
# perturb every step by a few ulp, about as much as the one-ulp start.
ULP_FACTOR = 4.0


def _ulp_bound(case, k, f):
    path = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "ulp_%s.json" % case)
    if not os.path.exists(path):
        return 0.0
    import json
    ck = json.load(open(path))["checkpoints"].get(str(k), {})
    return ULP_FACTOR * ck[f]["max_abs"] if f in ck else 0.0


@pytest.mark.parametrize("case", ["d1m", "fsi3d", "bar2d_400k"])
def test_full_size_matches_oracle(case):
    from oracle_bindings import OracleSolver
    _oracle_threads()
    cfg, parts = cases.get(case).build()
    solid = (parts.property >= 2) & (parts.property < 4)
    o = OracleSolver(cfg, parts)
    o.init()
    with MphSolver(cfg, parts) as s:
        assert np.array_equal(s.get("NeighborCount"), o.get("NeighborCount"))
        done = 0
        for k in CHECKPOINTS[case]:
            s.step(k - done)
            o.step(k - done)
            done = k
            assert np.array_equal(s.get("NeighborCount"), o.get("NeighborCount")), (case, k)
            fields = ["Position", "Velocity", "PressureP", "VolStrainP", "DivergenceP", "Force"]
            if solid.any():
                fields += ["DeformGradient", "Stress"]
            for f in fields:
                a, b = s.get(f), o.get(f)
                if f in ("DeformGradient", "Stress"):
                    a, b = a[solid], b[solid]
                scale = float(np.max(np.abs(b))) if b.size else 0.0
                # elastic cases run near the solid's stability limit, where reassociation roundoff
                # grows ~10x per 10 steps: the solid bound of test_gpu_parity / test_gpu_dist
                # (DivergenceP, a difference of nearly equal sums, 1e-6 as in test_gpu_dist)
                rel = (1e-6 if f == "DivergenceP" else 1e-7) if solid.any() else 1e-8
                t = {"Position": 1e-12, "Velocity": 1e-9}.get(f, rel * scale + FLOOR.get(f, 1e-12))
                t = max(t, _ulp_bound(case, k, f))
                err = float(np.max(np.abs(a - b))) if b.size else 0.0
                assert err <= t, (case, k, f, err, t)


def test_d1m_rerun_bitwise_and_time():
    cfg, parts = cases.get("d1m").build()
    outs = []
    for _ in range(2):
        with MphSolver(cfg, parts) as s:
            s.step(12)   # one 8-step graph + 4 single-step graphs
            outs.append((s.get("Position"), s.get("Velocity"), s.get("PressureP"), s.time))
    for a, b in zip(outs[0][:3], outs[1][:3]):
        assert np.array_equal(a, b)
    t = 0.0
    for _ in range(12):
        t += cfg.dt
    assert outs[0][3] == t
