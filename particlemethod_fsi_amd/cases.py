"""Benchmark and parity configurations, generated in memory.

All particle sets come from the reference generator's Cuboid algorithm (mphio.generate, byte-
identical to generator/generator.cpp on results/Dam/dam.boid) and all physical parameters from
the reference example ``results/Dam/dam.data`` (values below), with the documented changes.
There is no RNG anywhere in the reference, so the cases are fully deterministic.
"""
from __future__ import annotations

from dataclasses import dataclass, field

from . import mphio
from .mphio import Cuboid

# results/Dam/dam.data (the reference's only example parameter file), as key -> values.
DAM_DATA = {
    "Dt": [1.0e-4],
    "ElasticDt": [1.0e-4],
    "OutputInterval": [1.0],
    "VtkOutputInterval": [1.0e-2],
    "EndTime": [1.0],
    "RadiusRatioA": [2.5],
    "RadiusRatioP": [2.5],
    "RadiusRatioV": [2.5],
    "Density": [1.0e+3, 1.0e+3, 1.1e+3, 1.0e+3, 1.0e+3, 6.0e+3],
    "BulkModulus": [1.0e+4, 1.0e+4, 1.0e+4, 1.0e+6, 1.0e+4, 1.0e+5],
    "BulkViscosity": [1.0e+1, 1.0e-1, 1.0e-1, 1.0e+3, 1.0e-1, 1.0e+2],
    "ShearViscosity": [1.0e-2, 1.0e-3, 1.0e-2, 1.0e-1, 1.0e+3, 1.0e-1],
    "SurfaceTension": [0.0, 0.0, 0.0, 0.0],
    "YoungModulus": [1e5, 1e+5, 1e+8, 1e+4],
    "PoissonRatio": [0.2, 0.4, 0.3, 0.3],
    "Gravity": [0.0, -1.0, 0.0],
}
for _t in range(6):
    DAM_DATA["InteractionRatio(Type%d)" % _t] = [1.0] * 6


def data_text(values: dict) -> str:
    """A .data file in the reference's keyword format (main.cpp:743-767)."""
    lines = ["#######"]
    for k, v in values.items():
        if isinstance(v, str):   # e.g. "Wall6" -> "Center x y z Velocity ... Omega ..." (main.cpp:766)
            lines.append("%s  %s" % (k, v))
        else:
            lines.append("%s\t%s" % (k, "\t".join(repr(float(x)) for x in v)))
    return "\n".join(lines) + "\n"


@dataclass
class Case:
    name: str
    dim: int
    module: str
    spacing: float
    lower: tuple
    upper: tuple
    cuboids: list
    data_changes: dict = field(default_factory=dict)
    note: str = ""
    wall_motion: int = 0   # MphWallMotion: 1 = the reference's compile-time `Rolling` (main.cpp:58)
    time0: float = 0.0     # the .grid Time line (a restart time, main.cpp:797); "%f" text
    # reference functions run once after the initialisation sums, e.g. the commented
    # setInitialVelocityProfile() call of main.cpp:571
    init_calls: tuple = ()
    # off-lattice parity cases: every coordinate moved by a deterministic offset in
    # [-jitter, jitter) x spacing (mphio.jitter); 0 = the generator's lattice
    jitter: float = 0.0

    @property
    def ref_variant(self) -> str:
        """Which oracle/_ref build holds the reference for this case (module + #defines)."""
        return self.module + ("_rolling" if self.wall_motion else "")

    def describe(self) -> str:
        """One-line description for bench.py's config.workload."""
        return self.note or "%d-D %s-module case" % (self.dim, self.module)

    def data(self) -> dict:
        d = dict(DAM_DATA)
        d.update(self.data_changes)
        return d

    def build(self):
        """-> (MphConfig, Particles), exactly what the reference reads from data + grid files."""
        cfg, _ = self._config()
        return cfg, self._particles()

    def _particles(self):
        p = mphio.generate(self.cuboids)
        return mphio.jitter(p, self.spacing, self.jitter, self.dim) if self.jitter else p

    def build_window(self, axis: int, lo: float, hi: float):
        """-> (MphConfig, Particles, ids, n_glob): only the particles whose coordinate along `axis`
        lies in the periodic window [lo, hi) (a slab rank's share, mph_slab_window), generated
        without the rest of the problem; ids are their indices in build()'s order."""
        if self.jitter:
            raise ValueError("slab-local generation of a jittered case")
        cfg, _ = self._config()
        W = cfg.domain_max[axis] - cfg.domain_min[axis]
        parts, ids, n_glob = mphio.generate_window(self.cuboids, axis, lo, hi, cfg.domain_min[axis], W)
        return cfg, parts, ids, n_glob

    def _config(self):
        cfg = mphio.config_default(self.dim, self.module)
        _apply_data(cfg, self.data())
        cfg.wall_motion = self.wall_motion
        cfg.time = float("%f" % self.time0)
        cfg.particle_spacing = mphio._e(self.spacing)
        for d in range(3):
            cfg.domain_min[d] = mphio._e(self.lower[d])
            cfg.domain_max[d] = mphio._e(self.upper[d])
        return cfg, None

    def grid_text(self) -> str:
        return mphio.format_grid(self._particles(), self.spacing, self.lower, self.upper, self.time0)


def _apply_data(cfg, values):
    import tempfile, os
    with tempfile.NamedTemporaryFile("w", suffix=".data", delete=False) as fh:
        fh.write(data_text(values))
        path = fh.name
    try:
        mphio.read_data_file(path, cfg)
    finally:
        os.unlink(path)


CASES: dict[str, Case] = {}


def _reg(c: Case):
    CASES[c.name] = c
    return c


# results/Dam (as-shipped 2-D Bar_Module binary; no structure particles) -- 6,650 particles
_reg(Case("dam2d", 2, "bar", 0.001, (-0.01, 0.0, 0.0), (0.21, 0.40, 0.001), [
    Cuboid(1, (0.0, 0.003, 0.0), (0.05, 0.10, 0.001), 0.001),
    Cuboid(4, (0.0, 0.0, 0.0), (0.2, 0.003, 0.001), 0.001),
    Cuboid(4, (0.2, 0.0, 0.0), (0.203, 0.20, 0.001), 0.001),
    Cuboid(4, (-0.003, 0.0, 0.0), (0.0, 0.20, 0.001), 0.001),
], note="results/Dam/dam.boid"))

# 3-D dam break, 1,397,200 particles (970,000 fluid / 427,200 wall)
_reg(Case("d1m", 3, "dam", 0.001, (-0.01, 0.0, -0.01), (0.21, 0.40, 0.11), [
    Cuboid(1, (0.0, 0.003, 0.0), (0.1, 0.1, 0.1), 0.001),
    Cuboid(4, (0.0, 0.0, 0.0), (0.2, 0.003, 0.1), 0.001),
    Cuboid(4, (0.2, 0.0, 0.0), (0.203, 0.2, 0.1), 0.001),
    Cuboid(4, (-0.003, 0.0, 0.0), (0.0, 0.2, 0.1), 0.001),
    Cuboid(4, (-0.003, 0.0, -0.003), (0.203, 0.2, 0.0), 0.001),
    Cuboid(4, (-0.003, 0.0, 0.1), (0.203, 0.2, 0.103), 0.001),
], note="3-D dam break (SURVEY 8d D1M, BASELINE configs[1])"))

# 3-D dam break, dx 4e-4, 16,205,500 particles, Dt = ElasticDt = 4e-5
_reg(Case("d16m", 3, "dam", 0.0004, (-0.004, 0.0, -0.004), (0.208, 0.40, 0.108), [
    Cuboid(1, (0.0, 0.0012, 0.0), (0.1, 0.088, 0.1), 0.0004),
    Cuboid(4, (0.0, 0.0, 0.0), (0.2, 0.0012, 0.1), 0.0004),
    Cuboid(4, (0.2, 0.0, 0.0), (0.2012, 0.2, 0.1), 0.0004),
    Cuboid(4, (-0.0012, 0.0, 0.0), (0.0, 0.2, 0.1), 0.0004),
    Cuboid(4, (-0.0012, 0.0, -0.0012), (0.2012, 0.2, 0.0), 0.0004),
    Cuboid(4, (-0.0012, 0.0, 0.1), (0.2012, 0.2, 0.1012), 0.0004),
], data_changes={"Dt": [4e-5], "ElasticDt": [4e-5]},
   note="3-D dam break, dx 0.4 mm (SURVEY 8d D16M, BASELINE configs[4] on one GPU)"))

# SURVEY 8d FSI: 3-D dam break onto an elastic gate, DAM_Module, 2,259,700 particles
_reg(Case("fsi3d", 3, "dam", 0.001, (-0.01, 0.0, -0.01), (0.31, 0.40, 0.11), [
    Cuboid(1, (0.0, 0.003, 0.0), (0.12, 0.14, 0.1), 0.001),
    Cuboid(2, (0.2, 0.0, 0.0), (0.205, 0.08, 0.1), 0.001),
    Cuboid(4, (0.0, 0.0, 0.0), (0.2, 0.003, 0.1), 0.001),
    Cuboid(4, (0.205, 0.0, 0.0), (0.3, 0.003, 0.1), 0.001),
    Cuboid(4, (0.3, 0.0, 0.0), (0.303, 0.2, 0.1), 0.001),
    Cuboid(4, (-0.003, 0.0, 0.0), (0.0, 0.2, 0.1), 0.001),
    Cuboid(4, (-0.003, 0.0, -0.003), (0.303, 0.2, 0.0), 0.001),
    Cuboid(4, (-0.003, 0.0, 0.1), (0.303, 0.2, 0.103), 0.001),
], note="3-D dam break onto an elastic gate, coupled FSI (SURVEY 8d FSI, BASELINE configs[3]) at the survey's "
        "ElasticDt = Dt, at which the reference's own gate goes unstable within ~50 steps; the FSI "
        "workload that runs to completion is fsi3d_sub"))

# SURVEY 8d Bar (parity size): 2-D cantilever, Bar_Module, 4,000 structure particles
_reg(Case("bar2d", 2, "bar", 0.001, (-0.01, -0.1, 0.0), (0.25, 0.1, 0.001), [
    Cuboid(2, (0.0, -0.01, 0.0), (0.2, 0.01, 0.001), 0.001),
]))

# SURVEY 8d Bar (perf size): dx 1e-4, 400,000 structure particles, Dt = ElasticDt = 1e-5
_reg(Case("bar2d_400k", 2, "bar", 0.0001, (-0.001, -0.05, 0.0), (0.25, 0.05, 0.0001), [
    Cuboid(2, (0.0, -0.01, 0.0), (0.2, 0.01, 0.0001), 0.0001),
], data_changes={"Dt": [1e-5], "ElasticDt": [1e-5]},
   note="2-D elastic cantilever, total-Lagrangian solid (SURVEY 8d Bar, BASELINE configs[2])"))

# small 3-D cantilever (Bar_Module): the 3-D elastic path across slab faces (slab tests)
_reg(Case("bar3d", 3, "bar", 0.001, (-0.01, -0.03, -0.03), (0.08, 0.03, 0.03), [
    Cuboid(2, (0.0, -0.005, -0.005), (0.06, 0.005, 0.005), 0.001),
], note="3-D elastic cantilever, 6,000 structure particles (slab tests)"))

# 2-D dam break onto an elastic gate (DAM_Module), 7,035 particles = 4,850 + 400 + 1,785
_reg(Case("gate2d", 2, "dam", 0.001, (-0.01, 0.0, 0.0), (0.21, 0.40, 0.001), [
    Cuboid(1, (0.0, 0.003, 0.0), (0.05, 0.10, 0.001), 0.001),
    Cuboid(2, (0.1, 0.0, 0.0), (0.105, 0.08, 0.001), 0.001),
    Cuboid(4, (0.0, 0.0, 0.0), (0.1, 0.003, 0.001), 0.001),
    Cuboid(4, (0.105, 0.0, 0.0), (0.2, 0.003, 0.001), 0.001),
    Cuboid(4, (0.2, 0.0, 0.0), (0.203, 0.20, 0.001), 0.001),
    Cuboid(4, (-0.003, 0.0, 0.0), (0.0, 0.20, 0.001), 0.001),
]))

# small 3-D dam break in a closed tank (parity size for the 3-D code path)
_reg(Case("box3d", 3, "dam", 0.001, (-0.01, 0.0, -0.01), (0.04, 0.05, 0.025), [
    Cuboid(1, (0.0, 0.003, 0.0), (0.012, 0.02, 0.012), 0.001),
    Cuboid(4, (0.0, 0.0, 0.0), (0.025, 0.003, 0.012), 0.001),
    Cuboid(4, (0.025, 0.0, 0.0), (0.028, 0.025, 0.012), 0.001),
    Cuboid(4, (-0.003, 0.0, 0.0), (0.0, 0.025, 0.012), 0.001),
    Cuboid(4, (-0.003, 0.0, -0.003), (0.028, 0.025, 0.0), 0.001),
    Cuboid(4, (-0.003, 0.0, 0.012), (0.028, 0.025, 0.015), 0.001),
]))

# small 3-D dam break onto an elastic gate (DAM_Module): 3-D structure + FSI coupling path
_reg(Case("gate3d", 3, "dam", 0.001, (-0.01, 0.0, -0.01), (0.05, 0.05, 0.018), [
    Cuboid(1, (0.0, 0.003, 0.0), (0.012, 0.02, 0.008), 0.001),
    Cuboid(2, (0.022, 0.0, 0.0), (0.025, 0.015, 0.008), 0.001),
    Cuboid(4, (0.0, 0.0, 0.0), (0.022, 0.003, 0.008), 0.001),
    Cuboid(4, (0.025, 0.0, 0.0), (0.035, 0.003, 0.008), 0.001),
    Cuboid(4, (0.035, 0.0, 0.0), (0.038, 0.025, 0.008), 0.001),
    Cuboid(4, (-0.003, 0.0, 0.0), (0.0, 0.025, 0.008), 0.001),
    Cuboid(4, (-0.003, 0.0, -0.003), (0.038, 0.025, 0.0), 0.001),
    Cuboid(4, (-0.003, 0.0, 0.008), (0.038, 0.025, 0.011), 0.001),
]))


# surface-tension variants (the reference example has SurfaceTension = 0): exercise PressureA
# (main.cpp:2212-2259) and DiffuseInterface (2261-2312) with asymmetric InteractionRatio tables
_ST = {"SurfaceTension": [0.072, 0.05, 0.03, 0.01],
       "InteractionRatio(Type1)": [1.0, 1.0, 1.0, 1.0, 0.5, 0.7],
       "InteractionRatio(Type4)": [1.0, 0.8, 1.0, 1.0, 1.0, 1.0]}
_reg(Case("dam2d_st", 2, "bar", 0.001, CASES["dam2d"].lower, CASES["dam2d"].upper,
          CASES["dam2d"].cuboids, data_changes=_ST, note="dam2d with surface tension"))
_reg(Case("box3d_st", 3, "dam", 0.001, CASES["box3d"].lower, CASES["box3d"].upper,
          CASES["box3d"].cuboids, data_changes=_ST, note="box3d with surface tension"))


# the `Rolling` wall motion (calculateWall main.cpp:2974-3030): the tank walls turn about z
# through WallCenter (Wall6 = type 4) by MAX_ANGLE sin(2 pi t / 1.646) while the fluid settles
_ROLL = {"Wall6": "Center 0.1 0.1 0.0 Velocity 0.0 0.0 0.0 Omega 0.0 0.0 0.0"}
_reg(Case("rolling2d", 2, "dam", 0.001, CASES["dam2d"].lower, CASES["dam2d"].upper,
          CASES["dam2d"].cuboids, data_changes=_ROLL, wall_motion=1,
          note="dam2d in a rolling tank (Rolling wall motion)"))
_reg(Case("rolling3d", 3, "dam", 0.001, CASES["box3d"].lower, CASES["box3d"].upper,
          CASES["box3d"].cuboids, data_changes={"Wall6": "Center 0.0125 0.0125 0.006 Velocity 0.0 0.0 0.0 "
                                                         "Omega 0.0 0.0 0.0"}, wall_motion=1,
          note="box3d in a rolling tank (Rolling wall motion)"))


# the shipped rigid wall motion of calculateWall (main.cpp:3031-3071): Wall6/Wall7 (types 4/5)
# translate with Velocity and turn by the quaternion of Omega*Dt (initializeWall 1371-1410) while
# Time < 0.2, after which only WallCenter keeps advancing.  The .grid Time line starts the run at
# 0.1995 (a restart), so both sides of the switch are inside the checked steps.
_MOVE2 = {"Wall6": "Center 0.1 0.1 0.0 Velocity 0.02 0.01 0.0 Omega 0.0 0.0 0.3",
          "Wall7": "Center 0.2 0.1 0.0 Velocity -0.01 0.0 0.0 Omega 0.0 0.0 -0.2"}
_reg(Case("movwall2d", 2, "dam", 0.001, CASES["dam2d"].lower, CASES["dam2d"].upper, [
    Cuboid(1, (0.0, 0.003, 0.0), (0.05, 0.10, 0.001), 0.001),
    Cuboid(4, (0.0, 0.0, 0.0), (0.2, 0.003, 0.001), 0.001),
    Cuboid(5, (0.2, 0.0, 0.0), (0.203, 0.20, 0.001), 0.001),
    Cuboid(4, (-0.003, 0.0, 0.0), (0.0, 0.20, 0.001), 0.001),
], data_changes=_MOVE2, time0=0.1995, note="dam2d with moving walls (restart at Time 0.1995)"))
_reg(Case("movwall3d", 3, "dam", 0.001, CASES["box3d"].lower, CASES["box3d"].upper,
          CASES["box3d"].cuboids,
          data_changes={"Wall6": "Center 0.0125 0.0125 0.006 Velocity 0.01 0.0 -0.02 Omega 0.2 -0.1 0.3"},
          time0=0.1995, note="box3d with a translating + rotating wall (restart at Time 0.1995)"))

# the other case modules of main.cpp:54-59 (Turek_Hron, Rolling1, Hydroelastic):
# updateElasticPosition's clamps (1944-2044) and, for Turek_Hron, the per-step inlet profile
# (setInitialVelocityProfile 419-441, called at 592-594).
# Turek-Hron-like channel, dx 1 cm: fluid over x in (0, 1.6) (inlet x <= 0.01, outlet band
# x > 1.5), walls above and below, a small elastic plate around x0 = 0.205 (the clamp line).
_reg(Case("turek2d", 2, "turek_hron", 0.01, (0.0, -0.05, 0.0), (1.6, 0.46, 0.01), [
    Cuboid(1, (0.0, 0.0, 0.0), (0.19, 0.41, 0.01), 0.01),
    Cuboid(1, (0.19, 0.0, 0.0), (0.25, 0.19, 0.01), 0.01),
    Cuboid(1, (0.19, 0.22, 0.0), (0.25, 0.41, 0.01), 0.01),
    Cuboid(1, (0.25, 0.0, 0.0), (1.6, 0.41, 0.01), 0.01),
    Cuboid(2, (0.19, 0.19, 0.0), (0.25, 0.22, 0.01), 0.01),
    Cuboid(4, (0.0, -0.03, 0.0), (1.6, 0.0, 0.01), 0.01),
    Cuboid(4, (0.0, 0.41, 0.0), (1.6, 0.44, 0.01), 0.01),
], note="2-D Turek-Hron channel with inlet profile (Turek_Hron module)"))
_reg(Case("gate2d_rolling1", 2, "rolling1", 0.001, CASES["gate2d"].lower, CASES["gate2d"].upper,
          CASES["gate2d"].cuboids, note="gate2d under the Rolling1 clamp (x0.y < 0.003)"))
# Hydroelastic: a 2 m plate clamped at both ends (x0 < 0.01 or x0 > 1.99) loaded by a fluid block
_reg(Case("hydro2d", 2, "hydroelastic", 0.005, (-0.05, -0.05, 0.0), (2.05, 0.2, 0.005), [
    Cuboid(1, (0.5, 0.01, 0.0), (1.5, 0.06, 0.005), 0.005),
    Cuboid(2, (0.0, 0.0, 0.0), (2.0, 0.01, 0.005), 0.005),
], note="clamped elastic plate under a fluid block (Hydroelastic module)"))
# Bar_Module with the (commented-out, main.cpp:571) initial velocity profile of the beam
_reg(Case("bar2d_ivp", 2, "bar", CASES["bar2d"].spacing, CASES["bar2d"].lower, CASES["bar2d"].upper,
          CASES["bar2d"].cuboids, init_calls=("setInitialVelocityProfile",),
          note="bar2d started in its first bending mode (setInitialVelocityProfile)"))


# elastic sub-stepping (main.cpp:653-663): ElasticDt = Dt/5 -> 5 substeps per step.  With the
# example's ElasticDt = Dt the 3-D gate runs at dt*c/dx ~ 1 and (with the doubled drift of
# updateElasticPosition) goes unstable after ~20 steps; sub-stepping keeps it stable.
_reg(Case("gate2d_sub", 2, "dam", 0.001, CASES["gate2d"].lower, CASES["gate2d"].upper,
          CASES["gate2d"].cuboids, data_changes={"ElasticDt": [2e-5]}, note="gate2d, 5 substeps"))
_reg(Case("gate3d_sub", 3, "dam", 0.001, CASES["gate3d"].lower, CASES["gate3d"].upper,
          CASES["gate3d"].cuboids, data_changes={"ElasticDt": [2.5e-5]}, note="gate3d, 4 substeps"))
# The FSI workload that runs to completion: configs[3]'s geometry (fsi3d,
# 2,259,700 particles) with 4 elastic substeps per step, as gate3d_sub.  fsi3d itself keeps the
# survey's ElasticDt = Dt, at which the reference's own gate is unstable.
_reg(Case("fsi3d_sub", 3, "dam", 0.001, CASES["fsi3d"].lower, CASES["fsi3d"].upper,
          CASES["fsi3d"].cuboids, data_changes={"ElasticDt": [2.5e-5]},
          note="3-D dam break onto an elastic gate, coupled FSI, 4 elastic substeps per step "
               "(BASELINE configs[3] geometry; the stable FSI workload)"))


# Off-lattice 3-D cases: every particle of box3d / the sub-stepped gate moved by up to
# +-0.3 dx per axis, so neighbour distances are no longer whole multiples of dx and pairs lie
# anywhere around the cutoff -- the regime of a developed flow, for the search's FP32 band and the
# sums' tolerances.
_reg(Case("box3d_jit", 3, "dam", 0.001, CASES["box3d"].lower, CASES["box3d"].upper, CASES["box3d"].cuboids,
          jitter=0.3, note="box3d with +-0.3 dx deterministic offsets"))
_reg(Case("gate3d_jit", 3, "dam", 0.001, CASES["gate3d"].lower, CASES["gate3d"].upper, CASES["gate3d"].cuboids,
          data_changes={"ElasticDt": [2.5e-5]}, jitter=0.3,
          note="gate3d_sub with +-0.3 dx deterministic offsets"))


# Slab-decomposition (multi-GPU) parity cases: a fluid layer over a floor, periodic along the
# slab axis and streaming along it at 0.5 m/s, so that within ~20 steps every face-adjacent
# layer migrates to the next slab and the periodic seam is crossed (nothing moves far enough
# in the dam cases).  Slab axis: z (3-D), x (2-D).
_U = 0.5
_reg(Case("channel3d", 3, "dam", 0.001, (-0.01, 0.0, 0.0), (0.025, 0.04, 0.036), [
    Cuboid(1, (0.0, 0.003, 0.0), (0.012, 0.015, 0.036), 0.001, (0.0, 0.0, _U)),
    Cuboid(4, (-0.003, 0.0, 0.0), (0.015, 0.003, 0.036), 0.001),
    Cuboid(4, (-0.003, 0.003, 0.0), (0.0, 0.02, 0.036), 0.001),
    Cuboid(4, (0.012, 0.003, 0.0), (0.015, 0.02, 0.036), 0.001),
], note="periodic 3-D channel flow (slab tests)"))
_reg(Case("channel2d", 2, "dam", 0.001, (0.0, 0.0, 0.0), (0.04, 0.03, 0.001), [
    Cuboid(1, (0.0, 0.003, 0.0), (0.04, 0.015, 0.001), 0.001, (_U, 0.0, 0.0)),
    Cuboid(4, (0.0, 0.0, 0.0), (0.04, 0.003, 0.001), 0.001),
], note="periodic 2-D channel flow (slab tests)"))
# fluid on both sides of the periodic y face with empty space between: the GPU grid's origin
# moves into the gap (choose_grid_origin), so the y face lies inside the grid and the pairs across
# it need the search's face rule (DevState.seam_occ) -- parity test of that rule
_reg(Case("seam3d", 3, "dam", 0.001, (0.0, 0.0, 0.0), (0.03, 0.04, 0.02), [
    Cuboid(1, (0.0, 0.0, 0.0), (0.03, 0.006, 0.02), 0.001, (0.0, -_U, 0.0)),
    Cuboid(1, (0.0, 0.034, 0.0), (0.03, 0.04, 0.02), 0.001, (_U, 0.0, 0.0)),
], note="fluid across the periodic y face, empty band between (grid origin / face rule)"))
# a box of water on a floor 11 m along a 12 m periodic z axis: ~9,200 GPU cells along the search's
# contiguous axis, the water at cell ~8,460, past the 8,192 where an absolute FP32 cell coordinate
# would lose the 1e-3-cell margin of the search's column ranges
_reg(Case("longz3d", 3, "dam", 0.001, (-0.01, -0.01, 0.0), (0.04, 0.04, 12.0), [
    Cuboid(4, (0.0, 0.0, 11.0), (0.03, 0.003, 11.03), 0.001),
    Cuboid(1, (0.003, 0.003, 11.003), (0.027, 0.02, 11.027), 0.001),
], note="water on a floor far along a long contiguous cell axis"))
_reg(Case("channel3d_st", 3, "dam", 0.001, CASES["channel3d"].lower, CASES["channel3d"].upper,
          CASES["channel3d"].cuboids, data_changes=_ST, note="channel3d with surface tension"))


def d1m_weak(nranks: int) -> Case:
    """Weak-scaling workload of bench.py --gpus N: the D1M tank extended N-fold
    along z (slab axis), so each of N slabs holds about one D1M (N = 1 is D1M itself)."""
    if nranks == 1:
        return CASES["d1m"]
    zl = 0.1 * nranks
    return Case("d1m_x%d" % nranks, 3, "dam", 0.001, (-0.01, 0.0, -0.01), (0.21, 0.40, zl + 0.01), [
        Cuboid(1, (0.0, 0.003, 0.0), (0.1, 0.1, zl), 0.001),
        Cuboid(4, (0.0, 0.0, 0.0), (0.2, 0.003, zl), 0.001),
        Cuboid(4, (0.2, 0.0, 0.0), (0.203, 0.2, zl), 0.001),
        Cuboid(4, (-0.003, 0.0, 0.0), (0.0, 0.2, zl), 0.001),
        Cuboid(4, (-0.003, 0.0, -0.003), (0.203, 0.2, 0.0), 0.001),
        Cuboid(4, (-0.003, 0.0, zl), (0.203, 0.2, zl + 0.003), 0.001),
    ], note="3-D dam break, D1M extended %dx along z (weak scaling)" % nranks)


def get(name: str) -> Case:
    if name.startswith("d1m_x"):
        return d1m_weak(int(name[5:]))
    return CASES[name]
