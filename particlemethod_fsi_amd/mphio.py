"""Host-side data formats of the reference solver, mirrored in Python.

* ``MphConfig`` -- ctypes mirror of ``include/mph_gpu.h`` ``MphConfig`` (what the reference
  reads from its ``.data`` file, main.cpp:729-786, and its ``.grid`` header, main.cpp:796-804).
* ``read_data_file`` / ``read_grid_file`` -- pure-Python readers with the reference's
  ``sscanf`` keyword semantics (first matching keyword wins; partially parsed value lists are
  kept, as ``sscanf`` leaves them in the target arrays).
* ``format_grid`` -- the ``.grid`` writer of ``generator/generator.cpp:839-862`` (the solver
  re-reads its ``%e`` text, so positions are the 7-significant-digit values).

The product reader (C++, ``mph_read_data_file`` in libmph_gpu.so) is checked against this one
in tests/test_host_io.py.
"""
from __future__ import annotations

import ctypes
import math
from dataclasses import dataclass

import numpy as np

TYPE_COUNT = 6
MODULES = {"bar": 0, "dam": 1, "turek_hron": 2, "rolling1": 3, "hydroelastic": 4, "none": 5}

_D6 = ctypes.c_double * TYPE_COUNT
_D3 = ctypes.c_double * 3


class MphConfig(ctypes.Structure):
    """Layout-identical to ``MphConfig`` in include/mph_gpu.h."""

    _fields_ = [
        ("dim", ctypes.c_int),
        ("module", ctypes.c_int),
        ("dt", ctypes.c_double),
        ("elastic_dt", ctypes.c_double),
        ("output_interval", ctypes.c_double),
        ("vtk_output_interval", ctypes.c_double),
        ("end_time", ctypes.c_double),
        ("radius_ratio_a", ctypes.c_double),
        ("radius_ratio_p", ctypes.c_double),
        ("radius_ratio_v", ctypes.c_double),
        ("density", _D6),
        ("bulk_modulus", _D6),
        ("bulk_viscosity", _D6),
        ("shear_viscosity", _D6),
        ("surface_tension", _D6),
        ("young_modulus", _D6),
        ("poisson_ratio", _D6),
        ("interaction_ratio", _D6 * TYPE_COUNT),
        ("gravity", _D3),
        ("wall_center", _D3 * TYPE_COUNT),
        ("wall_velocity", _D3 * TYPE_COUNT),
        ("wall_omega", _D3 * TYPE_COUNT),
        ("time", ctypes.c_double),
        ("particle_spacing", ctypes.c_double),
        ("domain_min", _D3),
        ("domain_max", _D3),
        ("wall_motion", ctypes.c_int),
    ]

    def copy(self) -> "MphConfig":
        out = MphConfig()
        ctypes.memmove(ctypes.byref(out), ctypes.byref(self), ctypes.sizeof(MphConfig))
        return out


def config_default(dim: int = 2, module: str | int = "bar") -> MphConfig:
    """Static initial values of the reference globals (main.cpp:83-197: zeros, Dt=1e100)."""
    cfg = MphConfig()
    cfg.dim = int(dim)
    cfg.module = MODULES[module] if isinstance(module, str) else int(module)
    cfg.dt = 1.0e100
    cfg.elastic_dt = 1.0e100
    return cfg


def _floats(tokens, k):
    """sscanf-like: parse up to k leading floats, stop at the first non-number."""
    out = []
    for t in tokens[:k]:
        try:
            out.append(float(t))
        except ValueError:
            break
    return out


# keyword -> (target attribute, indices) in the order of the reference's else-if chain
_SCALARS = [("Dt", "dt"), ("ElasticDt", "elastic_dt"), ("OutputInterval", "output_interval"),
            ("VtkOutputInterval", "vtk_output_interval"), ("EndTime", "end_time"),
            ("RadiusRatioA", "radius_ratio_a"), ("RadiusRatioP", "radius_ratio_p"),
            ("RadiusRatioV", "radius_ratio_v")]
_ARRAYS = [("Density", "density", (0, 1, 2, 3, 4, 5)),
           ("BulkModulus", "bulk_modulus", (0, 1, 2, 3, 4, 5)),
           ("BulkViscosity", "bulk_viscosity", (0, 1, 2, 3, 4, 5)),
           ("ShearViscosity", "shear_viscosity", (0, 1, 2, 3, 4, 5)),
           ("SurfaceTension", "surface_tension", (0, 1, 4, 5)),
           ("YoungModulus", "young_modulus", (2, 3, 4, 5)),
           ("PoissonRatio", "poisson_ratio", (2, 3, 4, 5))]


def read_data_file(path: str, cfg: MphConfig) -> list[str]:
    """Parse a ``.data`` file into ``cfg`` (main.cpp:729-786).  Returns the ignored lines."""
    ignored = []
    with open(path, "r") as fh:
        for line in fh:
            if line.startswith("#"):
                continue
            tok = line.split()
            if not tok:
                ignored.append(line)
                continue
            key, rest = tok[0], tok[1:]
            done = False
            for name, attr in _SCALARS:
                if key == name:
                    vals = _floats(rest, 1)
                    if vals:
                        setattr(cfg, attr, vals[0])
                        done = True
                    break
            if not done:
                for name, attr, idx in _ARRAYS:
                    if key == name:
                        vals = _floats(rest, len(idx))
                        arr = getattr(cfg, attr)
                        for k, v in enumerate(vals):
                            arr[idx[k]] = v
                        done = len(vals) == len(idx)
                        break
            if not done and key.startswith("InteractionRatio(Type") and key.endswith(")") and len(key) == 23:
                t = ord(key[21]) - ord("0")
                if 0 <= t < TYPE_COUNT:
                    vals = _floats(rest, 6)
                    for k, v in enumerate(vals):
                        cfg.interaction_ratio[t][k] = v
                    done = len(vals) == 6
            if not done and key == "Gravity":
                vals = _floats(rest, 3)
                for k, v in enumerate(vals):
                    cfg.gravity[k] = v
                done = len(vals) == 3
            if not done and key in ("Wall6", "Wall7"):
                t = 4 if key == "Wall6" else 5
                done = _parse_wall(rest, cfg, t)
            if not done:
                ignored.append(line)
    return ignored


def _parse_wall(rest, cfg, t) -> bool:
    # " WallX  Center %lf %lf %lf Velocity %lf %lf %lf Omega %lf %lf %lf" (main.cpp:766-767)
    targets = (cfg.wall_center[t], cfg.wall_velocity[t], cfg.wall_omega[t])
    words = ("Center", "Velocity", "Omega")
    pos, got = 0, 0
    for w, arr in zip(words, targets):
        if pos >= len(rest) or rest[pos] != w:
            return False
        vals = _floats(rest[pos + 1:], 3)
        for k, v in enumerate(vals):
            arr[k] = v
        got += len(vals)
        if len(vals) < 3:
            return False
        pos += 4
    return got == 9


@dataclass
class Particles:
    property: np.ndarray      # int32[n]
    position: np.ndarray      # float64[n,3]
    initial_position: np.ndarray
    velocity: np.ndarray

    @property
    def n(self) -> int:
        return int(self.property.shape[0])


def read_grid_file(path: str, cfg: MphConfig) -> Particles:
    """``.grid`` / ``.prof`` reader (main.cpp:788-904)."""
    with open(path, "r") as fh:
        cfg.time = float(fh.readline().split()[0])
        h = fh.readline().split()
        n = int(h[0])
        cfg.particle_spacing = float(h[1])
        cfg.domain_min[0], cfg.domain_max[0] = float(h[2]), float(h[3])
        cfg.domain_min[1], cfg.domain_max[1] = float(h[4]), float(h[5])
        cfg.domain_min[2], cfg.domain_max[2] = float(h[6]), float(h[7])
        body = np.loadtxt(fh, dtype=np.float64, max_rows=n, ndmin=2)
    return Particles(property=body[:, 0].astype(np.int32),
                     position=np.ascontiguousarray(body[:, 1:4]),
                     initial_position=np.ascontiguousarray(body[:, 4:7]),
                     velocity=np.ascontiguousarray(body[:, 7:10]))


# ------------------------------------------------------------------------------------------
# generator (generator/generator.cpp): Cuboid primitive + .grid writer
# ------------------------------------------------------------------------------------------

@dataclass
class Cuboid:
    """One ``StartCuboid ... EndCuboid`` block of a ``.boid`` file (generator.cpp:22-30)."""
    type: int
    lower: tuple
    upper: tuple
    space: float
    velocity: tuple = (0.0, 0.0, 0.0)


def _c_round(x: float) -> int:
    # C round(): half away from zero
    return int(math.floor(x + 0.5)) if x >= 0 else -int(math.floor(-x + 0.5))


def _axis_values(lo: float, hi: float, space: float) -> list[float]:
    # generator.cpp:659-665 -- accumulate px += spacing from lower + 0.5*spacing
    width = hi - lo
    count = _c_round(width / space)
    sp = width / count
    vals = []
    p = lo + 0.5 * sp
    while p < hi - 0.49 * sp:
        vals.append(p)
        p += sp
    return vals


def _e(x: float) -> float:
    """Value the solver reads back from the generator's ``%e`` text."""
    return float("%e" % x)


def generate(cuboids: list[Cuboid]) -> Particles:
    """``genparticle`` for Cuboid blocks (generator.cpp:654-677), values rounded through the
    ``%e`` text of ``writefile`` exactly as the solver will read them."""
    props, pos, vel = [], [], []
    for cub in cuboids:
        ax = [np.array([_e(v) for v in _axis_values(cub.lower[d], cub.upper[d], cub.space)])
              for d in range(3)]
        X, Y, Z = np.meshgrid(ax[0], ax[1], ax[2], indexing="ij")
        p = np.stack([X.ravel(), Y.ravel(), Z.ravel()], axis=1)
        pos.append(p)
        props.append(np.full(p.shape[0], cub.type, dtype=np.int32))
        vel.append(np.tile(np.array([_e(v) for v in cub.velocity]), (p.shape[0], 1)))
    P = np.concatenate(pos) if pos else np.zeros((0, 3))
    return Particles(property=np.concatenate(props) if props else np.zeros(0, np.int32),
                     position=np.ascontiguousarray(P), initial_position=P.copy(),
                     velocity=np.ascontiguousarray(np.concatenate(vel)) if vel else np.zeros((0, 3)))


def generate_window(cuboids: list[Cuboid], axis: int, lo: float, hi: float, dmin: float, width: float):
    """The particles of ``generate(cuboids)`` whose coordinate along ``axis`` lies in the periodic
    window [lo, hi) of a domain starting at ``dmin`` with ``width``, without building the others
    (slab-local creation, include/mph_gpu.h mph_create_slab).  Returns (Particles, ids, n_glob):
    the original indices of the kept particles (ascending) and the total count.  Cuboid lattices
    are separable, so the window only filters the value list of one axis."""
    span = hi - lo
    props, pos, vel, ids = [], [], [], []
    base = 0
    for cub in cuboids:
        ax = [np.array([_e(v) for v in _axis_values(cub.lower[d], cub.upper[d], cub.space)])
              for d in range(3)]
        cnt = [len(a) for a in ax]
        keep = [np.arange(c) for c in cnt]
        if span < width:
            a = ax[axis]
            u = a - dmin
            u = u - width * np.floor(u / width) + dmin    # periodic wrap into [dmin, dmin + width)
            off = (u - lo) - width * np.floor((u - lo) / width)
            keep[axis] = np.nonzero(off < span)[0]
        if all(len(k) for k in keep):
            I, J, K = np.meshgrid(keep[0], keep[1], keep[2], indexing="ij")
            ids.append(base + ((I * cnt[1] + J) * cnt[2] + K).ravel())
            X, Y, Z = np.meshgrid(ax[0][keep[0]], ax[1][keep[1]], ax[2][keep[2]], indexing="ij")
            p = np.stack([X.ravel(), Y.ravel(), Z.ravel()], axis=1)
            pos.append(p)
            props.append(np.full(p.shape[0], cub.type, dtype=np.int32))
            vel.append(np.tile(np.array([_e(v) for v in cub.velocity]), (p.shape[0], 1)))
        base += cnt[0] * cnt[1] * cnt[2]
    P = np.concatenate(pos) if pos else np.zeros((0, 3))
    parts = Particles(property=np.concatenate(props) if props else np.zeros(0, np.int32),
                      position=np.ascontiguousarray(P), initial_position=P.copy(),
                      velocity=np.ascontiguousarray(np.concatenate(vel)) if vel else np.zeros((0, 3)))
    idx = np.concatenate(ids).astype(np.int32) if ids else np.zeros(0, np.int32)
    return parts, idx, base


def plane_counts(cuboids: list[Cuboid], axis: int, dmin: float, width: float):
    """(coordinates, counts): the lattice planes of ``generate(cuboids)`` along ``axis`` (wrapped
    into the periodic domain [dmin, dmin + width), ascending) and the particles on each -- the
    particle distribution along a slab axis without generating the particles."""
    vals, cnts = [], []
    for cub in cuboids:
        ax = [np.array([_e(v) for v in _axis_values(cub.lower[d], cub.upper[d], cub.space)])
              for d in range(3)]
        per = len(ax[(axis + 1) % 3]) * len(ax[(axis + 2) % 3])
        u = ax[axis] - dmin
        vals.append(u - width * np.floor(u / width) + dmin)
        cnts.append(np.full(len(ax[axis]), per, np.int64))
    if not vals:
        return np.zeros(0), np.zeros(0, np.int64)
    v, c = np.concatenate(vals), np.concatenate(cnts)
    order = np.argsort(v, kind="stable")
    v, c = v[order], c[order]
    uv, inv = np.unique(v, return_inverse=True)
    return uv, np.bincount(inv, weights=c).astype(np.int64)


def format_grid(p: Particles, spacing: float, lower, upper, time: float = 0.0) -> str:
    """Text of the generator's ``writefile`` (generator.cpp:839-862); ``time`` is the first line
    (0 from the generator; a .prof restart carries its Time, main.cpp:797, 961)."""
    out = ["%f\n" % time,
           "%d %e  %e %e %e  %e %e %e\n" % (p.n, spacing, lower[0], upper[0], lower[1], upper[1],
                                             lower[2], upper[2])]
    for i in range(p.n):
        x = p.position[i]
        v = p.velocity[i]
        out.append("%d   %e %e %e %e %e %e  %e %e %e \n" % (
            p.property[i], x[0], x[1], x[2], x[0], x[1], x[2], v[0], v[1], v[2]))
    return "".join(out)


def parse_boid(text: str):
    """Minimal ``.boid`` parser for Cuboid blocks (generator.cpp:128-184, readCuboid)."""
    spacing, lower, upper, cubs = None, None, None, []
    lines = iter(text.splitlines())
    for line in lines:
        tok = line.split()
        if not tok or tok[0].startswith("#"):
            continue
        if tok[0] == "ParticleDistance":
            spacing = float(tok[1])
        elif tok[0] == "LowerDomain":
            lower = tuple(float(t) for t in tok[1:4])
        elif tok[0] == "UpperDomain":
            upper = tuple(float(t) for t in tok[1:4])
        elif tok[0] == "StartCuboid":
            c = {"Velocity": (0.0, 0.0, 0.0)}
            for inner in lines:
                t2 = inner.split()
                if not t2:
                    continue
                if t2[0] == "EndCuboid":
                    break
                if t2[0] in ("Lower", "Upper", "Velocity"):
                    c[t2[0]] = tuple(float(t) for t in t2[1:4])
                elif t2[0] in ("Spacing",):
                    c["Spacing"] = float(t2[1])
                elif t2[0] == "Type":
                    c["Type"] = int(t2[1])
            cubs.append(Cuboid(type=c["Type"], lower=c["Lower"], upper=c["Upper"],
                               space=c["Spacing"], velocity=c["Velocity"]))
    return spacing, lower, upper, cubs
