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

# generator.cpp's shapes, in the order genparticle visits them (654-826): every Cuboid block of
# the .boid file first, then every Cuboid2, Cyboid, Cyboid2, Recboid, Recboid2 block
SHAPES = ("cuboid", "cuboid2", "cyboid", "cyboid2", "recboid", "recboid2")


@dataclass
class Cuboid:
    """One ``Start<Shape> ... End<Shape>`` block of a ``.boid`` file (generator.cpp:22-78).

    kind: "cuboid" (lattice from lower + 0.5 s to upper - 0.49 s on every axis, 663-665),
    "cuboid2" (x and y from lower + 0.01 s to upper, z as cuboid; 689-691), "cyboid" (the cuboid
    lattice inside the spherical shell ratio * w0/2 < r <= w0/2 about the centre; 714-725),
    "cyboid2" (the cuboid2 lattice inside the xy ring of generator.cpp:752), "recboid" (the cuboid2
    lattice where tan(angle) > y/x; 775-784), "recboid2" (the cuboid2 lattice rotated about z by
    angle; 807-811).  Angles in degrees, converted with 3.1415/180 like the generator."""
    type: int
    lower: tuple
    upper: tuple
    space: float
    velocity: tuple = (0.0, 0.0, 0.0)
    kind: str = "cuboid"
    ratio: float = 0.0
    angle: float = 0.0


def _c_round(x: float) -> int:
    # C round(): half away from zero
    return int(math.floor(x + 0.5)) if x >= 0 else -int(math.floor(-x + 0.5))


def _axis_values(lo: float, hi: float, space: float, start: float = 0.5, stop: float = 0.49,
                 stop_space: float | None = None) -> list[float]:
    # generator.cpp:659-665 (and the other shapes' loops): count = round(width / space), spacing
    # = width / count, p accumulated by p += spacing from lower + start * spacing while
    # p < upper - stop * spacing (Recboid's y loop scales its stop by the x spacing, 776, 808)
    width = hi - lo
    count = _c_round(width / space)
    sp = width / count
    lim = hi - stop * (sp if stop_space is None else stop_space)
    vals = []
    p = lo + start * sp
    while p < lim:
        vals.append(p)
        p += sp
    return vals


def _spacing(lo: float, hi: float, space: float) -> float:
    width = hi - lo
    return width / _c_round(width / space)


def _e(x: float) -> float:
    """Value the solver reads back from the generator's ``%e`` text."""
    return float("%e" % x)


def _shape_points(cub: Cuboid) -> np.ndarray:
    """Unrounded positions of one non-cuboid block, in the generator's loop order (x outermost),
    with its own double arithmetic (no FMA: the generator is built with g++ -g, makefile:8)."""
    k = cub.kind
    lo, hi, s = cub.lower, cub.upper, cub.space
    if k == "cyboid":
        ax = [_axis_values(lo[d], hi[d], s) for d in range(3)]
    else:
        sx = _spacing(lo[0], hi[0], s)
        ax = [_axis_values(lo[0], hi[0], s, 0.01, 0.0),
              _axis_values(lo[1], hi[1], s, 0.01, 0.0, stop_space=sx if k.startswith("recboid") else None),
              _axis_values(lo[2], hi[2], s)]
    X, Y, Z = np.meshgrid(np.array(ax[0]), np.array(ax[1]), np.array(ax[2]), indexing="ij")
    px, py, pz = X.ravel(), Y.ravel(), Z.ravel()
    w = [hi[d] - lo[d] for d in range(3)]
    if k == "cuboid2":
        return np.stack([px, py, pz], axis=1)
    if k == "cyboid":
        c = [0.5 * (hi[d] + lo[d]) for d in range(3)]
        x, y, z = px - c[0], py - c[1], pz - c[2]
        r2 = x * x + y * y + z * z
        inner = 0.25 * w[0] * w[0] * cub.ratio * cub.ratio
        outer = 0.25 * w[0] * w[0]
        keep = (r2 > inner) & (r2 <= outer)
        return np.stack([px[keep], py[keep], pz[keep]], axis=1)
    if k == "cyboid2":
        c = [0.5 * (hi[d] + lo[d]) for d in range(2)]
        x, y = px - c[0], py - c[1]
        q = x * x + y * y
        outer = 0.5 * 0.5 * 0.5 * 0.5 * w[0] * w[0] * w[1] * w[1]
        inner = outer * cub.ratio * cub.ratio * cub.ratio * cub.ratio
        keep = (q <= outer) & (q > inner)
        return np.stack([px[keep], py[keep], pz[keep]], axis=1)
    a = cub.angle * 3.1415 / 180
    if k == "recboid":
        with np.errstate(divide="ignore", invalid="ignore"):
            keep = math.tan(a) > py / px    # y / 0: +-inf or NaN as in C
        return np.stack([px[keep], py[keep], pz[keep]], axis=1)
    if k == "recboid2":
        ca, sa = math.cos(a), math.sin(a)
        return np.stack([px * ca - py * sa, px * sa + py * ca, pz], axis=1)
    raise ValueError("unknown generator shape %r" % k)


def generate(cuboids: list[Cuboid]) -> Particles:
    """``genparticle`` (generator.cpp:654-835): every shape kind in the generator's order, values
    rounded through the ``%e`` text of ``writefile`` exactly as the solver will read them."""
    props, pos, vel = [], [], []
    for kind in SHAPES:
        for cub in cuboids:
            if cub.kind != kind:
                continue
            if kind == "cuboid":
                ax = [np.array([_e(v) for v in _axis_values(cub.lower[d], cub.upper[d], cub.space)])
                      for d in range(3)]
                X, Y, Z = np.meshgrid(ax[0], ax[1], ax[2], indexing="ij")
                p = np.stack([X.ravel(), Y.ravel(), Z.ravel()], axis=1)
            else:
                p = np.vectorize(_e, otypes=[np.float64])(_shape_points(cub)).reshape(-1, 3)
            pos.append(p)
            props.append(np.full(p.shape[0], cub.type, dtype=np.int32))
            vel.append(np.tile(np.array([_e(v) for v in cub.velocity]), (p.shape[0], 1)))
    P = np.concatenate(pos) if pos else np.zeros((0, 3))
    return Particles(property=np.concatenate(props) if props else np.zeros(0, np.int32),
                     position=np.ascontiguousarray(P), initial_position=P.copy(),
                     velocity=np.ascontiguousarray(np.concatenate(vel)) if vel else np.zeros((0, 3)))


def jitter(p: Particles, spacing: float, amp: float, dim: int, seed: int = 0) -> Particles:
    """Off-lattice variant of a generated set (parity cases only; the reference generator has no
    such option): every coordinate of the active axes moves by a deterministic offset in
    [-amp, amp) x spacing -- a splitmix64 hash of (seed, particle, axis), no RNG state -- and is
    rounded through the same %e text as the generator's, so the reference reads the exact values.
    Position and InitialPosition stay equal (the grid file carries x twice, generator.cpp:853)."""
    n = p.n
    m = np.uint64(0xFFFFFFFFFFFFFFFF)
    k = (np.arange(n, dtype=np.uint64)[:, None] * np.uint64(3) + np.arange(3, dtype=np.uint64)[None, :]
         + np.uint64(seed) * np.uint64(0x9E3779B97F4A7C15)) & m
    with np.errstate(over="ignore"):
        z = (k + np.uint64(0x9E3779B97F4A7C15)) & m
        z = ((z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)) & m
        z = ((z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)) & m
        z = z ^ (z >> np.uint64(31))
    u = (z >> np.uint64(11)).astype(np.float64) * (1.0 / 9007199254740992.0) * 2.0 - 1.0   # [-1, 1)
    if dim == 2:
        u[:, 2] = 0.0
    x = np.vectorize(_e, otypes=[np.float64])(p.position + amp * spacing * u)
    return Particles(property=p.property.copy(), position=np.ascontiguousarray(x),
                     initial_position=x.copy(), velocity=p.velocity.copy())


def generate_window(cuboids: list[Cuboid], axis: int, lo: float, hi: float, dmin: float, width: float):
    """The particles of ``generate(cuboids)`` whose coordinate along ``axis`` lies in the periodic
    window [lo, hi) of a domain starting at ``dmin`` with ``width``, without building the others
    (slab-local creation, include/mph_gpu.h mph_create_slab).  Returns (Particles, ids, n_glob):
    the original indices of the kept particles (ascending) and the total count.  Cuboid lattices
    are separable, so the window only filters the value list of one axis."""
    span = hi - lo
    if any(c.kind != "cuboid" for c in cuboids):
        # the other shapes are not separable: generate them all and keep the window's particles
        parts = generate(cuboids)
        a = parts.position[:, axis]
        u = a - dmin
        u = u - width * np.floor(u / width) + dmin
        off = (u - lo) - width * np.floor((u - lo) / width)
        idx = np.nonzero(off < span)[0] if span < width else np.arange(parts.n)
        sub = Particles(property=parts.property[idx], position=np.ascontiguousarray(parts.position[idx]),
                        initial_position=np.ascontiguousarray(parts.initial_position[idx]),
                        velocity=np.ascontiguousarray(parts.velocity[idx]))
        return sub, idx.astype(np.int32), parts.n
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
    if any(c.kind != "cuboid" for c in cuboids):
        u = generate(cuboids).position[:, axis] - dmin
        v = u - width * np.floor(u / width) + dmin
        uv, inv = np.unique(v, return_inverse=True)
        return uv, np.bincount(inv).astype(np.int64)
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


# block keywords of each shape (generator.cpp:186-652); every one is required by the generator
_BOID_KEYS = {
    "cuboid": ("Spacing", "Type", "RigidType", "Lower", "Upper", "Velocity", "Enthalpy"),
    "cuboid2": ("Spacing", "Type", "Lower", "Upper", "Velocity", "Enthalpy"),
    "cyboid": ("Spacing", "Type", "RigidType", "Lower", "Upper", "Velocity", "Enthalpy", "Ratio"),
    "cyboid2": ("Spacing", "Type", "Lower", "Upper", "Velocity", "Enthalpy", "Ratio"),
    "recboid": ("Spacing", "Type", "Lower", "Upper", "Velocity", "Enthalpy", "Angle"),
    "recboid2": ("Spacing", "Type", "Lower", "Upper", "Velocity", "Enthalpy", "Angle"),
}
_BOID_START = {"Start" + k[0].upper() + k[1:]: k for k in _BOID_KEYS}


class BoidError(ValueError):
    """A .boid file the reference generator would not read completely (generator.cpp:128-184:
    it stops at the first malformed block and writes the particles read so far)."""


def parse_boid(text: str):
    """``.boid`` parser (generator.cpp:128-652, readfile and read<Shape>): the domain lines and
    every Cuboid/Cuboid2/Cyboid/Cyboid2/Recboid/Recboid2 block, whose keywords are read as a
    token stream up to the block's End keyword.  Where the reference silently stops (a block with
    an unknown keyword or a missing one) or skips (an unknown Start* block), this raises BoidError
    instead of returning a grid with particles missing.  Returns (spacing, lower, upper, blocks)."""
    spacing, lower, upper, cubs = None, None, None, []
    lines = text.splitlines()
    i = 0
    while i < len(lines):
        line = lines[i]
        i += 1
        tok = line.split()
        if not tok or line.startswith("#"):
            continue
        key = tok[0]
        if key == "ParticleDistance":
            spacing = float(tok[1])
        elif key == "LowerDomain":
            lower = tuple(float(t) for t in tok[1:4])
        elif key == "UpperDomain":
            upper = tuple(float(t) for t in tok[1:4])
        elif key in _BOID_START:
            kind = _BOID_START[key]
            end = "End" + key[len("Start"):]
            # the block body is a whitespace token stream (fscanf "%s"), from the next line on
            words = []
            while i < len(lines):
                w = lines[i].split()
                i += 1
                if end in w:
                    words += w[:w.index(end)]
                    break
                words += w
            else:
                raise BoidError("%s without %s" % (key, end))
            vals, k = {}, 0
            n_of = {"Lower": 3, "Upper": 3, "Velocity": 3}
            while k < len(words):
                w = words[k]
                if w not in _BOID_KEYS[kind]:
                    raise BoidError("%s: no such indication %r (generator.cpp)" % (key, w))
                m = n_of.get(w, 1)
                try:
                    v = [float(t) for t in words[k + 1:k + 1 + m]] if w != "Type" and w != "RigidType" \
                        else [int(words[k + 1])]
                except (ValueError, IndexError):
                    raise BoidError("%s: bad value for %s" % (key, w)) from None
                if len(v) != m:
                    raise BoidError("%s: bad value for %s" % (key, w))
                vals[w] = v
                k += 1 + m
            missing = [w for w in _BOID_KEYS[kind] if w not in vals]
            if missing:
                raise BoidError("%s: missing %s (the generator would stop reading here)" % (key, ", ".join(missing)))
            cubs.append(Cuboid(type=vals["Type"][0], lower=tuple(vals["Lower"]), upper=tuple(vals["Upper"]),
                               space=vals["Spacing"][0], velocity=tuple(vals["Velocity"]), kind=kind,
                               ratio=vals.get("Ratio", [0.0])[0], angle=vals.get("Angle", [0.0])[0]))
        elif key.startswith("Start"):
            raise BoidError("unknown block %r (the generator reads %s)" % (key, ", ".join(_BOID_START)))
    return spacing, lower, upper, cubs
