"""Python mirror of the reference driver over the C ABI of ``include/mph_gpu.h``.

``MphSolver`` plays the role of the reference's ``main()`` (src/main.cpp:490-727) for tests,
benchmarks and scripting: construct it from a ``.data``/``.grid`` pair (or an in-memory case),
advance with ``step(k)`` (each step = main.cpp:597-686) and read any per-particle array with
``get(<reference array name>)`` in the reference's layout and original particle order.

All compute runs in libmph_gpu.so (HIP kernels for gfx950).  There is no CPU fallback: if the
library is missing or no HIP device is present the constructor raises.
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

from . import mphio

PKG_DIR = os.path.dirname(os.path.abspath(__file__))
LIB_DIR = os.path.join(PKG_DIR, "lib")
LIB_PATH = os.environ.get("MPH_GPU_LIB") or os.path.join(LIB_DIR, "libmph_gpu.so")   # env: A/B builds
CSRC_DIR = os.path.join(PKG_DIR, "csrc")

# MphField (include/mph_gpu.h) keyed by the reference's array names (main.cpp:102-197)
FIELDS = {
    "Position": (0, 3, np.float64), "InitialPosition": (1, 3, np.float64),
    "Velocity": (2, 3, np.float64), "Force": (3, 3, np.float64),
    "Acceleration": (4, 3, np.float64), "GravityCenter": (5, 3, np.float64),
    "PressureP": (6, 1, np.float64), "PressureA": (7, 1, np.float64),
    "DensityA": (8, 1, np.float64), "VolStrainP": (9, 1, np.float64),
    "DivergenceP": (10, 1, np.float64), "Mass": (11, 1, np.float64), "Kappa": (12, 1, np.float64),
    "Lambda": (13, 1, np.float64), "Mu": (14, 1, np.float64),
    "NeighborCount": (15, 1, np.int32), "InitialStructureNeighborCount": (16, 1, np.int32),
    "Property": (17, 1, np.int32), "DeformGradient": (18, 9, np.float64),
    "Strain": (19, 9, np.float64), "Stress": (20, 9, np.float64),
    "Normalizer": (21, 9, np.float64), "LambdaLames": (22, 1, np.float64),
    "MuLames": (23, 1, np.float64),
    "VirialStressAtParticle": (24, 9, np.float64), "VirialPressureAtParticle": (25, 1, np.float64),
}

STATUS = {0: "MPH_OK", -1: "MPH_ERR_ARG", -2: "MPH_ERR_IO", -3: "MPH_ERR_NEIGHBOR_OVERFLOW",
          -4: "MPH_ERR_DEVICE_OOM", -5: "MPH_ERR_HIP", -6: "MPH_ERR_RCCL", -7: "MPH_ERR_DOMAIN",
          -8: "MPH_ERR_UNSUPPORTED", -9: "MPH_ERR_NONFINITE", -10: "MPH_ERR_TRANSPORT",
          -11: "MPH_ERR_CAPACITY"}

EXPORTED_SYMBOLS = [
    "mph_config_default", "mph_read_data_file", "mph_read_grid_header", "mph_read_grid_particles",
    "mph_write_prof_arrays", "mph_write_vtk_arrays", "mph_create", "mph_step", "mph_synchronize",
    "mph_get", "mph_set", "mph_particle_count", "mph_time", "mph_get_scalars", "mph_write_prof",
    "mph_write_vtk", "mph_last_error", "mph_destroy", "mph_profile_steps", "mph_profile_graphs", "mph_neighbor_stats",
    "mph_dist_unique_id", "mph_create_dist", "mph_owned_count", "mph_derive_scalars",
    "mph_structure_init", "mph_create_dist_host", "mph_owned_ids", "mph_slab_bounds",
    "mph_slab_owner", "mph_dist_selftest", "mph_compute_virial",
    "mph_config_sizeof", "mph_write_vtk_async", "mph_output_wait", "mph_write_grid_binary",
    "mph_write_vtu_arrays", "mph_write_vtu", "mph_velocity_profile_arrays",
    "mph_set_initial_velocity_profile", "mph_dist_info", "mph_create_slab", "mph_slab_window",
    "mph_list_stats", "mph_abi_version", "mph_phase_timing", "mph_phase_times",
    "mph_set_step_batching", "mph_neighbor_rows", "mph_dist_overlap",
]

ABI_VERSION = 4   # MPH_ABI_VERSION of include/mph_gpu.h that these bindings follow

# mph_host_exchange_fn (include/mph_gpu.h): (user, send_l, n, send_r, n, recv_l, n, recv_r, n)
HOST_EXCHANGE_FN = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t,
                                    ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p, ctypes.c_size_t,
                                    ctypes.c_void_p, ctypes.c_size_t)


class MphSlabOptions(ctypes.Structure):
    """include/mph_gpu.h MphSlabOptions."""
    _fields_ = [("rank", ctypes.c_int), ("nranks", ctypes.c_int), ("axis", ctypes.c_int),
                ("unique_id128", ctypes.c_char_p), ("host_fn", HOST_EXCHANGE_FN),
                ("host_user", ctypes.c_void_p), ("n_glob", ctypes.c_int), ("ids", ctypes.c_void_p),
                ("cuts", ctypes.c_void_p)]


class MphError(RuntimeError):
    def __init__(self, code: int, msg: str):
        super().__init__("%s (%d): %s" % (STATUS.get(code, "?"), code, msg))
        self.code = code


def build(verbose: bool = False) -> str:
    """Compile libmph_gpu.so and mph_explicit for gfx950 (hipcc, in-tree)."""
    r = subprocess.run(["make", "-C", CSRC_DIR, "-j8"], capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError("building libmph_gpu.so failed:\n" + r.stdout + r.stderr)
    if verbose:
        print(r.stdout)
    return LIB_PATH


_lib = None


def load_library() -> ctypes.CDLL:
    """Load libmph_gpu.so (fails loudly when it is missing -- there is no fallback path)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise ImportError("libmph_gpu.so not built (run particlemethod_fsi_amd.solver.build())")
    L = ctypes.CDLL(LIB_PATH)
    vp, ip, dp = ctypes.c_void_p, ctypes.c_int, ctypes.c_double
    cfgp = ctypes.POINTER(mphio.MphConfig)
    sig = {
        "mph_config_default": (ip, [cfgp, ip, ip]),
        "mph_read_data_file": (ip, [ctypes.c_char_p, cfgp]),
        "mph_read_grid_header": (ip, [ctypes.c_char_p, cfgp, ctypes.POINTER(ctypes.c_int)]),
        "mph_read_grid_particles": (ip, [ctypes.c_char_p, ip, vp, vp, vp, vp]),
        "mph_write_prof_arrays": (ip, [ctypes.c_char_p, cfgp, dp, ip, vp, vp, vp, vp]),
        "mph_write_vtk_arrays": (ip, [ctypes.c_char_p, ip] + [vp] * 10),
        "mph_create": (ip, [ctypes.POINTER(vp), cfgp, ip, vp, vp, vp, vp, ip]),
        "mph_step": (ip, [vp, ip]),
        "mph_synchronize": (ip, [vp]),
        "mph_get": (ip, [vp, ip, vp]),
        "mph_set": (ip, [vp, ip, vp]),
        "mph_particle_count": (ip, [vp]),
        "mph_time": (dp, [vp]),
        "mph_get_scalars": (ip, [vp, vp]),
        "mph_write_prof": (ip, [vp, ctypes.c_char_p]),
        "mph_write_vtk": (ip, [vp, ctypes.c_char_p]),
        "mph_last_error": (ctypes.c_char_p, [vp]),
        "mph_destroy": (None, [vp]),
        "mph_profile_steps": (ip, [vp, ip, vp, vp, vp]),
        "mph_profile_graphs": (ip, [vp, ip, vp]),
        "mph_neighbor_stats": (ip, [vp, ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_int)]),
        "mph_dist_unique_id": (ip, [vp]),
        "mph_create_dist": (ip, [ctypes.POINTER(vp), cfgp, ip, vp, vp, vp, vp, ip, ip, ip, vp, ip]),
        "mph_owned_count": (ip, [vp]),
        "mph_create_dist_host": (ip, [ctypes.POINTER(vp), cfgp, ip, vp, vp, vp, vp, ip, ip, ip, ip,
                                      HOST_EXCHANGE_FN, vp]),
        "mph_owned_ids": (ip, [vp, vp]),
        "mph_slab_bounds": (ip, [cfgp, ip, ip, ip, vp, vp]),
        "mph_slab_owner": (ip, [cfgp, ip, ip, vp, dp]),
        "mph_dist_selftest": (ip, [ip]),
        "mph_derive_scalars": (ip, [cfgp, vp]),
        "mph_structure_init": (ip, [cfgp, ip, vp, vp, vp, vp, vp, vp]),
        "mph_compute_virial": (ip, [vp]),
        "mph_config_sizeof": (ip, []),
        "mph_abi_version": (ip, []),
        "mph_write_grid_binary": (ip, [ctypes.c_char_p, cfgp, ip, vp, vp, vp, vp]),
        "mph_write_vtk_async": (ip, [vp, ctypes.c_char_p]),
        "mph_write_vtu_arrays": (ip, [ctypes.c_char_p, ip] + [vp] * 10),
        "mph_write_vtu": (ip, [vp, ctypes.c_char_p]),
        "mph_output_wait": (ip, [vp]),
        "mph_velocity_profile_arrays": (ip, [cfgp, dp, ip, vp, vp, vp, vp]),
        "mph_set_initial_velocity_profile": (ip, [vp]),
        "mph_dist_info": (ip, [vp, vp]),
        "mph_list_stats": (ip, [vp, vp, vp]),
        "mph_create_slab": (ip, [ctypes.POINTER(vp), cfgp, ip, vp, vp, vp, vp, ip, ctypes.POINTER(MphSlabOptions)]),
        "mph_slab_window": (ip, [cfgp, ip, ip, ip, vp, vp]),
        "mph_phase_timing": (ip, [vp, ip]),
        "mph_phase_times": (ip, [vp, vp]),
        "mph_set_step_batching": (ip, [vp, ip]),
        "mph_neighbor_rows": (ip, [vp, ip, ip, vp, vp, ctypes.c_longlong]),
        "mph_dist_overlap": (ip, [vp, vp]),
    }
    # entry points an older library may lack (A/B runs against earlier builds)
    optional = {"mph_phase_timing", "mph_phase_times", "mph_set_step_batching", "mph_neighbor_rows",
                "mph_dist_overlap", "mph_profile_graphs", "mph_list_stats"}
    for name, (res, args) in sig.items():
        if name in optional and not hasattr(L, name):
            continue
        f = getattr(L, name)
        f.restype = res
        f.argtypes = args
    # MPH_ABI_ACCEPT=3: an A/B run against a round-5 build (ABI 3 differs only by mph_list_formats,
    # replaced by mph_list_stats in 4; tools/lib_bitwise.py)
    accept = {ABI_VERSION} | {int(v) for v in os.environ.get("MPH_ABI_ACCEPT", "").split(",") if v.strip()}
    if L.mph_abi_version() not in accept:
        raise ImportError("%s has C ABI version %d, these bindings expect %d (rebuild the library)"
                          % (LIB_PATH, L.mph_abi_version(), ABI_VERSION))
    if L.mph_config_sizeof() != ctypes.sizeof(mphio.MphConfig):
        raise ImportError("MphConfig layout mismatch between %s and mphio.MphConfig" % LIB_PATH)
    _lib = L
    return L


def read_case_files(data_path: str, grid_path: str, dim: int, module: str | int = "bar"):
    """readDataFile + readGridFile through the C++ host layer -> (MphConfig, Particles)."""
    L = load_library()
    cfg = mphio.MphConfig()
    mod = mphio.MODULES[module] if isinstance(module, str) else int(module)
    _check(L.mph_config_default(ctypes.byref(cfg), int(dim), mod))
    _check(L.mph_read_data_file(data_path.encode(), ctypes.byref(cfg)))
    n = ctypes.c_int(0)
    _check(L.mph_read_grid_header(grid_path.encode(), ctypes.byref(cfg), ctypes.byref(n)))
    N = n.value
    prop = np.zeros(N, np.int32)
    pos, pos0, vel = (np.zeros((N, 3)) for _ in range(3))
    _check(L.mph_read_grid_particles(grid_path.encode(), N, prop.ctypes.data, pos.ctypes.data,
                                     pos0.ctypes.data, vel.ctypes.data))
    return cfg, mphio.Particles(prop, pos, pos0, vel)


def write_grid_binary(path: str, cfg: mphio.MphConfig, parts: "mphio.Particles"):
    """Binary grid (include/mph_gpu.h mph_write_grid_binary); read_case_files reads it back."""
    p = [np.ascontiguousarray(a, np.float64) for a in (parts.position, parts.initial_position, parts.velocity)]
    prop = np.ascontiguousarray(parts.property, np.int32)
    _check(load_library().mph_write_grid_binary(path.encode(), ctypes.byref(cfg), parts.n, prop.ctypes.data,
                                                p[0].ctypes.data, p[1].ctypes.data, p[2].ctypes.data))


def read_vtu(path: str) -> dict:
    """Arrays of a .vtu written by mph_write_vtu(_arrays): {name: ndarray}, 'Points' for the
    coordinates (raw appended data, UInt64 block headers)."""
    import re
    raw = open(path, "rb").read()
    head, _, data = raw.partition(b'<AppendedData encoding="raw">')
    data = data[data.index(b"_") + 1:]
    dt = {"Float32": np.float32, "Int32": np.int32, "UInt8": np.uint8}
    out = {}
    for m in re.finditer(rb"<DataArray ([^>]*)/>", head):
        attrs = dict(re.findall(rb'(\w+)="([^"]*)"', m.group(1)))
        off = int(attrs[b"offset"])
        nb = int(np.frombuffer(data[off:off + 8], np.uint64)[0])
        a = np.frombuffer(data[off + 8:off + 8 + nb], dt[attrs[b"type"].decode()])
        k = int(attrs.get(b"NumberOfComponents", b"1"))
        out[attrs.get(b"Name", b"Points").decode()] = a.reshape(-1, k) if k > 1 else a
    return out


def derive_scalars(cfg: mphio.MphConfig) -> np.ndarray:
    """Derived constants of initializeWeight/Fluid/Wall/Domain, host only (no device needed)."""
    out = np.zeros(36)
    _check(load_library().mph_derive_scalars(ctypes.byref(cfg), out.ctypes.data))
    return out


def _check(rc, ctx=None):
    if rc < 0:
        msg = ""
        if ctx is not None:
            msg = (load_library().mph_last_error(ctx) or b"").decode()
        raise MphError(rc, msg)
    return rc


def _cuts(cuts, nranks: int):
    """(array kept alive, pointer or None) for MphSlabOptions.cuts / the host helpers."""
    if cuts is None:
        return None, None
    c = np.ascontiguousarray(cuts, np.float64)
    if c.shape != (nranks - 1,):
        raise ValueError("cuts: %d interior boundaries expected for %d slabs" % (nranks - 1, nranks))
    return c, c.ctypes.data


def slab_bounds(cfg: mphio.MphConfig, rank: int, nranks: int, axis: int, cuts=None):
    """(lo, hi, halo) of a rank's slab, as a slab context computes them (host only)."""
    out = np.zeros(3)
    c, p = _cuts(cuts, nranks)
    _check(load_library().mph_slab_bounds(ctypes.byref(cfg), rank, nranks, axis, p, out.ctypes.data))
    return float(out[0]), float(out[1]), float(out[2])


def slab_window(cfg: mphio.MphConfig, rank: int, nranks: int, axis: int, cuts=None):
    """(lo, hi): the periodic window of particles a rank needs for slab-local creation."""
    out = np.zeros(2)
    c, p = _cuts(cuts, nranks)
    _check(load_library().mph_slab_window(ctypes.byref(cfg), rank, nranks, axis, p, out.ctypes.data))
    return float(out[0]), float(out[1])


def slab_owner(cfg: mphio.MphConfig, nranks: int, axis: int, x: float, cuts=None) -> int:
    c, p = _cuts(cuts, nranks)
    return _check(load_library().mph_slab_owner(ctypes.byref(cfg), nranks, axis, p, float(x)))


class Slab:
    """Slab-mode options of MphSolver: this process is `rank` of `nranks`, slabs along `axis`.
    Transport: RCCL with the 128-byte unique id `uid` (mph_create_dist), or a host callback
    `exchange(send_l, send_r, recv_l, recv_r)` over memoryviews (mph_create_dist_host)."""

    def __init__(self, rank: int, nranks: int, axis: int, uid: bytes | None = None, exchange=None,
                 ids: np.ndarray | None = None, n_glob: int = 0, cuts=None):
        """ids/n_glob: slab-local creation -- the particles handed to MphSolver are only this
        rank's window (slab_window), with their original indices ids among n_glob.
        cuts: the nranks - 1 interior slab boundaries (None: equal slabs), the same on every rank
        (dist.balanced_cuts)."""
        if (uid is None) == (exchange is None):
            raise ValueError("Slab needs exactly one of uid (RCCL) or exchange (host transport)")
        self.rank, self.nranks, self.axis, self.uid, self.exchange = rank, nranks, axis, uid, exchange
        self.ids = None if ids is None else np.ascontiguousarray(ids, np.int32)
        self.n_glob = int(n_glob) if ids is not None else 0
        self.cuts = _cuts(cuts, nranks)[0]


def unique_id() -> bytes:
    """A fresh RCCL unique id (rank 0 calls this and shares it with the other ranks)."""
    buf = ctypes.create_string_buffer(128)
    _check(load_library().mph_dist_unique_id(buf))
    return buf.raw


class MphSolver:
    """One MI355X context running the reference hot path (see module docstring).  With
    `slab=Slab(...)` the context is one rank of the multi-GPU slab decomposition: get() then fills
    only the entries of the particles this rank owns (see owned_ids())."""

    def __init__(self, cfg: mphio.MphConfig, parts: mphio.Particles, device: int = 0,
                 slab: Slab | None = None):
        L = load_library()
        self._L = L
        self.cfg = cfg.copy()
        self.n = parts.n
        self.slab = slab
        self._arrays = [np.ascontiguousarray(parts.property, np.int32),
                        np.ascontiguousarray(parts.position, np.float64),
                        np.ascontiguousarray(parts.initial_position, np.float64),
                        np.ascontiguousarray(parts.velocity, np.float64)]
        h = ctypes.c_void_p()
        ptrs = [a.ctypes.data for a in self._arrays]
        if slab is None:
            rc = L.mph_create(ctypes.byref(h), ctypes.byref(self.cfg), self.n, *ptrs, int(device))
        else:
            opt = MphSlabOptions()
            opt.rank, opt.nranks, opt.axis = slab.rank, slab.nranks, slab.axis
            if slab.uid is not None:
                self._uid = ctypes.create_string_buffer(bytes(slab.uid), 128)
                opt.unique_id128 = ctypes.cast(self._uid, ctypes.c_char_p)
            else:
                self._cb = HOST_EXCHANGE_FN(_host_exchange_adapter(slab.exchange))
                opt.host_fn = self._cb
            if slab.ids is not None:
                if len(slab.ids) != parts.n:
                    raise ValueError("Slab.ids must index the particles passed in")
                opt.n_glob = slab.n_glob
                opt.ids = slab.ids.ctypes.data
                self._keep_ids = slab.ids
                self.n = slab.n_glob
            if slab.cuts is not None:
                opt.cuts = slab.cuts.ctypes.data
            rc = L.mph_create_slab(ctypes.byref(h), ctypes.byref(self.cfg), parts.n, *ptrs, int(device),
                                   ctypes.byref(opt))
        if rc < 0:
            msg = (L.mph_last_error(None) or b"").decode()
            raise MphError(rc, msg or "mph_create failed")
        self._h = h

    @classmethod
    def from_files(cls, data_path: str, grid_path: str, dim: int, module="bar", device: int = 0):
        cfg, parts = read_case_files(data_path, grid_path, dim, module)
        return cls(cfg, parts, device)

    # -- lifecycle -------------------------------------------------------------------------
    def close(self):
        if getattr(self, "_h", None) is not None and self._h.value:
            self._L.mph_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    # -- stepping ----------------------------------------------------------------------------
    def step(self, k: int = 1):
        _check(self._L.mph_step(self._h, int(k)), self._h)

    def synchronize(self):
        _check(self._L.mph_synchronize(self._h), self._h)

    @property
    def time(self) -> float:
        return self._L.mph_time(self._h)

    # -- data ----------------------------------------------------------------------------------
    def get(self, name: str) -> np.ndarray:
        fid, w, dt = FIELDS[name]
        shape = (self.n,) if w == 1 else ((self.n, 3) if w == 3 else (self.n, 3, 3))
        out = np.zeros(shape, dt)
        _check(self._L.mph_get(self._h, fid, out.ctypes.data), self._h)
        return out

    def set(self, name: str, values: np.ndarray):
        fid, _, _ = FIELDS[name]
        arr = np.ascontiguousarray(values, np.float64)
        _check(self._L.mph_set(self._h, fid, arr.ctypes.data), self._h)

    def set_initial_velocity_profile(self):
        """setInitialVelocityProfile (main.cpp:395-441) once on the current state: Bar beam mode or
        Turek_Hron inlet, by the configured module (the Turek inlet also runs every step)."""
        _check(self._L.mph_set_initial_velocity_profile(self._h), self._h)

    def scalars(self) -> np.ndarray:
        out = np.zeros(36)
        _check(self._L.mph_get_scalars(self._h, out.ctypes.data), self._h)
        return out

    def write_vtk(self, path: str):
        _check(self._L.mph_write_vtk(self._h, path.encode()), self._h)

    def write_vtu(self, path: str):
        """Binary VTK XML (.vtu) of the same fields as write_vtk (Float32, appended raw data)."""
        _check(self._L.mph_write_vtu(self._h, path.encode()), self._h)

    def write_vtk_async(self, path: str):
        """Snapshot now, format and write in the background (wait with output_wait())."""
        _check(self._L.mph_write_vtk_async(self._h, path.encode()), self._h)

    def output_wait(self):
        _check(self._L.mph_output_wait(self._h), self._h)

    def write_prof(self, path: str):
        _check(self._L.mph_write_prof(self._h, path.encode()), self._h)

    # -- measurement ----------------------------------------------------------------------------
    def profile(self, nsteps: int) -> dict:
        """Per-kernel average duration (ms) over nsteps, HIP events around every launch."""
        avg = np.zeros(24)
        cnt = np.zeros(24, np.int32)
        names = ctypes.create_string_buffer(24 * 32)
        k = _check(self._L.mph_profile_steps(self._h, int(nsteps), avg.ctypes.data, cnt.ctypes.data,
                                             ctypes.addressof(names)), self._h)
        raw = names.raw
        out = {}
        for i in range(k):
            nm = raw[32 * i:32 * (i + 1)].split(b"\0", 1)[0].decode()
            out[nm] = {"avg_ms": float(avg[i]), "launches": int(cnt[i])}
        return out

    def profile_graphs(self, reps: int = 16) -> dict:
        """The list kernels timed as graph replays (mph_profile_graphs): ms per launch of the search
        (with the XCD split), pass A and pass B; None where not measured."""
        out = np.zeros(3)
        _check(self._L.mph_profile_graphs(self._h, int(reps), out.ctypes.data), self._h)
        return {k: (float(v) if v >= 0 else None) for k, v in zip(("neighbors", "pass_a", "pass_b"), out)}

    def step_batching(self, on: bool = True):
        """mph_set_step_batching: step(1) per time-loop iteration costs what step(8) does; pending
        steps run (and their errors surface) at the next synchronize/get/write."""
        _check(self._L.mph_set_step_batching(self._h, 1 if on else 0), self._h)

    def phase_timing(self, on: bool = True):
        """Time the reference's clock() buckets (main.cpp:695-700) with HIP events at every step's
        phase boundaries; read the sums with phase_times().  While on, mph_step launches the steps'
        kernels directly instead of replaying the captured graphs (HIP cannot time events inside a
        graph) and waits for the events after every batch of up to 8 steps, so it is slower."""
        _check(self._L.mph_phase_timing(self._h, 1 if on else 0), self._h)

    def phase_times(self) -> dict:
        """Accumulated GPU milliseconds: neighbour search (sort + search), explicit calculation
        (sums, integration, elastic substeps), virial."""
        a = np.zeros(3)
        _check(self._L.mph_phase_times(self._h, a.ctypes.data), self._h)
        return {"neighbor_ms": float(a[0]), "explicit_ms": float(a[1]), "virial_ms": float(a[2])}

    def owned_ids(self) -> np.ndarray:
        """Original indices of the particles this context owns (all of them without a slab)."""
        k = self._L.mph_owned_count(self._h)
        out = np.zeros(max(self.n, 1), np.int32)
        _check(self._L.mph_owned_ids(self._h, out.ctypes.data), self._h)
        return out[:k].copy()

    def list_stats(self):
        """(mean, max) length of the stored neighbour lists of the last search (mph_list_stats: the
        pairs the passes walk; every neighbour with MPH_LIST_FULL=1)."""
        m = ctypes.c_double()
        x = ctypes.c_int()
        _check(self._L.mph_list_stats(self._h, ctypes.byref(m), ctypes.byref(x)), self._h)
        return m.value, x.value

    def neighbor_rows(self, first: int = 0, count: int | None = None):
        """(counts, offsets, ids): the neighbour sets of the particles [first, first + count) from
        the last search (mph_neighbor_rows; calculateNeighbor's Neighbor[i][k], main.cpp:1764-1772),
        each row as ascending original indices, row k = ids[offsets[k]:offsets[k + 1]]."""
        if count is None:
            count = self.n - first
        counts = np.zeros(count, np.int32)
        cap = max(1, count * 128)
        while True:
            ids = np.zeros(cap, np.int32)
            r = self._L.mph_neighbor_rows(self._h, int(first), int(count), counts.ctypes.data, ids.ctypes.data, cap)
            need = int(np.minimum(counts, 512).sum()) if r == -1 else 0
            if r == -1 and need > cap:
                cap = need
                continue
            _check(r, self._h)
            break
        offsets = np.concatenate([[0], np.cumsum(np.minimum(counts, 512))]).astype(np.int64)
        return counts, offsets, ids[:r].copy()

    def dist_info(self) -> dict:
        """Slab-mode facts (mph_dist_info): slab ranks, RCCL communicator size (0: host-staged),
        graph replay, capacities."""
        a = np.zeros(8, np.int32)
        _check(self._L.mph_dist_info(self._h, a.ctypes.data), self._h)
        keys = ["nranks", "rank", "rccl_ranks", "graphs", "cap", "cap_send", "cap_recv", "held"]
        return {k: int(v) for k, v in zip(keys, a)}

    def dist_overlap(self) -> dict:
        """Pass-B mode of a slab context (mph_dist_overlap): overlap on/off, whether MPH_SLAB_OVERLAP
        forced it or the creation probe chose it, and the probe's maxima over ranks (ms)."""
        a = np.zeros(5)
        _check(self._L.mph_dist_overlap(self._h, a.ctypes.data), self._h)
        return {"overlap": bool(a[0] == 1.0), "chosen_by": {-1: "probe", 0: "forced", 1: "forced"}.get(int(a[1]), "none"),
                "halo_exchange_ms": float(a[2]), "redistribution_exchange_ms": float(a[3]),
                "split_pass_b_cost_ms": float(a[4])}

    def compute_virial(self):
        """calculateVirialStressAtParticle (main.cpp:3077-3318) on the current state; read the result
        with get("VirialStressAtParticle") / get("VirialPressureAtParticle")."""
        _check(self._L.mph_compute_virial(self._h), self._h)

    def neighbor_stats(self):
        m = ctypes.c_double()
        x = ctypes.c_int()
        _check(self._L.mph_neighbor_stats(self._h, ctypes.byref(m), ctypes.byref(x)), self._h)
        return m.value, x.value


def _host_exchange_adapter(fn):
    """Wrap a Python exchange(send_l, send_r, recv_l, recv_r) over writable memoryviews as an
    mph_host_exchange_fn; exceptions become a nonzero return (MPH_ERR_TRANSPORT)."""
    def view(ptr, n):
        if not n:
            return memoryview(bytearray(0))
        return memoryview((ctypes.c_uint8 * n).from_address(ptr)).cast("B")

    def cb(user, sl, nsl, sr, nsr, rl, nrl, rr, nrr):
        try:
            fn(view(sl, nsl), view(sr, nsr), view(rl, nrl), view(rr, nrr))
            return 0
        except Exception as e:  # reported through the status code
            import sys
            print("mph host exchange failed: %r" % (e,), file=sys.stderr)
            return 1
    return cb
