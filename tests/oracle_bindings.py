"""ctypes bindings for the TEST INFRASTRUCTURE libraries under oracle/.

* ``RefSolver``    -- oracle/_ref/libmphref_<dim>_<module>.so: the reference solver compiled from
                      /root/reference by oracle/Makefile (only where it was built).
* ``OracleSolver`` -- oracle/_build/libmph_oracle.so: the clean-room CPU restatement.

Both expose the same tiny interface (``init``, ``step``, ``call``, ``get``, ``neighbors``,
``scalars``) so that tests read like the reference's own driver.  Only tests/, smoke() and
bench.py's cpu_baseline may use this module.
"""
from __future__ import annotations

import ctypes
import os
import subprocess
import tempfile

import numpy as np

from particlemethod_fsi_amd import mphio

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ORACLE_DIR = os.path.join(ROOT, "oracle")
# MPH_ORACLE_LIB: an alternative build of the same source (the 128-entry rows of oracle128)
ORACLE_LIB = os.environ.get("MPH_ORACLE_LIB") or os.path.join(ORACLE_DIR, "_build", "libmph_oracle.so")
REF_DIR = os.path.join(ORACLE_DIR, "_ref")

VEC3 = {"Position", "InitialPosition", "Velocity", "Force", "Acceleration", "GravityCenter"}
MAT3 = {"DeformGradient", "Strain", "Stress", "Normalizer", "VirialStressAtParticle"}
INTS = {"NeighborCount", "InitialStructureNeighborCount", "Property"}
SCALARS = {"PressureP", "PressureA", "DensityA", "VolStrainP", "DivergenceP", "Mass", "Kappa",
           "Lambda", "Mu", "LambdaLames", "MuLames", "VirialPressureAtParticle"}
# the virial diagnostic (main.cpp:3077-3318) is only defined after calculateVirialStressAtParticle
VIRIAL = {"VirialStressAtParticle", "VirialPressureAtParticle"}
ALL_FIELDS = sorted((VEC3 | MAT3 | INTS | SCALARS) - VIRIAL)


def build_oracle() -> str:
    if not os.path.exists(ORACLE_LIB):
        subprocess.run(["make", "-C", ORACLE_DIR, "oracle"], check=True, capture_output=True)
    return ORACLE_LIB


def ref_lib_path(dim: int, module: str) -> str:
    return os.path.join(REF_DIR, "libmphref_%dd_%s.so" % (dim, module))


def ref_available(dim: int = 2, module: str = "bar") -> bool:
    return os.path.exists(ref_lib_path(dim, module))


def _alloc(name: str, n: int) -> np.ndarray:
    if name in VEC3:
        return np.zeros((n, 3), np.float64)
    if name in MAT3:
        return np.zeros((n, 3, 3), np.float64)
    if name in INTS:
        return np.zeros(n, np.int32)
    return np.zeros(n, np.float64)


class RefSolver:
    """The reference solver (one instance per process per variant: it uses file-scope globals)."""

    def __init__(self, dim: int, module: str, data_path: str, grid_path: str):
        self.lib = ctypes.CDLL(ref_lib_path(dim, module), mode=ctypes.RTLD_LOCAL)
        L = self.lib
        L.ref_load.argtypes = [ctypes.c_char_p] * 3
        L.ref_get.argtypes = [ctypes.c_char_p, ctypes.c_void_p]
        L.ref_neighbors.argtypes = [ctypes.c_int, ctypes.c_void_p]
        L.ref_structure_neighbors.argtypes = [ctypes.c_int, ctypes.c_void_p]
        L.ref_scalars.argtypes = [ctypes.c_void_p]
        L.ref_call.argtypes = [ctypes.c_char_p]
        L.ref_time.restype = ctypes.c_double
        L.ref_write_vtk.argtypes = [ctypes.c_char_p]
        L.ref_write_prof.argtypes = [ctypes.c_char_p]
        self.n = L.ref_load(data_path.encode(), grid_path.encode(), os.devnull.encode())

    def init(self):
        self.lib.ref_init()

    def step(self, k: int = 1):
        self.lib.ref_steps(int(k))

    def call(self, name: str):
        assert self.lib.ref_call(name.encode()) == 0, name

    def get(self, name: str) -> np.ndarray:
        out = _alloc(name, self.n)
        assert self.lib.ref_get(name.encode(), out.ctypes.data) > 0, name
        return out

    def neighbors(self, i: int) -> np.ndarray:
        buf = np.zeros(512, np.int32)
        c = self.lib.ref_neighbors(int(i), buf.ctypes.data)
        return buf[:min(c, 512)].copy()

    def scalars(self) -> np.ndarray:
        out = np.zeros(36)
        self.lib.ref_scalars(out.ctypes.data)
        return out

    @property
    def time(self) -> float:
        return self.lib.ref_time()

    def write_vtk(self, path: str):
        self.lib.ref_write_vtk(path.encode())

    def write_prof(self, path: str):
        self.lib.ref_write_prof(path.encode())


class OracleSolver:
    """The CPU restatement (oracle/mph_oracle.c)."""

    _lib = None

    @classmethod
    def lib(cls):
        if cls._lib is None:
            L = ctypes.CDLL(build_oracle())
            L.orc_create.restype = ctypes.c_void_p
            L.orc_create.argtypes = [ctypes.POINTER(mphio.MphConfig), ctypes.c_int] + [ctypes.c_void_p] * 4
            L.orc_destroy.argtypes = [ctypes.c_void_p]
            L.orc_init.argtypes = [ctypes.c_void_p]
            L.orc_step.argtypes = [ctypes.c_void_p, ctypes.c_int]
            L.orc_call.argtypes = [ctypes.c_void_p, ctypes.c_char_p]
            L.orc_get.argtypes = [ctypes.c_void_p, ctypes.c_char_p, ctypes.c_void_p]
            L.orc_neighbors.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p]
            L.orc_scalars.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
            L.orc_time.argtypes = [ctypes.c_void_p]
            L.orc_time.restype = ctypes.c_double
            L.orc_set_threads.argtypes = [ctypes.c_int]
            cls._lib = L
        return cls._lib

    def __init__(self, cfg: mphio.MphConfig, parts: mphio.Particles):
        L = self.lib()
        self.cfg = cfg.copy()
        self.n = parts.n
        self._keep = [np.ascontiguousarray(parts.property, np.int32),
                      np.ascontiguousarray(parts.position, np.float64),
                      np.ascontiguousarray(parts.initial_position, np.float64),
                      np.ascontiguousarray(parts.velocity, np.float64)]
        self.h = L.orc_create(ctypes.byref(self.cfg), self.n, *[a.ctypes.data for a in self._keep])

    def __del__(self):
        if getattr(self, "h", None) and self._lib is not None:
            self._lib.orc_destroy(self.h)
            self.h = None

    @staticmethod
    def set_threads(n: int):
        OracleSolver.lib().orc_set_threads(int(n))

    def init(self):
        self._lib.orc_init(self.h)

    def step(self, k: int = 1):
        self._lib.orc_step(self.h, int(k))

    def call(self, name: str):
        assert self._lib.orc_call(self.h, name.encode()) == 0, name

    def get(self, name: str) -> np.ndarray:
        out = _alloc(name, self.n)
        assert self._lib.orc_get(self.h, name.encode(), out.ctypes.data) > 0, name
        return out

    def neighbors(self, i: int) -> np.ndarray:
        buf = np.zeros(512, np.int32)
        c = self._lib.orc_neighbors(self.h, int(i), buf.ctypes.data)
        return buf[:min(c, 512)].copy()

    def scalars(self) -> np.ndarray:
        out = np.zeros(36)
        self._lib.orc_scalars(self.h, out.ctypes.data)
        return out

    @property
    def time(self) -> float:
        return self._lib.orc_time(self.h)


def write_case_files(cfg_text: str, grid_text: str, tmpdir: str | None = None):
    d = tmpdir or tempfile.mkdtemp(prefix="mphcase_")
    dp, gp = os.path.join(d, "case.data"), os.path.join(d, "case.grid")
    with open(dp, "w") as fh:
        fh.write(cfg_text)
    with open(gp, "w") as fh:
        fh.write(grid_text)
    return dp, gp
