"""particlemethod_fsi_amd -- MI355X-native hot path of Ryo1011gd/ParticleMethod_FSI.

The per-step particle-interaction path of the reference MPH explicit FSI solver (neighbour
search, kernel-weighted density / pressure / surface-tension / viscous sums, total-Lagrangian
elastic stress, symplectic-Euler integration; src/main.cpp:597-686) as hand-written HIP kernels
for gfx950 behind the C ABI of include/mph_gpu.h (libmph_gpu.so).  This package holds the
Python mirror of the reference's driver and file formats.
"""
from . import mphio, cases  # noqa: F401
from .solver import MphSolver, MphError, build, load_library, read_case_files, derive_scalars  # noqa: F401

__all__ = ["MphSolver", "MphError", "build", "load_library", "read_case_files", "derive_scalars",
           "mphio", "cases"]
