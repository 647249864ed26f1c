"""Loading of the golden vectors (tests/golden/*.npz, made by tests/golden/make_golden.py from the
compiled reference) and the comparison helpers shared by the parity tests."""
from __future__ import annotations

import json
import os

import numpy as np

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
CASES = ["dam2d", "gate2d", "bar2d", "box3d", "gate3d", "dam2d_st", "box3d_st", "gate2d_sub",
         "gate3d_sub", "rolling2d", "rolling3d", "movwall2d", "movwall3d", "turek2d", "gate2d_rolling1",
         "hydro2d", "bar2d_ivp", "box3d_jit", "gate3d_jit"]


class Golden:
    def __init__(self, case: str):
        self.case = case
        self.z = np.load(os.path.join(GOLDEN, case + ".npz"), allow_pickle=False)
        self.meta = json.loads(bytes(self.z["meta"]).decode())
        self.prop = self.z["Property"]
        self.solid = (self.prop >= 2) & (self.prop < 4)

    @property
    def steps(self):
        return list(self.meta["steps"])

    def has(self, step: int, field: str) -> bool:
        return "s%d/%s" % (step, field) in self.z.files

    def get(self, step: int, field: str) -> np.ndarray:
        return self.z["s%d/%s" % (step, field)]

    def fields(self, step: int):
        pre = "s%d/" % step
        return [k[len(pre):] for k in self.z.files if k.startswith(pre) and "nbr_" not in k]


SOLID_ROWS = {"DeformGradient", "Strain", "Stress", "Normalizer", "LambdaLames", "MuLames"}


def restrict(g: Golden, field: str, full: np.ndarray) -> np.ndarray:
    """Bring a full-length array into the golden's stored shape (structure rows only, ...)."""
    return full[g.solid] if field in SOLID_ROWS else full


def max_abs_diff(a: np.ndarray, b: np.ndarray) -> float:
    m = ~(np.isnan(a) | np.isnan(b)) if a.dtype.kind == "f" else np.ones(a.shape, bool)
    if not m.any():
        return 0.0
    return float(np.max(np.abs(a[m].astype(np.float64) - b[m].astype(np.float64))))


def bit_equal(a: np.ndarray, b: np.ndarray) -> bool:
    """Exact equality, NaN slots (reference-uninitialised entries) skipped."""
    if a.shape != b.shape:
        return False
    if a.dtype.kind == "f":
        m = ~(np.isnan(a) | np.isnan(b))
        return bool(np.array_equal(a[m], b[m]))
    return bool(np.array_equal(a, b))
