#!/usr/bin/env python3
"""Wavefront census of one D16M z-slab rank (no GPU): the rank's held particles (owned + the
ghosts within one halo of its faces, generated for its window like bench.py --gpus 8), sorted in
the slab order (y, z, x) on cells of rc/3 (y, z) and rc/2 (x), cut into wavefronts of 64 -- how
many are all-ghost (skipped by the list kernels), mixed, or fully owned.

usage: python tools/slab_waves.py [rank] [nranks]     
"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from particlemethod_fsi_amd import cases, solver  # noqa: E402
from particlemethod_fsi_amd.dist import balanced_cuts, build_local  # noqa: E402


def main():
    r = int(sys.argv[1]) if len(sys.argv) > 1 else 5
    nr = int(sys.argv[2]) if len(sys.argv) > 2 else 8
    case, axis = cases.get("d16m"), 2
    cuts = balanced_cuts(case, nr, axis)
    cfg, parts, _, _ = build_local(case, r, nr, axis, cuts)
    lo, hi, _ = solver.slab_bounds(cfg, r, nr, axis, cuts)
    rc = 2.6 * case.spacing
    pos = parts.position
    z = pos[:, 2]
    own = (z >= lo) & (z < hi)
    held = own | ((z >= lo - rc) & (z < lo)) | ((z >= hi) & (z < hi + rc))
    p, o = pos[held], own[held]
    cy = np.floor(p[:, 1] / (rc / 3)).astype(np.int64)
    cz = np.floor((p[:, 2] - lo + 2 * rc) / (rc / 3)).astype(np.int64)
    cx = np.floor((p[:, 0] - cfg.domain_min[0]) / (rc / 2)).astype(np.int64)
    o = o[np.argsort((cy * 4096 + cz) * 4096 + cx, kind="stable")]
    nw = (len(o) + 63) // 64
    w = np.zeros(nw * 64, bool)
    w[:len(o)] = o
    cnt = w.reshape(nw, 64).sum(1)
    mixed = (cnt > 0) & (cnt < 64)
    print({"rank": r, "held": int(len(o)), "owned": int(o.sum()), "waves": int(nw),
           "all_ghost": int((cnt == 0).sum()), "mixed": int(mixed.sum()), "full": int((cnt == 64).sum()),
           "ghost_lanes_in_mixed": int((64 - cnt[mixed]).sum())})


if __name__ == "__main__":
    main()
