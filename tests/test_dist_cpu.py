"""CPU tests of the multi-GPU slab decomposition (no device): slab geometry of the library's
host functions, and world-size 2/3 gloo runs of the neighbour exchange routing and of the
halo-band rule (every reference neighbour of an owned particle is owned or a received ghost)."""
import multiprocessing as mp
import os
import socket

import numpy as np
import pytest

from particlemethod_fsi_amd import cases, solver

import dist_worker


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _spawn(target, world, *args):
    ctx = mp.get_context("spawn")
    port = _free_port()
    ps = [ctx.Process(target=target, args=(r, world, port) + args) for r in range(world)]
    for p in ps:
        p.start()
    for p in ps:
        p.join(180)
    for p in ps:
        if p.is_alive():
            p.kill()
    assert all(p.exitcode == 0 for p in ps), [p.exitcode for p in ps]


@pytest.mark.parametrize("case,axis", [("channel3d", 2), ("d1m", 2), ("dam2d", 0)])
@pytest.mark.parametrize("nranks", [2, 3, 5])
def test_slab_bounds_partition_domain(case, axis, nranks):
    cfg, parts = cases.get(case).build()
    b = [solver.slab_bounds(cfg, r, nranks, axis) for r in range(nranks)]
    assert b[0][0] == cfg.domain_min[axis]
    assert b[-1][1] == cfg.domain_max[axis]
    for r in range(nranks - 1):
        assert b[r][1] == b[r + 1][0]          # same expression -> no gap, no overlap
    h = b[0][2]
    assert h > 0 and all(x[2] == h for x in b)
    # every particle has exactly one owner, the one whose [lo, hi) holds it
    xs = parts.position[:: max(1, parts.n // 4000), axis]
    for x in xs:
        r = solver.slab_owner(cfg, nranks, axis, x)
        assert b[r][0] <= x < b[r][1] or (r == nranks - 1 and x >= b[r][0]) or (r == 0 and x < b[0][1])


def test_slab_halo_covers_cutoff():
    cfg, _ = cases.get("d1m").build()
    lo, hi, h = solver.slab_bounds(cfg, 0, 2, 2)
    scal = solver.derive_scalars(cfg)
    # halo = (MaxRadius + MARGIN) * (1 + 1e-6) >= the acceptance radius of calculateNeighbor
    assert h >= 2.5 * cfg.particle_spacing


@pytest.mark.parametrize("world", [2, 3])
def test_gloo_exchange_routing(tmp_path, world):
    out = str(tmp_path / "flags.npy")
    _spawn(dist_worker.exchange_worker, world, out)
    assert np.load(out).all()


@pytest.mark.parametrize("world", [2, 3, 4])
def test_halo_band_contains_all_neighbours(tmp_path, world):
    out = str(tmp_path / "band.npy")
    _spawn(dist_worker.band_worker, world, "dam2d", out)
    res = np.load(out)
    n = cases.get("dam2d").build()[1].n
    assert res[:, 0].sum() == n             # ownership is a partition
    assert (res[:, 1] == 0).all(), res       # no owned particle misses a neighbour
    assert (res[:, 2] > 0).all()             # dam2d's fluid spans the slab faces


@pytest.mark.parametrize("case,nranks", [("d16m", 8), ("d16m", 2), ("d1m", 4), ("dam2d", 3)])
def test_balanced_cuts_equalise_shares(case, nranks):
    """dist.balanced_cuts (bench.py's slab boundaries): the cuts ascend inside the domain, the
    library's bounds/owner functions follow them, the initial particles split into shares within
    two lattice planes of equal, and the largest cost owned + GHOST_WEIGHT x ghosts is no larger
    than with the count quantiles (ghost_weight=0), which it improves at D16M / 8."""
    from particlemethod_fsi_amd import mphio
    from particlemethod_fsi_amd.dist import balanced_cuts
    c = cases.get(case)
    axis = 2 if c.dim == 3 else 0
    cfg, _ = c._config()
    cuts = balanced_cuts(c, nranks, axis)
    assert cuts.shape == (nranks - 1,) and np.all(np.diff(cuts) > 0)
    b = [solver.slab_bounds(cfg, r, nranks, axis, cuts) for r in range(nranks)]
    assert b[0][0] == cfg.domain_min[axis] and b[-1][1] == cfg.domain_max[axis]
    for r in range(nranks - 1):
        assert b[r][1] == b[r + 1][0] == cuts[r]
    dmin = cfg.domain_min[axis]
    v, n = mphio.plane_counts(c.cuboids, axis, dmin, cfg.domain_max[axis] - dmin)
    owner = np.array([solver.slab_owner(cfg, nranks, axis, x, cuts) for x in v])
    share = np.bincount(owner, weights=n, minlength=nranks)
    assert share.sum() == n.sum()
    assert share.max() - share.min() <= 2 * n.max(), share
    # equal slabs are the cuts=None default
    assert solver.slab_bounds(cfg, 1, nranks, axis) == solver.slab_bounds(cfg, 1, nranks, axis, None)
    from particlemethod_fsi_amd.dist import GHOST_WEIGHT
    halo = b[0][2]

    def max_cost(cs):
        e = np.concatenate([[dmin], cs, [cfg.domain_max[axis]]])
        own = [n[(v >= e[r]) & (v < e[r + 1])].sum() for r in range(nranks)]
        gh = [n[((v >= e[r] - halo) & (v < e[r])) | ((v >= e[r + 1]) & (v < e[r + 1] + halo))].sum()
              for r in range(nranks)]
        return max(o + GHOST_WEIGHT * g for o, g in zip(own, gh))

    quant = balanced_cuts(c, nranks, axis, ghost_weight=0.0)
    assert max_cost(cuts) <= max_cost(quant)
    if (case, nranks) == ("d16m", 8):
        assert max_cost(cuts) < 0.98 * max_cost(quant)


def test_bad_cuts_rejected():
    cfg, _ = cases.get("d1m").build()
    with pytest.raises(solver.MphError):
        solver.slab_bounds(cfg, 0, 3, 2, [0.05, 0.02])        # not ascending
    with pytest.raises(solver.MphError):
        solver.slab_owner(cfg, 2, 2, 0.0, [cfg.domain_max[2] + 1.0])   # outside the domain
    with pytest.raises(ValueError):
        solver.slab_window(cfg, 0, 3, 2, [0.05])              # wrong length
