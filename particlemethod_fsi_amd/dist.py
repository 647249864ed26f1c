"""Multi-process glue for the slab decomposition (include/mph_gpu.h, csrc/mph_dist.hip).

One process per GPU, launched by torchrun / torch.multiprocessing; `torch.distributed` is the
control plane only (rendezvous, the RCCL unique id, result gathering).  The particle data path
between neighbouring slabs is the library's own: RCCL ncclSend/ncclRecv on the context's stream
(`rccl_slab`), or -- to run several ranks on one GPU, or without RCCL -- the host-staged
transport driven by `GlooExchange` over a gloo process group.
"""
from __future__ import annotations

import numpy as np

from . import mphio, solver


class GlooExchange:
    """mph_host_exchange_fn over torch.distributed point-to-point (gloo, CPU tensors).

    send_l goes to the left neighbour, which receives it as its recv_r; send_r goes right
    (received as recv_l).  Tags keep the two directions apart when left == right (2 ranks)."""

    TAG_LEFTWARD = 17
    TAG_RIGHTWARD = 23

    def __init__(self, rank: int, nranks: int, group=None, delay_ms: float | None = None):
        self.rank, self.nranks, self.group = rank, nranks, group
        self.left = (rank - 1) % nranks
        self.right = (rank + 1) % nranks
        # diagnostics / tests of the overlap probe: every exchange takes this much longer
        # (MPH_HOST_EXCHANGE_DELAY_MS), as over a slow link
        if delay_ms is None:
            import os
            delay_ms = float(os.environ.get("MPH_HOST_EXCHANGE_DELAY_MS", "0"))
        self.delay_s = delay_ms * 1e-3

    def __call__(self, send_l, send_r, recv_l, recv_r):
        import torch
        import torch.distributed as dist
        if self.delay_s > 0:
            import time
            time.sleep(self.delay_s)

        def t(mv):
            return torch.from_numpy(np.frombuffer(mv, dtype=np.uint8))

        reqs = []
        if len(send_l):
            reqs.append(dist.isend(t(send_l), self.left, group=self.group, tag=self.TAG_LEFTWARD))
        if len(send_r):
            reqs.append(dist.isend(t(send_r), self.right, group=self.group, tag=self.TAG_RIGHTWARD))
        bufs = []
        if len(recv_r):
            b = torch.empty(len(recv_r), dtype=torch.uint8)
            reqs.append(dist.irecv(b, self.right, group=self.group, tag=self.TAG_LEFTWARD))
            bufs.append((b, recv_r))
        if len(recv_l):
            b = torch.empty(len(recv_l), dtype=torch.uint8)
            reqs.append(dist.irecv(b, self.left, group=self.group, tag=self.TAG_RIGHTWARD))
            bufs.append((b, recv_l))
        for r in reqs:
            r.wait()
        for b, mv in bufs:
            np.frombuffer(mv, dtype=np.uint8)[:] = b.numpy()


def rccl_slab(rank: int, nranks: int, axis: int, group=None, ids=None, n_glob: int = 0, cuts=None) -> solver.Slab:
    """Slab options with an RCCL communicator: rank 0 makes the unique id, everyone receives it
    through torch.distributed (any backend)."""
    import torch.distributed as dist
    obj = [solver.unique_id() if rank == 0 else None]
    dist.broadcast_object_list(obj, src=0, group=group)
    return solver.Slab(rank, nranks, axis, uid=obj[0], ids=ids, n_glob=n_glob, cuts=cuts)


def gloo_slab(rank: int, nranks: int, axis: int, group=None, ids=None, n_glob: int = 0, cuts=None) -> solver.Slab:
    return solver.Slab(rank, nranks, axis, exchange=GlooExchange(rank, nranks, group), ids=ids, n_glob=n_glob,
                       cuts=cuts)


# Relative GPU cost of a ghost particle against an owned one: the per-rank GPU times of D16M in 8
# slabs, one rank at a time (tools/slab_serial.py, profiles/r03/slab/), fit t = a owned + b ghosts
# with a ~0.83 and b ~0.6 ms per million (ghosts are sorted, packed, exchanged and unpacked, and
# their mixed waves run the list loops, but they compute no sums of their own).
GHOST_WEIGHT = 0.7


def balanced_cuts(case, nranks: int, axis: int, ghost_weight: float | None = None) -> np.ndarray:
    """Interior slab boundaries (MphSlabOptions.cuts) that balance the ranks' GPU work: the largest
    per-rank cost  owned + ghost_weight x ghosts  is minimised over cuts halfway between the case's
    lattice planes along `axis` (mphio.plane_counts; ghosts: the planes within one halo of an
    interior face, periodic).  ghost_weight 0 (or MPH_SLAB_GHOST_WEIGHT=0): equal shares of the
    initial particles, the count quantiles.  Deterministic, so every rank computes the same array."""
    import os
    cfg, _ = case._config()
    dmin = cfg.domain_min[axis]
    W = cfg.domain_max[axis] - dmin
    v, c = mphio.plane_counts(case.cuboids, axis, dmin, W)
    cum = np.cumsum(c)
    total = int(cum[-1]) if len(cum) else 0
    cuts = []
    for k in range(1, nranks):
        p = int(np.searchsorted(cum, total * k / nranks))   # first plane reaching the quantile
        p = min(p, len(v) - 2)
        cuts.append(0.5 * (v[p] + v[p + 1]))
    cuts = np.array(cuts, np.float64)
    if ghost_weight is None:
        ghost_weight = float(os.environ.get("MPH_SLAB_GHOST_WEIGHT", GHOST_WEIGHT))
    if ghost_weight <= 0.0 or nranks < 2 or len(v) < 2:
        return cuts
    halo = solver.slab_bounds(cfg, 0, nranks, axis, cuts)[2]
    min_width = 2.0 * halo + 2.0 * cfg.particle_spacing   # the slab context's own lower bound
    csum = np.concatenate([[0], cum])

    def count(a, b):   # particles on the planes in [a, b), periodic, b - a <= W
        a0 = dmin + (a - dmin) % W
        b0 = a0 + (b - a)
        n = csum[np.searchsorted(v, min(b0, dmin + W), "left")] - csum[np.searchsorted(v, a0, "left")]
        if b0 > dmin + W:
            n += csum[np.searchsorted(v, b0 - W, "left")]
        return int(n)

    def cost(lo, hi):
        return count(lo, hi) + ghost_weight * (count(lo - halo, lo) + count(hi, hi + halo))

    mids = 0.5 * (v[:-1] + v[1:])

    def place(T):   # greedy: each slab as wide as the bound allows (leaving room for the rest)
        out, lo, k = [], dmin, 0
        for r in range(nranks - 1):
            best = None
            room = dmin + W - (nranks - 1 - r) * min_width
            while k < len(mids) and mids[k] <= room and cost(lo, mids[k]) <= T:
                if mids[k] - lo >= min_width:
                    best = k
                k += 1
            if best is None:
                return None
            out.append(mids[best])
            lo = mids[best]
            k = best + 1
        if dmin + W - lo < min_width or cost(lo, dmin + W) > T:
            return None
        return out

    # bisection below the quantile cuts' largest cost (the greedy's feasibility is monotone near
    # the optimum, not for bounds so loose that the room left for the last slabs decides)
    edges = np.concatenate([[dmin], cuts, [dmin + W]])
    lo_t = 0.0
    hi_t = max(cost(edges[r], edges[r + 1]) for r in range(nranks))
    best = None
    for _ in range(60):
        mid = 0.5 * (lo_t + hi_t)
        got = place(mid)
        if got is None:
            lo_t = mid
        else:
            hi_t, best = mid, got
    return np.array(best, np.float64) if best is not None else cuts


def build_local(case, rank: int, nranks: int, axis: int, cuts=None):
    """This rank's share of a registered case for slab-local creation: (cfg, particles of its
    window, their original indices, total count) -- generated without the rest of the problem.
    cuts: the slab boundaries the contexts will use (None: equal slabs)."""
    cfg, _ = case._config()
    lo, hi = solver.slab_window(cfg, rank, nranks, axis, cuts)
    return case.build_window(axis, lo, hi)


def gather_field(s: solver.MphSolver, name: str, group=None) -> np.ndarray:
    """Merge a field over all ranks (owned entries of each) into the full original-order array,
    returned on every rank."""
    import torch.distributed as dist
    mine_ids = s.owned_ids()
    vals = s.get(name)[mine_ids]
    parts = [None] * dist.get_world_size(group)
    dist.all_gather_object(parts, (mine_ids, vals), group=group)
    fid, w, dt = solver.FIELDS[name]
    shape = (s.n,) if w == 1 else ((s.n, 3) if w == 3 else (s.n, 3, 3))
    out = np.zeros(shape, dt)
    seen = np.zeros(s.n, np.int32)
    for ids, v in parts:
        out[ids] = v
        seen[ids] += 1
    if not np.all(seen == 1):
        raise RuntimeError("slab ownership is not a partition: %d missing, %d duplicated"
                           % (int((seen == 0).sum()), int((seen > 1).sum())))
    return out
