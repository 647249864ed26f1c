"""Worker processes of the slab-decomposition tests (tests/test_dist_cpu.py, test_gpu_dist.py).

Each worker is one rank: it joins a gloo process group on 127.0.0.1 and either runs a GPU slab
context (host-staged transport over gloo, several ranks sharing one GPU) or, on CPU, exercises
the exchange routing and the halo-band rule of the decomposition.
"""
from __future__ import annotations

import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

SLAB_AXIS = {"channel3d": 2, "channel3d_st": 2, "channel2d": 0, "dam2d": 0, "box3d": 0,
             "bar2d": 0, "bar3d": 0, "gate2d_sub": 0}


def _init(rank, world, port):
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    return dist


def make_cuts(c, world, axis, mode):
    """Slab boundaries of a test run: None (equal slabs), "balanced" (dist.balanced_cuts, as
    bench.py) or "skew" (equal cuts moved alternately by a tenth of a slab width)."""
    if mode is None:
        return None
    from particlemethod_fsi_amd.dist import balanced_cuts
    if mode == "balanced":
        return balanced_cuts(c, world, axis)
    cfg, _ = c._config()
    dmin, W = cfg.domain_min[axis], cfg.domain_max[axis] - cfg.domain_min[axis]
    return np.array([dmin + W * k / world + (0.1 if k % 2 else -0.1) * W / world for k in range(1, world)])


def gpu_worker(rank, world, port, case, checkpoints, fields, out_path, local=False, cuts_mode=None):
    """Run `case` as rank `rank` of `world` on cuda:0; at every checkpoint (cumulative step
    count) gather `fields` over the ranks; rank 0 saves them to out_path (.npz).  local: the rank
    is created from its own window of the case only (slab-local creation); cuts_mode: make_cuts."""
    dist = _init(rank, world, port)
    from particlemethod_fsi_amd import MphSolver, cases
    from particlemethod_fsi_amd.dist import build_local, gather_field, gloo_slab
    c = cases.get(case)
    axis = SLAB_AXIS[case]
    cuts = make_cuts(c, world, axis, cuts_mode)
    if local:
        cfg, parts, ids, n_glob = build_local(c, rank, world, axis, cuts)
        slab = gloo_slab(rank, world, axis, ids=ids, n_glob=n_glob, cuts=cuts)
    else:
        cfg, parts = c.build()
        slab = gloo_slab(rank, world, axis, cuts=cuts)
    res = {}
    with MphSolver(cfg, parts, device=0, slab=slab) as s:
        ov = s.dist_overlap()
        res["overlap"] = np.array([float(ov["overlap"]), ov["halo_exchange_ms"], ov["redistribution_exchange_ms"],
                                   ov["split_pass_b_cost_ms"]])

        def owner_map():
            parts_ = [None] * world
            dist.all_gather_object(parts_, s.owned_ids())
            m = np.full(s.n, -1, np.int32)
            for r, ids in enumerate(parts_):
                m[ids] = r
            return m

        res["owner0"] = owner_map()
        done = 0
        for k in checkpoints:
            s.step(k - done)
            done = k
            if os.environ.get("MPH_TEST_PROFILE_GRAPHS") == "1" and k == checkpoints[0]:
                res["graph_ms"] = np.array([v if v is not None else -1.0
                                            for v in s.profile_graphs(4).values()])   # no exchange
            for f in fields:
                res["s%d/%s" % (k, f)] = gather_field(s, f)
            res["s%d/owner" % k] = owner_map()
    if rank == 0:
        np.savez(out_path, **res)
    dist.barrier()
    dist.destroy_process_group()


def exchange_worker(rank, world, port, out_path):
    """CPU: route tagged messages through GlooExchange and record what arrived."""
    dist = _init(rank, world, port)
    from particlemethod_fsi_amd.dist import GlooExchange
    ex = GlooExchange(rank, world)
    left, right = (rank - 1) % world, (rank + 1) % world
    # message sizes depend on (sender, direction) so a mis-route shows up as a size/content error
    def msg(src, direction):
        n = 8 + 3 * src + (5 if direction == "L" else 0)
        return bytearray([(src * 7 + (1 if direction == "L" else 2) + i) % 251 for i in range(n)])
    send_l, send_r = msg(rank, "L"), msg(rank, "R")
    recv_l = bytearray(len(msg(left, "R")))
    recv_r = bytearray(len(msg(right, "L")))
    ex(memoryview(send_l), memoryview(send_r), memoryview(recv_l), memoryview(recv_r))
    ok = recv_l == msg(left, "R") and recv_r == msg(right, "L")
    flags = [None] * world
    dist.all_gather_object(flags, bool(ok))
    if rank == 0:
        np.save(out_path, np.array(flags))
    dist.barrier()
    dist.destroy_process_group()


def band_worker(rank, world, port, case, out_path):
    """CPU: each rank selects its owned particles and the band particles it sends to its two
    neighbours (the rule of mph_params.h slab_class, via the library's host functions), ships the
    bands through GlooExchange, and checks that owned + received ghosts contain every reference
    neighbour (golden lists) of every owned particle."""
    dist = _init(rank, world, port)
    from golden_utils import Golden
    from particlemethod_fsi_amd import solver, cases
    from particlemethod_fsi_amd.dist import GlooExchange
    c = cases.get(case)
    cfg, _ = c.build()
    g = Golden(case)
    pos = g.get(1, "Position")
    off, ids = g.get(1, "nbr_offsets"), g.get(1, "nbr_ids")
    axis = SLAB_AXIS[case]
    lo, hi, h = solver.slab_bounds(cfg, rank, world, axis)
    owner = np.array([solver.slab_owner(cfg, world, axis, x) for x in pos[:, axis]])
    mine = np.nonzero(owner == rank)[0]
    a = pos[mine, axis]
    band_l = mine[(a - lo) < h]          # -> left neighbour
    band_r = mine[(hi - a) <= h]         # -> right neighbour
    ex = GlooExchange(rank, world)
    # sizes first (fixed 8-byte messages), then the index lists
    sl = np.array([len(band_l)], np.int64).tobytes()
    sr = np.array([len(band_r)], np.int64).tobytes()
    rl, rr = bytearray(8), bytearray(8)
    ex(memoryview(bytearray(sl)), memoryview(bytearray(sr)), memoryview(rl), memoryview(rr))
    nl, nr = int(np.frombuffer(rl, np.int64)[0]), int(np.frombuffer(rr, np.int64)[0])
    bl, br = bytearray(4 * nl), bytearray(4 * nr)
    ex(memoryview(bytearray(band_l.astype(np.int32).tobytes())),
       memoryview(bytearray(band_r.astype(np.int32).tobytes())), memoryview(bl), memoryview(br))
    ghosts = np.concatenate([np.frombuffer(bl, np.int32), np.frombuffer(br, np.int32)])
    have = np.zeros(len(pos), bool)
    have[mine] = True
    have[ghosts] = True
    missing = 0
    for i in mine:
        nb = ids[off[i]:off[i + 1]]
        missing += int((~have[nb]).sum())
    res = [None] * world
    dist.all_gather_object(res, (len(mine), missing, int(len(ghosts))))
    if rank == 0:
        np.save(out_path, np.array(res))
    dist.barrier()
    dist.destroy_process_group()


def gpu_rank_worker(rank, world, port, case, axis, nsteps, fields, out_dir, transport="host", cuts_mode=None):
    """One slab rank of a large case on cuda:0 (several ranks share the GPU), created from its own
    window of the case only (slab-local creation): run `nsteps`, then save this rank's owned
    particle ids and their `fields` to out_dir/rank<r>.npz (no gather through the process group,
    so it scales to the 16M-particle configuration)."""
    dist = _init(rank, world, port)
    from particlemethod_fsi_amd import MphSolver, cases
    from particlemethod_fsi_amd.dist import build_local, gloo_slab, rccl_slab
    c = cases.get(case)
    cuts = make_cuts(c, world, axis, cuts_mode)
    cfg, parts, ids, n_glob = build_local(c, rank, world, axis, cuts)
    mk = gloo_slab if transport == "host" else rccl_slab
    with MphSolver(cfg, parts, device=0, slab=mk(rank, world, axis, ids=ids, n_glob=n_glob, cuts=cuts)) as s:
        del parts
        s.step(nsteps)
        ids = s.owned_ids()
        res = {"ids": ids, "time": np.array([s.time])}
        for f in fields:
            res[f] = s.get(f)[ids]
    np.savez(os.path.join(out_dir, "rank%d.npz" % rank), **res)
    dist.barrier()
    dist.destroy_process_group()


def gpu_capacity_worker(rank, world, port, case, batches, out_dir):
    """Slab rank of `case` on cuda:0 (host-staged transport): run the step batches (one mph_step
    call each), after each one record the message capacities of mph_dist_info, and stop at the
    first error with its status code; rank r saves rank<r>.npz (caps [batch, 2], code, fields)."""
    dist = _init(rank, world, port)
    from particlemethod_fsi_amd import MphSolver, cases
    from particlemethod_fsi_amd.dist import gloo_slab
    from particlemethod_fsi_amd.solver import MphError
    c = cases.get(case)
    axis = SLAB_AXIS[case]
    cfg, parts = c.build()
    caps, code, res = [], 0, {}
    try:
        with MphSolver(cfg, parts, device=0, slab=gloo_slab(rank, world, axis)) as s:
            info = s.dist_info()
            caps.append([info["cap_send"], info["cap_recv"]])   # as created
            for k in batches:
                s.step(k)
                info = s.dist_info()
                caps.append([info["cap_send"], info["cap_recv"]])
            ids = s.owned_ids()
            res = {"ids": ids, "Position": s.get("Position")[ids], "Velocity": s.get("Velocity")[ids],
                   "PressureP": s.get("PressureP")[ids], "NeighborCount": s.get("NeighborCount")[ids]}
    except MphError as e:   # creation included: its first exchange may already overflow
        code = e.code
    np.savez(os.path.join(out_dir, "rank%d.npz" % rank), caps=np.array(caps, np.int64).reshape(-1, 2),
             code=np.array([code]), **res)
    dist.barrier()
    dist.destroy_process_group()


def gpu_state_worker(rank, world, port, case, state_path, axis, nsteps, fields, out_dir, cuts_mode=None):
    """One slab rank of `case` on cuda:0 started from a saved state (state_path .npz: position,
    velocity, time -- what the reference's .prof restart holds; property and InitialPosition from
    the case), host-staged transport: record the owned ids at creation, run `nsteps`, then save the
    owned ids and their `fields` to out_dir/rank<r>.npz."""
    dist = _init(rank, world, port)
    from particlemethod_fsi_amd import MphSolver, cases, mphio
    from particlemethod_fsi_amd.dist import gloo_slab
    c = cases.get(case)
    cfg, parts = c.build()
    z = np.load(state_path)
    cfg.time = float(z["time"][0])
    parts = mphio.Particles(parts.property, np.ascontiguousarray(z["position"]), parts.initial_position,
                            np.ascontiguousarray(z["velocity"]))
    cuts = make_cuts(c, world, axis, cuts_mode)
    with MphSolver(cfg, parts, device=0, slab=gloo_slab(rank, world, axis, cuts=cuts)) as s:
        del parts
        ids0 = s.owned_ids()
        s.step(nsteps)
        ids = s.owned_ids()
        res = {"ids0": ids0, "ids": ids, "time": np.array([s.time])}
        for f in fields:
            res[f] = s.get(f)[ids]
    np.savez(os.path.join(out_dir, "rank%d.npz" % rank), **res)
    dist.barrier()
    dist.destroy_process_group()
