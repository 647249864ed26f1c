#!/usr/bin/env python3
"""Benchmark: particle-steps/s of the MPH explicit hot path on MI355X (BASELINE.json metric).

Workload (BASELINE.json configs[1], SURVEY 8d "D1M"): 3-D dam break, 1,397,200 particles
(970,000 fluid + 427,200 wall), dx = 1 mm, Dt = 1e-4 s, generated in memory with the reference
generator's algorithm and the reference's results/Dam/dam.data parameters.  One "step" = one
iteration of the reference's time loop (main.cpp:597-686): wall motion, periodic wrap, cell sort,
neighbour search, density/pressure sums, pressure/surface/viscous forces, gravity, kick, drift
(+ elastic substeps when structure particles exist).  Inputs are resident in HBM before timing.

  python bench.py [--gpus N] [--steps K] [--warmup W] [--case d1m] [--no-cpu-baseline]

For N > 1 (torchrun, one rank per GPU) the ranks run BASELINE configs[4]: the 16,205,500-particle
dam break cut into N z slabs (csrc/mph_dist.hip: RCCL ncclSend/Recv with the two
slab neighbours, steps replayed from captured hipGraphs), strong scaling; `value` counts every
particle of the whole job per step.  Each rank generates only its own window of the problem
(slab-local creation).  Other cases (`--case bar2d_400k`, `fsi3d`, `d1m_x8` ...) split the same
way (2-D cases in x slabs, 3-D in z slabs; elastic particles stay with the slab of their
InitialPosition).  After the timed steps the ranks check that ownership is a partition of all
particles and that the NeighborCount total matches the single-GPU run's at the same step
(profiles/d16m_ncount_sum.json), so a scaling run is also a correctness run.
MPH_SLAB_TRANSPORT=host switches the halo transport to host staging over gloo (diagnostics).

Rank 0 prints ONE JSON line.  `roofline` is the dominant stage's algorithmic HBM bytes per step
(SURVEY 8d per-particle figures: pass 1 = neighbour search + pass A, 92 B; pass 2 = pass B, 140 B;
grid build, 140 B) over the HIP-event-timed time of the kernels that carry it;
`roofline.step_frac` is the whole step's 372 B per particle at the measured rate, and
`neighbor_list` the list bytes SURVEY's figures leave out.  `cpu_baseline` times the reference
solver itself (oracle/_ref, built from /root/reference) on a bounded sample of the same workload
on this host's cores.
"""
from __future__ import annotations

import argparse
import json
import os
import subprocess
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBPS = 8000.0      # MI355X HBM3E spec (MI355X_MICROARCH.md, chip-level parameters)
FP64_PEAK_TFLOPS = 78.6     # MI355X FP64 vector spec
# algorithmic bytes per particle per launch
ALG_BYTES = {"pass_a": 92.0, "neighbors_pass_a": 92.0, "pass_b": 140.0, "sort": 140.0}
# SURVEY 8d's stages and the kernels that carry them: "pass 1" (read x, v, type; write PressureP,
# PressureA, GravityCenter: 92 B) is the neighbour search and pass A together (or their fused
# form), "pass 2" (140 B) is pass B, the grid build + reorder (140 B) the sort kernels
STAGES = {
    "neighbors+pass_a": (92.0, ("neighbors", "neighbors_redo", "search_pass_a", "pass_a")),
    "pass_b": (140.0, ("pass_b", "pass_b_inner", "pass_b_face")),
    "sort": (140.0, ("prep", "scan_reduce", "scan_top", "scan_down", "place", "rank_scatter")),
}
# elastic substep kernels, per structure particle and launch (SURVEY 8d "500 + 8 n_s" split by
# kernel; n_s = mean InitialStructureNeighborCount; output-only DeformGradient/Strain/Stress
# excluded as for the fluid passes):
#   struct_stress   read x, x0 (48), L (72), Lame (16), list (4 n_s); write P (72)
#   struct_velocity read P (72), v, x (48), out- and in-lists (8 n_s); write v, x (48)
STRUCT_BYTES = {"struct_stress": (208.0, 4.0), "struct_velocity": (168.0, 8.0)}
B_ALG_STEP = 372.0          # grid build 140 + pass 1 92 + pass 2 140
# the reference-literal gather bytes per particle-step (3-D): neighbour fields of its 8
# neighbour loops, the 343-cell search, the list reset/write and the bitonic passes -- what the
# north star's "50 % of HBM at 1e8" is consistent with; a label, never a measured figure
B_GATHER_3D = 42.7e3
SLAB_AXIS = {2: 0, 3: 2}    # by dimension: z slabs for the 3-D dam workloads, x in 2-D


def dist_env():
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    return rank, world, local


def cpu_baseline(case_name: str, seconds_target: float = 15.0):
    """Time the reference (oracle/_ref) -- or, if absent, the CPU oracle port -- on the same
    workload, in a child process, on this host's cores (OMP_NUM_THREADS)."""
    script = r"""
import sys, os, time, json, ctypes, numpy as np, tempfile
sys.path.insert(0, %(root)r); sys.path.insert(0, %(root)r + '/tests')
from particlemethod_fsi_amd import cases, solver
from oracle_bindings import RefSolver, OracleSolver, ref_available
c = cases.get(%(case)r)
cfg, p = c.build()
threads = int(os.environ.get('OMP_NUM_THREADS', os.cpu_count() or 1))
if ref_available(c.dim, c.ref_variant):
    d = tempfile.mkdtemp(prefix='mphcpu_')
    dp, gp = os.path.join(d, 'c.data'), os.path.join(d, 'c.grid')
    open(dp, 'w').write(cases.data_text(c.data()))
    L = solver.load_library()
    L.mph_write_prof_arrays(gp.encode(), ctypes.byref(cfg), 0.0, p.n, p.property.ctypes.data,
                            p.position.ctypes.data, p.initial_position.ctypes.data, p.velocity.ctypes.data)
    s = RefSolver(c.dim, c.ref_variant, dp, gp); kind = 'reference'
else:
    s = OracleSolver(cfg, p); kind = 'port'
s.init()
t0 = time.time(); s.step(1); t1 = time.time()
per = t1 - t0
k = max(1, min(20, int(%(target)f / max(per, 1e-6))))
t2 = time.time(); s.step(k); t3 = time.time()
print(json.dumps({'value': p.n * k / (t3 - t2), 'unit': 'particle-steps/s', 'cores': threads,
                  'kind': kind, 'sample': '%%s: %%d particles, %%d timed steps after 1 warm-up step (%%.1f s)'
                  %% (%(case)r, p.n, k, t3 - t2)}))
""" % {"root": ROOT, "case": case_name, "target": seconds_target}
    try:
        r = subprocess.run([sys.executable, "-c", script], capture_output=True, text=True, timeout=900)
        for line in r.stdout.splitlines()[::-1]:
            if line.startswith("{"):
                return json.loads(line)
        return {"error": (r.stderr or r.stdout)[-500:]}
    except Exception as e:  # pragma: no cover
        return {"error": repr(e)}


def load_pmc(name: str, case: str, kernel: str, key: str):
    """`key` of `kernel` from a committed rocprofv3 PMC summary (profiles/<name>.json, written by
    tools/pmc_traffic.py / tools/pmc_fp64.py), if it was measured on this case."""
    try:
        with open(os.path.join(ROOT, "profiles", name + ".json")) as fh:
            d = json.load(fh)
    except (OSError, ValueError):
        return None
    if d.get("case") != case:
        return None
    return d.get(kernel, {}).get(key)


def _id_hash(ids):
    """xor of a 64-bit mix of every id (order-free fingerprint of an id set)."""
    import numpy as np
    x = ids.astype(np.uint64) * np.uint64(0x9E3779B97F4A7C15)
    x ^= x >> np.uint64(29)
    x *= np.uint64(0xBF58476D1CE4E5B9)
    x ^= x >> np.uint64(32)
    return int(np.bitwise_xor.reduce(x)) if len(x) else 0


def slab_checks(solver, dist, n_total, case_name, steps_done):
    """After a multi-rank run: RCCL communicator size, graph replay, ownership a partition of all
    particles (count, id sum, id-set fingerprint), and the NeighborCount total over the owned
    particles against the single-GPU run's at the same step (bit-exact neighbour sets)."""
    import numpy as np
    import torch
    info = solver.dist_info()
    ids = solver.owned_ids()
    nc = solver.get("NeighborCount")[ids]
    loc = torch.tensor([len(ids), int(ids.astype(np.int64).sum()), int(nc.astype(np.int64).sum()),
                        int(nc.max()) if len(nc) else 0], dtype=torch.int64)
    tot = loc.clone()
    dist.all_reduce(tot, op=dist.ReduceOp.SUM)
    mx = loc[3:4].clone()
    dist.all_reduce(mx, op=dist.ReduceOp.MAX)
    hashes = [None] * dist.get_world_size()
    dist.all_gather_object(hashes, _id_hash(ids))
    h = 0
    for v in hashes:
        h ^= v
    partition = (int(tot[0]) == n_total and int(tot[1]) == n_total * (n_total - 1) // 2
                 and h == _id_hash(np.arange(n_total)))
    expected = None
    try:
        with open(os.path.join(ROOT, "profiles", "%s_ncount_sum.json" % case_name)) as fh:
            table = json.load(fh)["sum_after_steps"]
        if steps_done < len(table):
            expected = int(table[steps_done])
    except (OSError, ValueError, KeyError):
        pass
    return {"slab_ranks": info["nranks"], "rccl_nranks": info["rccl_ranks"],
            "pass_b_mode": solver.dist_overlap(),
            "transport": "rccl" if info["rccl_ranks"] else "host-staged",
            "graphs": bool(info["graphs"]), "partition_ok": bool(partition), "owned_total": int(tot[0]),
            "steps_done": steps_done, "neighbor_count_sum": int(tot[2]),
            "neighbor_count_sum_single_gpu": expected,
            "neighbor_count_ok": (expected == int(tot[2])) if expected is not None else None,
            "neighbor_count_max": int(mx[0])}



def graph_times(solver_obj, prof, reps=16):
    """Replace the list kernels' direct-launch times in a mph_profile_steps result by their times
    as graph replays (mph_profile_graphs), as the timed steps run them; the direct times stay under
    "avg_ms_direct".  The search's graph includes the XCD split, whose direct time is taken off."""
    try:
        g = solver_obj.profile_graphs(reps)
    except Exception as e:   # slab contexts, or no step yet
        print("bench: graph-replay kernel times unavailable: %s" % e, file=sys.stderr)
        return False
    for k, v in g.items():
        if v is None or k not in prof:
            continue
        if k == "neighbors" and "xcd_split" in prof:
            v = max(0.0, v - prof["xcd_split"]["avg_ms"])
        prof[k]["avg_ms_direct"] = prof[k]["avg_ms"]
        prof[k]["avg_ms"] = v
    return True

def loop_steps(t0: float, dt: float, end_time: float) -> int:
    """Iterations of the reference's time loop (main.cpp:581: while (Time < EndTime + 1e-5 Dt),
    Time += Dt at its end) from Time t0, in the same double arithmetic."""
    t, k = t0, 0
    while t < end_time + 1.0e-5 * dt:
        t += dt
        k += 1
    return k


def run_whole(first, cfg, parts, n_total, end_time, profile_steps, device):
    """The reference's whole run on a fresh context (bench line `run_average`).  The headline's
    context is kept for the rest of the line; this one is created after it and closed here."""
    from particlemethod_fsi_amd import MphSolver
    total = loop_steps(cfg.time, cfg.dt, end_time)
    mid = min(total, loop_steps(cfg.time, cfg.dt, cfg.time + 0.25 * (end_time - cfg.time)))
    segs, kern = [], {}
    with MphSolver(cfg, parts, device=device) as s:
        s.synchronize()
        done = 0
        for upto, label in ((mid, "t=%.3g" % (mid * cfg.dt)), (total, "t=%.3g" % (total * cfg.dt))):
            n = upto - done - (profile_steps if done else 0)
            t0 = time.perf_counter()
            s.step(n)
            s.synchronize()
            segs.append((n, time.perf_counter() - t0))
            done = upto
            p = s.profile(profile_steps)
            p.pop("gpu_busy", None)
            graph_times(s, p)
            kern[label] = {k: round(v["avg_ms"], 5) for k, v in p.items()}
            done += profile_steps
        mean_nb, max_nb = s.neighbor_stats()
    steps = sum(n for n, _ in segs)
    secs = sum(e for _, e in segs)
    return {"value": n_total * steps / secs, "ms_per_step": secs * 1e3 / steps, "steps_timed": steps,
            "loop_steps": total, "end_time": end_time, "wall_s": secs,
            "segments": [{"steps": n, "ms_per_step": e * 1e3 / n} for n, e in segs],
            "kernels_ms": kern, "neighbors_at_end": {"mean": mean_nb, "max": max_nb},
            "note": "fresh context, t = 0 -> EndTime, wall time between synchronizes; the %d profiled "
                    "steps after each segment are neither timed nor counted" % profile_steps}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=40)
    ap.add_argument("--warmup", type=int, default=8)
    ap.add_argument("--case", default="d1m")
    ap.add_argument("--profile-steps", type=int, default=4)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    # the developed flow: after the headline measurement the same context runs on to
    # this many steps in all (D1M: t = 0.25 s of the reference's 1 s dam run, main.cpp:581 with
    # results/Dam/dam.data EndTime 1.0) and times --steps more there; 0 skips it
    ap.add_argument("--developed-steps", type=int, default=None)
    # start from a saved state instead of the generator's lattice (a binary grid of
    # tools/dev_state.py: Time, x, x0, v -- the reference's .prof restart); profiles of the developed flow
    ap.add_argument("--state", default=None)
    # the reference's whole run as one figure (run_whole): EndTime in s; default 1.0 for d1m, 0 skips
    ap.add_argument("--run-average-end", type=float, default=None)
    args = ap.parse_args()

    rank, world, local = dist_env()
    device = int(os.environ.get("MPH_BENCH_DEVICE", local))   # rehearsals: ranks sharing a GPU
    from particlemethod_fsi_amd import MphSolver, cases

    dist = None
    cuts = None
    fallback = None
    case_name = args.case
    if world > 1:
        # one process per GPU; torch.distributed (gloo) is only the control plane (rendezvous,
        # RCCL unique id, timing reduction, the post-run checks).  Particle data moves over the
        # library's own RCCL communicator (ncclSend/Recv with the two slab neighbours).
        import torch
        import torch.distributed as tdist
        torch.cuda.set_device(device)
        tdist.init_process_group("gloo")
        dist = tdist
        if case_name == "d1m":
            case_name = "d16m"   # BASELINE configs[4]: 16M particles, N MI355X, z slabs

    case = cases.get(case_name)
    if dist is not None:
        from particlemethod_fsi_amd.dist import balanced_cuts, build_local, gloo_slab, rccl_slab
        axis = SLAB_AXIS[case.dim]
        # slab boundaries at the particle-count quantiles (equal shares; MPH_SLAB_EQUAL=1: equal widths)
        cuts = None if os.environ.get("MPH_SLAB_EQUAL") == "1" else balanced_cuts(case, world, axis)
        cfg, parts, ids, n_total = build_local(case, rank, world, axis, cuts)
        host = os.environ.get("MPH_SLAB_TRANSPORT") == "host"
        mk = gloo_slab if host else rccl_slab

        def agreed(ok):   # every rank's verdict (gloo all-reduce): False if any rank failed
            import torch
            t = torch.tensor([1 if ok else 0], dtype=torch.int32)
            dist.all_reduce(t, op=dist.ReduceOp.MIN)
            return bool(t.item())

        # RCCL over xGMI has not run on this code's 8-GPU path before the driver's first scaling
        # run: a rank whose RCCL communicator or first (graph-captured) step fails makes every rank
        # fall back to the host-staged transport, and the line says so (`slab.transport_fallback`)
        # instead of the job dying.  (A hang cannot be caught this way.)
        solver, err = None, None
        try:
            solver = MphSolver(cfg, parts, device=device,
                               slab=mk(rank, world, axis, ids=ids, n_glob=n_total, cuts=cuts))
            solver.step(1)
            solver.synchronize()
        except Exception as e:   # noqa: BLE001 -- reported in the JSON line
            err = "%s: %s" % (type(e).__name__, e)
        if not host and not agreed(err is None):
            fallback = {"from": "rccl", "to": "host-staged", "rank": rank, "error": err}
            if solver is not None:
                solver.close()
            solver = MphSolver(cfg, parts, device=device,
                               slab=gloo_slab(rank, world, axis, ids=ids, n_glob=n_total, cuts=cuts))
            solver.step(1)
        elif err is not None:
            raise RuntimeError(err)
        del parts, ids
        n_local = len(solver.owned_ids())
    else:
        cfg, parts = case.build()
        if args.state:
            from particlemethod_fsi_amd.solver import read_case_files
            d = tempfile.mkdtemp(prefix="mphstate_")
            with open(os.path.join(d, "c.data"), "w") as fh:
                fh.write(cases.data_text(case.data()))
            scfg, sparts = read_case_files(os.path.join(d, "c.data"), args.state, case.dim, case.module)
            assert sparts.n == parts.n and (sparts.property == parts.property).all(), "state of another case"
            cfg.time = scfg.time
            parts = sparts
        n_total = parts.n
        solver = MphSolver(cfg, parts, device=device)
        n_local = n_total

    def barrier():
        solver.synchronize()
        if dist is not None:
            import torch
            torch.cuda.synchronize()
            dist.barrier()

    solver.step(max(0, args.warmup - (1 if dist is not None else 0)))   # (slab mode: one step ran above)
    barrier()
    t0 = time.perf_counter()
    solver.step(args.steps)
    barrier()
    elapsed = time.perf_counter() - t0
    elapsed_local = elapsed
    if dist is not None:
        import torch
        t = torch.tensor([elapsed], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    value = n_total * args.steps / elapsed   # every particle of the whole job, once per step

    # the drop-in binding's own call pattern: one mph_step(ctx, 1) per
    # time-loop iteration over the same number of steps, with step batching on as INTEGRATION.md
    # recommends (mph_set_step_batching: the steps run 8 per graph, flushed by the synchronize that
    # closes the timed region), and without it ("sync": a 1-step graph that stores every
    # output-only field and one readback of the error flags per call)
    step1 = None
    if world == 1:
        def per_call(batched):
            solver.step_batching(batched)
            barrier()
            t1 = time.perf_counter()
            for _ in range(args.steps):
                solver.step(1)
            barrier()
            e1 = time.perf_counter() - t1
            solver.step_batching(False)
            return n_total * args.steps / e1, e1 * 1e3 / args.steps
        v_sync, ms_sync = per_call(False)
        v_b, ms_b = per_call(True)
        step1 = {"value": v_b, "ms_per_step": ms_b, "gap": 1.0 - v_b / value, "batching": True,
                 "sync": {"value": v_sync, "ms_per_step": ms_sync, "gap": 1.0 - v_sync / value}}

    mean_nb, max_nb = solver.neighbor_stats()
    nc_created = solver.get("NeighborCount") if world == 1 else None
    prof = solver.profile(args.profile_steps)
    graph_timed = world == 1 and dist is None and graph_times(solver, prof)
    checks = None
    if dist is not None:
        checks = slab_checks(solver, dist, n_total, case_name, max(args.warmup, 1) + args.steps + args.profile_steps)
        # per rank, so that the first multi-GPU run is diagnosable: the rank's own wall time per
        # timed step (before the max over ranks), its kernels' summed HIP-event time per step
        # (compute, mph_profile_steps) and the rest (exchange + waiting for the slowest neighbour)
        info = solver.dist_info()
        kern_ms = sum(v["avg_ms"] * v["launches"] for k, v in prof.items() if k != "gpu_busy") / max(1, args.profile_steps)
        mine = {"rank": rank, "owned": len(solver.owned_ids()), "held": info["held"],
                "ms_per_step": elapsed_local * 1e3 / args.steps, "compute_ms": kern_ms,
                "exchange_and_wait_ms": elapsed_local * 1e3 / args.steps - kern_ms,
                "kernels_ms": {k: round(v["avg_ms"] * v["launches"] / max(1, args.profile_steps), 5)
                               for k, v in prof.items() if k != "gpu_busy"}}
        per_rank = [None] * world
        dist.all_gather_object(per_rank, mine)
        checks["per_rank"] = per_rank
    ns, mean_ns = 0, 0.0
    if any(k in prof for k in STRUCT_BYTES):
        isnc = solver.get("InitialStructureNeighborCount")
        prop = solver.get("Property")
        smask = (prop == 2) | (prop == 3)
        ns = int(smask.sum())
        mean_ns = float(isnc[smask].mean()) if ns else 0.0

    def alg_bytes_of(k):
        if k in STRUCT_BYTES:
            a, b = STRUCT_BYTES[k]
            return (a + b * mean_ns) * ns
        return ALG_BYTES[k] * n_local

    # dominant stage by total time per step: SURVEY 8d's stages (STAGES, each the sum of its
    # kernels' HIP-event time per step) and the elastic substep kernels
    steps_prof = max(1, args.profile_steps)
    units = {}
    for st, (b, ks) in STAGES.items():
        ms = sum(prof[k]["avg_ms"] * prof[k]["launches"] for k in ks if k in prof) / steps_prof
        if ms > 0:
            units[st] = {"ms": ms, "bytes": b * n_local, "kernels": [k for k in ks if k in prof]}
    for k in STRUCT_BYTES:
        if k in prof:
            units[k] = {"ms": prof[k]["avg_ms"], "bytes": alg_bytes_of(k), "kernels": [k],
                        "per_launch": True, "launches_per_step": prof[k]["launches"] / steps_prof}
    dom = max(units, key=lambda u: units[u]["ms"] * units[u].get("launches_per_step", 1.0))
    # "gpu_busy" (mph_profile_steps) is the union of the kernel intervals, not a kernel
    busy_ms = prof.pop("gpu_busy", {}).get("avg_ms")
    step_ms = sum(v["avg_ms"] * v["launches"] for v in prof.values()) / steps_prof
    alg_bytes = units[dom]["bytes"]
    achieved = alg_bytes / (units[dom]["ms"] * 1e-3) / 1e9
    # PMC bytes of the same kernels per step (committed rocprofv3 summary of this case)
    traffic = None
    tr = [load_pmc("pmc_traffic", case_name, k, "hbm_bytes_per_launch") for k in units[dom]["kernels"]
          if k != "neighbors_redo"]
    if tr and all(t is not None for t in tr):
        traffic = float(sum(tr))
    # the neighbour list, which SURVEY's 372 B leave out: written by the search, read by both
    # passes; algorithmic 4 B per entry against the search's measured WRITE_SIZE
    list_info = None
    if world == 1:
        try:
            mean_stored = solver.list_stats()[0]   # the stored lists (the passes' radius), not NeighborCount
        except AttributeError:   # an ABI-3 library in a same-box A/B (MPH_ABI_ACCEPT=3)
            mean_stored = solver.neighbor_stats()[0]
        list_alg = 4.0 * mean_stored * n_local
        wr = load_pmc("pmc_traffic", case_name, "neighbors", "write_kib")
        list_info = {"entries_per_particle": mean_stored, "alg_bytes_written": list_alg,
                     "alg_bytes_read_by_passes": 2.0 * list_alg,
                     "search_write_bytes_measured": wr * 1024.0 if wr else None,
                     "write_amplification": (wr * 1024.0 / list_alg) if wr and list_alg else None}
    # measured HBM traffic of a whole step: rocprofv3 FETCH_SIZE/WRITE_SIZE per kernel in the timed
    # region's store pattern (tools/profile.sh + tools/pmc_traffic.py, calibration
    # profiles/pmc_calib.json), over this run's own step time
    step_bytes = None
    try:
        with open(os.path.join(ROOT, "profiles", "pmc_traffic.json")) as fh:
            d = json.load(fh)
        if d.get("case") == case_name and world == 1:
            step_bytes = d.get("hbm_bytes_per_step")
    except (OSError, ValueError):
        pass
    # what binds the dominant stage's kernels (the HBM roofline does not): the
    # larger of VALU issue and the L1 (TCP) tag-lookup rate, each as a fraction of its ceiling, from
    # the committed PMC summary of this case (tools/pmc_ab.sh + tools/pmc_issue.py)
    binding = None
    try:
        with open(os.path.join(ROOT, "profiles", "pmc_issue.json")) as fh:
            iss = json.load(fh)
        if iss.get("case") == case_name and world == 1:
            per = {}
            for k in units[dom]["kernels"]:
                v = iss.get(k)
                if not v:
                    continue
                # the measured verdict when the summary records one (e.g. the search: latency, since
                # fewer VALU per wave did not shorten it), else the larger of the two rates
                res = v.get("binding") or ("valu_issue" if v["valu_busy"] >= v["l1_lookups_per_clk"]
                                           else "l1_tag_lookups")
                ta = v.get("ta_busy", 0.0)   # texture-address unit busy fraction
                per[k] = {"resource": res, "frac": max(v["valu_busy"], v["l1_lookups_per_clk"], ta),
                          "valu_issue": v["valu_busy"], "l1_tag_lookups_per_clk_cu": v["l1_lookups_per_clk"],
                          "ta_busy": ta}
                if v.get("binding_note"):
                    per[k]["note"] = v["binding_note"]
            if per:
                w = {k: prof[k]["avg_ms"] * prof[k]["launches"] for k in per if k in prof}
                tot = sum(w.values()) or 1.0
                top = max(per, key=lambda k: w.get(k, 0.0))
                binding = {"resource": per[top]["resource"],
                           "frac": sum(per[k]["frac"] * w.get(k, 0.0) for k in per) / tot,
                           "kernels": per, "source": "profiles/pmc_issue.json (%s)" % iss.get("source")}
    except (OSError, ValueError, KeyError):
        pass
    # FP64 utilisation: PMC lane FLOPs per launch over the same live launch time
    flops = {k: load_pmc("pmc_fp64", case_name, k, "lane_flops_per_launch") for k in prof}
    fp64 = {k: {"tflops": f / (prof[k]["avg_ms"] * 1e-3) / 1e12,
                "frac": f / (prof[k]["avg_ms"] * 1e-3) / 1e12 / FP64_PEAK_TFLOPS}
            for k, f in flops.items() if f}
    # The headline times the first steps of a column at rest (particles still on the lattice).  The
    # developed flow -- the dam collapsed for t = 0.25 s, particles off the lattice, neighbour sets
    # changed -- is timed on the same context after running on untimed.
    developed = None
    dev_total = args.developed_steps if args.developed_steps is not None else (
        2500 if case_name == "d1m" and not args.state else 0)
    done = args.warmup + 3 * args.steps + args.profile_steps if world == 1 else 0
    if world == 1 and dev_total > done + args.warmup:
        solver.step(dev_total - done)
        barrier()
        td0 = time.perf_counter()
        solver.step(args.steps)
        barrier()
        e_dev = time.perf_counter() - td0
        dmean, dmax = solver.neighbor_stats()
        nc_dev = solver.get("NeighborCount")
        dprof = solver.profile(args.profile_steps)
        dprof.pop("gpu_busy", None)
        graph_times(solver, dprof)
        dev_units = {st: sum(dprof[k]["avg_ms"] * dprof[k]["launches"] for k in ks if k in dprof) / steps_prof
                     for st, (b, ks) in STAGES.items()}
        developed = {"value": n_total * args.steps / e_dev, "ms_per_step": e_dev * 1e3 / args.steps,
                     "steps_before_timing": dev_total, "time_s": round(dev_total * cfg.dt, 9),
                     "gap": 1.0 - (n_total * args.steps / e_dev) / value,
                     "neighbors": {"mean": dmean, "max": dmax},
                     "neighbor_count_changed_frac": float((nc_dev != nc_created).mean()),
                     "kernels_ms": {k: round(v["avg_ms"], 5) for k, v in dprof.items()},
                     "kernels_ms_direct": {k: round(v["avg_ms_direct"], 5) for k, v in dprof.items()
                                           if "avg_ms_direct" in v},
                     "stages_ms": {k: round(v, 5) for k, v in dev_units.items()},
                     "roofline_frac": (STAGES[dom][0] * n_local / (dev_units[dom] * 1e-3) / 1e9 / HBM_PEAK_GBPS)
                     if dom in dev_units and dev_units[dom] > 0 else None}
    # The reference's whole run: a fresh context from t = 0 to EndTime (D1M:
    # results/Dam/dam.data EndTime 1.0, the loop `while (Time < EndTime + 1e-5 Dt)` of main.cpp:581,
    # 10,001 steps), wall time between synchronizes in two segments; the kernels are profiled
    # between them at t = 0.25 s and after the last step at t = 1.0 s (those profiled steps are
    # neither timed nor counted).  The VTK/.prof writes of the reference's loop are not in it.
    run_average = None
    end_time = args.run_average_end if args.run_average_end is not None else (
        1.0 if case_name == "d1m" and not args.state else 0.0)
    if world == 1 and end_time > 0.0:
        run_average = run_whole(solver, cfg, parts, n_total, end_time, args.profile_steps, device)
    out = {
        "metric": "particle-steps/sec + achieved HBM GB/s, dam-break, 1/2/4/8 MI355X",
        "value": value,
        "unit": "particle-steps/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": elapsed * 1e3 / args.steps,
        "higher_is_better": True,
        "scaling": "weak" if world == 1 else "strong",
        "vs_baseline": None,
        "dtype": "f64",
        "data": "synthetic (reference generator algorithm + results/Dam/dam.data parameters)",
        "config": {"workload": "%s: %s, %d particles, ~%d per GPU"
                               % (case_name, case.describe(), n_total, n_total // world),
                   "particles": n_total, "dim": case.dim, "module": case.module, "dt": cfg.dt,
                   "parallelism": "single" if world == 1 else "slab%d-%s (%s halo exchange, %s)" % (
                       world, "xyz"[SLAB_AXIS[case.dim]],
                       "host-staged" if os.environ.get("MPH_SLAB_TRANSPORT") == "host" or fallback else "RCCL",
                       "equal widths" if cuts is None else "cuts at particle-count quantiles"),
                "slab_cuts": None if cuts is None else [round(float(x), 9) for x in cuts]},
        "achieved_hbm_gbps_alg": B_ALG_STEP * value / 1e9,
        "achieved_hbm_gbps_measured": (step_bytes / (elapsed / args.steps) / 1e9) if step_bytes else None,
        "hbm_measured": ({"bytes_per_step": step_bytes, "bytes_per_particle_step": step_bytes / n_total,
                          "source": "profiles/pmc_traffic.json: 2 x FETCH_SIZE + WRITE_SIZE per kernel, "
                                    "8-step store pattern (calibrated: profiles/pmc_calib.json)"}
                         if step_bytes else None),
        "gather_literal_gbps": {"value": (B_GATHER_3D if case.dim == 3 else 12e3) * value / 1e9,
                                "note": "reference-literal gather bytes (SURVEY 8d B_gather, %.1f kB per "
                                        "particle-step) x rate: a label for the north-star target, not "
                                        "HBM traffic" % ((B_GATHER_3D if case.dim == 3 else 12e3) / 1e3)},
        "neighbors": {"mean": mean_nb, "max": max_nb},
        # bound: the resource the PMC summary measured as binding the dominant stage (not HBM, DESIGN.md
        # section 3); achieved / peak / frac stay the HBM roofline's (peak_of)
        "roofline": {"bound": binding["resource"] if binding else "hbm", "peak_of": "hbm",
                     "kernel": dom, "kernels": units[dom]["kernels"],
                     "achieved": achieved, "peak": HBM_PEAK_GBPS,
                     "unit": "GB/s", "frac": achieved / HBM_PEAK_GBPS,
                     "traffic": traffic, "alg_bytes_per_launch": alg_bytes,
                     "avg_launch_ms": units[dom]["ms"],
                     "step_frac": B_ALG_STEP * value / world / (HBM_PEAK_GBPS * 1e9),
                     "binding": binding,
                     "stages": {u: {"ms": round(v["ms"], 5),
                                    "frac": v["bytes"] / (v["ms"] * 1e-3) / 1e9 / HBM_PEAK_GBPS}
                                for u, v in units.items()}},
        "neighbor_list": list_info,
        "fp64": ({"peak_tflops": FP64_PEAK_TFLOPS, "source": "profiles/pmc_fp64.json (64 x "
                  "SQ_INSTS_VALU_FLOPS_FP64 per launch, masked lanes included)",
                  "kernels": {k: {a: round(b, 4) for a, b in v.items()} for k, v in fp64.items()}}
                 if fp64 else None),
        # HIP events: the search, pass A and pass B as graph replays (mph_profile_graphs, as the timed
        # steps run), the other kernels as direct launches (mph_profile_steps; kernels_ms_direct:
        # the list kernels that way too, 3-8 % slower)
        "kernels_ms": {k: round(v["avg_ms"], 5) for k, v in prof.items()},
        "kernels_ms_direct": {k: round(v["avg_ms_direct"], 5) for k, v in prof.items() if "avg_ms_direct" in v},
        "kernels_timed_as": "graph replays (search, pass A, pass B)" if graph_timed else "direct launches",
        "profiled_step_ms": step_ms,
        "profiled_gpu_busy_ms": busy_ms,
        "value_step1": step1["value"] if step1 else None,
        "step1": step1,
        "developed": developed,
        "run_average": run_average,
    }
    if checks is not None:
        if fallback is not None:
            checks["transport_fallback"] = fallback
        out["slab"] = checks
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        if case_name == "d16m":
            out["cpu_baseline"] = {"value": None, "unit": "particle-steps/s", "kind": "reference",
                                   "note": "not run: the reference allocates three int[N][512] tables "
                                           "(main.cpp:878-882), ~100 GB at 16.2M particles"}
        else:
            out["cpu_baseline"] = cpu_baseline(args.case)
    solver.close()
    if rank == 0:
        print(json.dumps(out), flush=True)
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
