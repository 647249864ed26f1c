"""Clean per-slab kernel timings of the multi-GPU path on ONE GPU.

The 8-rank rehearsal (tools/gpu_dist_rehearsal.sh) runs eight processes on one card at once, so
their kernels overlap and the per-kernel times it reports are inflated by the others.  Here the
N slab contexts live in one process, one thread each, and move their messages through an
in-process host exchange; a token serialises the GPU phases between exchanges (the device is
drained before a rank gives the token back inside the host exchange -- its second stream may
still run the kernels it enqueued before the exchange -- and each thread synchronises before it
gives the token back at the end of a call), so every rank's kernels run alone on the card and
the HIP-event profile of each rank is what that rank would see on its own GPU.

With --replay the profiled steps run a second time from a fresh start: every rank
then receives the messages recorded in the first run at once (bit-identical runs), holds the
token through its whole profile call and does not drain the device in an exchange, so its second
stream runs beside its main stream as on a rank of its own (the inner pass B / inner elastic
slots beside the halo, the face pass B and the early send) -- the exchange latency left is the
host staging's own copies.  The first run's figures are "serialised", the replay's "replay"
("consistent": every rank ended with the recorded run's held and owned counts).  The replay
exposed a race of the host transport (an exchange on one stream refilled the pinned staging
buffers while the previous exchange's copies on the other stream still read them; a rank then
diverged): each host-staged exchange now waits for the previous one's copies (mph_dist.hip).

usage: python tools/slab_serial.py [--case d16m] [--ranks 8] [--steps 4] [--warmup 2] [--replay]
prints one JSON line: per-rank kernel averages, held/owned counts, their GPU time per step (the
sum of the kernel times, and gpu_busy: the union of the kernel intervals, less than the sum where
the kernels of the two streams run concurrently).
"""
from __future__ import annotations

import argparse
import json
import os
import queue
import sys
import threading
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from particlemethod_fsi_amd import MphSolver, cases, solver  # noqa: E402
from particlemethod_fsi_amd.dist import balanced_cuts, build_local  # noqa: E402

SLAB_AXIS = {2: 0, 3: 2}


_HIP = None


def _device_sync():
    global _HIP
    if _HIP is None:
        import ctypes
        _HIP = ctypes.CDLL("libamdhip64.so")
    rc = _HIP.hipDeviceSynchronize()
    if rc != 0:
        raise RuntimeError("hipDeviceSynchronize: %d" % rc)


class Token:
    """The GPU: held by one rank thread while it launches work."""

    def __init__(self):
        self.lock = threading.Lock()


class InProcExchange:
    """mph_host_exchange_fn between threads: send_l -> left neighbour's recv_r, send_r -> right
    neighbour's recv_l; gives the token back while it waits for its peers."""

    def __init__(self, rank, nranks, boxes, token):
        self.rank, self.nranks, self.boxes, self.token = rank, nranks, boxes, token
        self.left, self.right = (rank - 1) % nranks, (rank + 1) % nranks
        self.record = None   # list: the received messages are appended (first run)
        self.replay = None   # iterator over recorded (recv_l, recv_r): no peers, no token hand-over

    def __call__(self, send_l, send_r, recv_l, recv_r):
        if self.replay is not None:
            bl, br = next(self.replay)
            if len(bl) != len(recv_l) or len(br) != len(recv_r):
                raise RuntimeError("replayed exchange differs from the recorded one")
            recv_l[:] = bl
            recv_r[:] = br
            return
        self._live(send_l, send_r, recv_l, recv_r)
        if self.record is not None:
            self.record.append((bytes(recv_l), bytes(recv_r)))

    def _live(self, send_l, send_r, recv_l, recv_r):
        # the rank's other stream may still run kernels it enqueued before this exchange (the
        # inner pass B / inner elastic slots): drain the device before another rank takes it
        _device_sync()
        self.token.lock.release()
        try:
            if len(send_l):
                self.boxes[(self.rank, self.left, "L")].put(bytes(send_l))
            if len(send_r):
                self.boxes[(self.rank, self.right, "R")].put(bytes(send_r))
            if len(recv_r):
                b = self.boxes[(self.right, self.rank, "L")].get(timeout=300)
                recv_r[:len(b)] = b
            if len(recv_l):
                b = self.boxes[(self.left, self.rank, "R")].get(timeout=300)
                recv_l[:len(b)] = b
        finally:
            self.token.lock.acquire()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--case", default="d16m")
    ap.add_argument("--ranks", type=int, default=8)
    ap.add_argument("--steps", type=int, default=4)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--replay", action="store_true")
    args = ap.parse_args()
    case = cases.get(args.case)
    axis = SLAB_AXIS[case.dim]
    R = args.ranks
    cuts = None if os.environ.get("MPH_SLAB_EQUAL") == "1" else balanced_cuts(case, R, axis)
    locals_ = [build_local(case, r, R, axis, cuts) for r in range(R)]
    records = [[] for _ in range(R)]
    serial = run_ranks(args, R, axis, cuts, locals_, records=records)
    result = {"case": args.case, "ranks": R, "perm": os.environ.get("MPH_SLAB_PERM", "default"),
              "cuts": [float(c) for c in cuts] if cuts is not None else None}
    result.update(summary(serial))
    result["per_rank"] = serial
    if args.replay:
        rep = run_ranks(args, R, axis, cuts, locals_, replay=records)
        # the replay is only meaningful while every rank ends where the recorded run did
        same = all(a["held"] == b["held"] and a["owned"] == b["owned"] for a, b in zip(serial, rep))
        result["replay"] = dict(summary(rep), consistent=same, per_rank=rep)
    print(json.dumps(result))


def summary(out):
    return {"max_rank_gpu_ms_per_step": max(o["gpu_ms_per_step"] for o in out),
            "max_rank_gpu_ms_per_step_graph": max((o.get("gpu_ms_per_step_graph") or 0.0) for o in out) or None,
            "max_rank_gpu_busy_ms_per_step": max(o["gpu_busy_ms_per_step"] or 0.0 for o in out)}


def run_ranks(args, R, axis, cuts, locals_, records=None, replay=None):
    """One run of the R rank threads: create, warm up, profile.  records: per-rank lists that
    collect the profiled steps' received messages; replay: such lists, handed to the profiled
    steps instead of the peers' messages."""
    token = Token()
    boxes = {}
    for r in range(R):
        for d, peer in (("L", (r - 1) % R), ("R", (r + 1) % R)):
            boxes[(r, peer, d)] = queue.Queue()
    out = [None] * R
    errs = []

    def run(r):
        try:
            cfg, parts, ids, n_glob = locals_[r]
            ex = InProcExchange(r, R, boxes, token)
            with token.lock:
                s = MphSolver(cfg, parts, device=0,
                              slab=solver.Slab(r, R, axis, exchange=ex, ids=ids, n_glob=n_glob, cuts=cuts))
                s.synchronize()
            with token.lock:
                s.step(args.warmup)
                s.synchronize()
            if records is not None:
                ex.record = records[r]
            if replay is not None:
                ex.replay = iter(replay[r])
            with token.lock:
                t0 = time.perf_counter()
                prof = s.profile(args.steps)
                s.synchronize()
                wall = time.perf_counter() - t0
            ex.record = ex.replay = None
            # the list kernels as graph replays (mph_profile_graphs; no exchange), as the RCCL
            # steps replay them: pass B only when it runs as one launch (overlap off)
            graph = None
            with token.lock:
                try:
                    graph = s.profile_graphs(8)
                except Exception:  # noqa: BLE001 -- older library
                    graph = None
            xcd = None   # (per-XCD wave timing: the diagnostic build of tag r05-variants)
            with token.lock:   # device copies: not beside another rank's timed work
                info = s.dist_info()
                owned = len(s.owned_ids())
            busy = prof.pop("gpu_busy", {}).get("avg_ms")   # union of the kernel intervals per step
            out[r] = {"rank": r, "owned": owned, "held": info["held"],
                      "gpu_busy_ms_per_step": busy,
                      "kernels_ms": {k: round(v["avg_ms"], 5) for k, v in prof.items()},
                      "ms_per_step": {k: round(v["avg_ms"] * v["launches"] / args.steps, 5)
                                      for k, v in prof.items()},
                      "gpu_ms_per_step": sum(v["avg_ms"] * v["launches"] for v in prof.values()) / args.steps,
                      "wall_s": wall}
            if graph is not None:
                gk = dict(out[r]["kernels_ms"])
                for k, v in graph.items():
                    if v is None or k not in gk or (k == "pass_b" and "pass_b_face" in gk):
                        continue
                    gk[k] = round(max(0.0, v - gk.get("xcd_split", 0.0)) if k == "neighbors" else v, 5)
                out[r]["kernels_ms_graph"] = gk
                out[r]["gpu_ms_per_step_graph"] = sum(gk[k] * prof[k]["launches"] for k in gk) / args.steps
            if xcd is not None:
                out[r]["xcd"] = xcd
            with token.lock:
                s.close()
        except Exception as e:  # noqa: BLE001 -- reported below
            errs.append((r, repr(e)))

    th = [threading.Thread(target=run, args=(r,)) for r in range(R)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    if errs:
        print(json.dumps({"errors": errs}))
        sys.exit(1)
    return out


if __name__ == "__main__":
    main()
