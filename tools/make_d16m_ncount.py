#!/usr/bin/env python3
"""Fixture for tests/test_gpu_d16m.py: the CPU oracle's NeighborCount of BASELINE configs[4]
(D16M, 16,205,500 particles) after creation and after steps 1, 10, 29 and 52 (the bench's
horizon) -- sum, extremes and the sha256 of the int32 array in original particle order -- so that
the GPU test checks the whole array bit for bit without the oracle on the GPU box.

The oracle (oracle/mph_oracle.c, bit-identical to the reference on every golden case) runs here
with 128-entry list rows (oracle/Makefile `oracle128`: the case's lists hold at most 80
neighbours, overflow is still detected) so its lists take 8 GB instead of 33 GB of host memory.
Writes tests/golden/d16m_ncount.json.  Run: python tools/make_d16m_ncount.py (≈ 1 min per step on
8 cores; the file is rewritten after every checkpoint).
"""
import hashlib
import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
subprocess.run(["make", "-C", os.path.join(ROOT, "oracle"), "oracle128"], check=True, capture_output=True)
os.environ["MPH_ORACLE_LIB"] = os.path.join(ROOT, "oracle", "_build", "libmph_oracle_n128.so")
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

import numpy as np  # noqa: E402

from oracle_bindings import OracleSolver  # noqa: E402
from particlemethod_fsi_amd import cases  # noqa: E402


def stats(nc):
    nc = np.ascontiguousarray(nc, np.int32)
    return {"sum": int(nc.astype(np.int64).sum()), "min": int(nc.min()), "max": int(nc.max()),
            "sha256": hashlib.sha256(nc.tobytes()).hexdigest()}


def main():
    OracleSolver.set_threads(os.cpu_count() or 1)
    t0 = time.time()
    cfg, parts = cases.get("d16m").build()
    o = OracleSolver(cfg, parts)
    n = parts.n
    del parts
    o.init()
    out = {"case": "d16m", "particles": n, "source": "oracle/mph_oracle.c (MPH_ORACLE_MAXN=128), "
           "tools/make_d16m_ncount.py", "init": stats(o.get("NeighborCount"))}
    print("init", out["init"], "%.1f s" % (time.time() - t0), flush=True)
    done = 0
    for k in (1, 10, 29, 52):
        o.step(k - done)
        done = k
        out["step%d" % k] = stats(o.get("NeighborCount"))
        print("step%d" % k, out["step%d" % k], "%.1f s" % (time.time() - t0), flush=True)
        with open(os.path.join(ROOT, "tests", "golden", "d16m_ncount.json"), "w") as fh:
            json.dump(out, fh, indent=1)


if __name__ == "__main__":
    main()
