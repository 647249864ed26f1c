"""The unbatched drop-in call pattern alone (one mph_step(ctx, 1) per iteration), for kernel traces:
python tools/sync_loop.py [case] [calls]"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from particlemethod_fsi_amd import MphSolver, cases  # noqa: E402

name = sys.argv[1] if len(sys.argv) > 1 else "d1m"
calls = int(sys.argv[2]) if len(sys.argv) > 2 else 50
cfg, parts = cases.get(name).build()
with MphSolver(cfg, parts) as s:
    s.step(8)
    s.synchronize()
    t0 = time.perf_counter()
    for _ in range(calls):
        s.step(1)
    print("%s: %d calls, %.4f ms per call" % (name, calls, (time.perf_counter() - t0) * 1e3 / calls))
