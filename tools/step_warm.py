"""Consecutive timed mph_step(K) calls after a W-step warm-up on one case (default D1M): does the
first timed call pay for something later ones do not (graph first launch, clock ramp)?

  python tools/step_warm.py [case] [W] [K] [repeats]
"""
import sys
import time

sys.path.insert(0, __import__("os").path.dirname(__import__("os").path.dirname(__import__("os").path.abspath(__file__))))
from particlemethod_fsi_amd import MphSolver, cases  # noqa: E402

case = sys.argv[1] if len(sys.argv) > 1 else "d1m"
w = int(sys.argv[2]) if len(sys.argv) > 2 else 5
k = int(sys.argv[3]) if len(sys.argv) > 3 else 20
rep = int(sys.argv[4]) if len(sys.argv) > 4 else 4
cfg, parts = cases.get(case).build()
with MphSolver(cfg, parts) as s:
    s.step(w)
    s.synchronize()
    for r in range(rep):
        t0 = time.perf_counter()
        s.step(k)
        s.synchronize()
        print("call %d: %.4f ms/step" % (r, (time.perf_counter() - t0) * 1e3 / k), flush=True)
    time.sleep(0.05)
    t0 = time.perf_counter()
    s.step(k)
    s.synchronize()
    print("after 50 ms idle: %.4f ms/step" % ((time.perf_counter() - t0) * 1e3 / k), flush=True)
