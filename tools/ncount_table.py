"""NeighborCount total after every step of a single-GPU run (the reference for bench.py's
multi-rank correctness check, profiles/<case>_ncount_sum.json).

usage: python tools/ncount_table.py [case] [steps] [out.json]
"""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    case = sys.argv[1] if len(sys.argv) > 1 else "d16m"
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else 200
    out = sys.argv[3] if len(sys.argv) > 3 else os.path.join(ROOT, "profiles", "%s_ncount_sum.json" % case)
    from particlemethod_fsi_amd import MphSolver, cases
    cfg, parts = cases.get(case).build()
    n = parts.n
    sums = []
    with MphSolver(cfg, parts) as s:
        del parts
        sums.append(int(s.get("NeighborCount").astype(np.int64).sum()))
        for k in range(steps):
            s.step(1)
            sums.append(int(s.get("NeighborCount").astype(np.int64).sum()))
            if k % 20 == 0:
                print("step", k + 1, sums[-1], flush=True)
    with open(out, "w") as fh:
        json.dump({"case": case, "particles": n, "generator": "tools/ncount_table.py (one MI355X, mph_step(1) "
                   "per step)", "sum_after_steps": sums}, fh)
    print("wrote", out, len(sums))


if __name__ == "__main__":
    main()
