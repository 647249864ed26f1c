"""sha256 of every state field after a few steps, for bitwise A/B comparison of builds
(MPH_GPU_LIB selects the library).  usage: python tools/state_hash.py case steps"""
import hashlib
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    case, steps = sys.argv[1], int(sys.argv[2])
    from particlemethod_fsi_amd import MphSolver, cases
    cfg, parts = cases.get(case).build()
    out = {}
    with MphSolver(cfg, parts) as s:
        s.step(steps)
        for f in ("Position", "Velocity", "PressureP", "PressureA", "GravityCenter", "Force", "DensityA",
                  "NeighborCount", "DivergenceP"):
            out[f] = hashlib.sha256(s.get(f).tobytes()).hexdigest()[:16]
    print(json.dumps({"case": case, "steps": steps, "lib": os.environ.get("MPH_GPU_LIB", "default"), **out}))


if __name__ == "__main__":
    main()
