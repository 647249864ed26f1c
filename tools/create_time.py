"""mph_create time with the elastic-solid lists built on the device (default) and on the host
(MPH_STRUCT_INIT=host), for the configurations with structure particles.

usage: python tools/create_time.py [case ...]   (default: bar2d_400k fsi3d)
"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    from particlemethod_fsi_amd import MphSolver, cases
    out = {}
    for name in sys.argv[1:] or ["bar2d_400k", "fsi3d"]:
        cfg, parts = cases.get(name).build()
        res = {}
        for mode in ("device", "host", "device"):   # first device run also warms the HIP runtime up
            if mode == "host":
                os.environ["MPH_STRUCT_INIT"] = "host"
            else:
                os.environ.pop("MPH_STRUCT_INIT", None)
            t0 = time.perf_counter()
            s = MphSolver(cfg, parts)
            s.synchronize()
            res[mode] = time.perf_counter() - t0
            s.close()
        out[name] = {"particles": parts.n, "mph_create_s_device_init": res["device"],
                     "mph_create_s_host_init": res["host"]}
        print(name, out[name], flush=True)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
