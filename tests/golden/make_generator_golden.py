"""Golden .grid digests of the reference particle generator (TEST INFRASTRUCTURE).

Runs oracle/_ref/mph_reference_generator (the reference's generator/ sources compiled by
oracle/Makefile, never copied here) on every tests/golden/boid/*.boid and records the sha256 and
particle count of the .grid it writes (generator.cpp:839-862) in tests/golden/generator_grids.json,
so tests/test_host_io.py can check the in-repo generator (mphio.generate + format_grid) without
/root/reference.

  make -C oracle ref && python tests/golden/make_generator_golden.py
"""
import glob
import hashlib
import json
import os
import shutil
import subprocess
import tempfile

HERE = os.path.dirname(os.path.abspath(__file__))
GEN = os.path.join(HERE, "..", "..", "oracle", "_ref", "mph_reference_generator")


def reference_grid(boid_path: str) -> str:
    """Text of the .grid the reference generator writes for boid_path (run in a scratch dir)."""
    with tempfile.TemporaryDirectory() as d:
        shutil.copy(boid_path, os.path.join(d, "case.boid"))
        subprocess.run([os.path.abspath(GEN), "case"], cwd=d, stdout=subprocess.DEVNULL,
                       stderr=subprocess.DEVNULL, check=True)
        return open(os.path.join(d, "case.grid")).read()


def main():
    out = {}
    for p in sorted(glob.glob(os.path.join(HERE, "boid", "*.boid"))):
        t = reference_grid(p)
        out[os.path.basename(p)] = {"sha256": hashlib.sha256(t.encode()).hexdigest(),
                                    "n": int(t.splitlines()[1].split()[0])}
    with open(os.path.join(HERE, "generator_grids.json"), "w") as fh:
        json.dump(out, fh, indent=1, sort_keys=True)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
