"""Sanitizers on the host layer (CPU only): the C++ readers, writers, derived constants and
elastic-solid initialisation of libmph_gpu.so, compiled with -fsanitize=address,undefined into a
small driver (tests/native/host_asan.cpp) and run on every parity case.  (GPU ASan is not
available on the MI355X pool; the device side is covered by the parity tests.)"""
import os
import shutil
import subprocess

import pytest

from oracle_bindings import write_case_files
from particlemethod_fsi_amd import cases

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def asan_binary(tmp_path_factory):
    if shutil.which("g++") is None:
        pytest.skip("g++ not available")
    out = str(tmp_path_factory.mktemp("asan") / "host_asan")
    cmd = ["g++", "-std=c++17", "-O1", "-g", "-fsanitize=address,undefined", "-fno-omit-frame-pointer",
           "-fno-sanitize-recover=all", "-ffp-contract=off", "-D__HIP_PLATFORM_AMD__", "-I/opt/rocm/include",
           os.path.join(ROOT, "tests", "native", "host_asan.cpp"),
           os.path.join(ROOT, "particlemethod_fsi_amd", "csrc", "mph_host.cpp"), "-o", out]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        pytest.skip("sanitizer build unavailable: " + r.stderr[-500:])
    return out


@pytest.mark.parametrize("case", ["dam2d", "bar2d", "gate2d", "box3d", "gate3d"])
def test_host_layer_under_asan_ubsan(asan_binary, case, tmp_path):
    c = cases.get(case)
    dp, gp = write_case_files(cases.data_text(c.data()), c.grid_text(), str(tmp_path))
    r = subprocess.run([asan_binary, dp, gp, str(c.dim), str({"bar": 0, "dam": 1}[c.module]),
                        str(tmp_path / "out.txt")], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    assert "runtime error" not in r.stderr
