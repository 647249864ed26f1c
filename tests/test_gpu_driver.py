"""End to end: the drop-in executable (particlemethod_fsi_amd/lib/mph_explicit) against the
reference executable itself (oracle/_ref/mph_reference_2d_bar, built from the reference's own
src/main.cpp by oracle/Makefile) on the same .data/.grid files, same command line
(main.cpp:494-508).

Both write output.vtk, the .prof files at OutputInterval and the .vtk files at VtkOutputInterval
(main.cpp:572-683).  Compared:
  * the same file names;
  * output.vtk byte for byte (written before the first step);
  * every later .prof / .vtk section by section: integers (types, neighbour counts) exactly,
    numbers printed with %e to within one unit of their 7th significant digit (2e-6 relative)
    plus 1e-9 of the section's largest magnitude, plus the parity tests' absolute tolerances
    for the quantity (FLOORS), since many entries are pure roundoff in both runs (e.g. the
    horizontal velocity of fluid at rest, ~1e-13 m/s).
"""
import os
import subprocess

import numpy as np
import pytest

from particlemethod_fsi_amd import cases

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REF_DIR = os.path.join(ROOT, "oracle", "_ref")
REF_EXE = os.path.join(REF_DIR, "mph_reference_2d_bar")
# case -> (reference build, MPH_DIM, MPH_MODULE of the drop-in driver)
VARIANTS = {"dam2d": ("mph_reference_2d_bar", "2", "bar"),
            # the sub-stepped gate: with ElasticDt = Dt the reference solid is unstable
            "gate3d_sub": ("mph_reference_3d_dam", "3", "dam")}
DRIVER = os.path.join(ROOT, "particlemethod_fsi_amd", "lib", "mph_explicit")
# 31 steps of the results/Dam case with .prof every 10 steps and .vtk every 10 steps
RUN = {"EndTime": [0.003], "OutputInterval": [0.001], "VtkOutputInterval": [0.001]}


def write_case(d, case="dam2d"):
    c = cases.get(case)
    values = c.data()
    values.update(RUN)
    with open(os.path.join(d, "dam.data"), "w") as fh:
        fh.write(cases.data_text(values))
    with open(os.path.join(d, "dam.grid"), "w") as fh:
        fh.write(c.grid_text())


def run(exe, d, env=None):
    cmd = [exe, "dam.data", "dam.grid", "dam%03d.prof", "dam%03d.vtk", "dam.log", "4"]
    r = subprocess.run(cmd, cwd=d, env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, (exe, r.stdout[-1000:], r.stderr[-2000:])
    return sorted(f for f in os.listdir(d) if f.endswith((".vtk", ".prof")))


def sections(path):
    """-> list of (header, [token rows]): a .vtk splits at its keyword lines, a .prof into its two
    header lines and one section per column of the particle rows."""
    with open(path) as fh:
        lines = [ln.split() for ln in fh.read().splitlines()]
    if path.endswith(".prof"):
        rows = lines[2:]
        cols = [("prof col %d" % k, [[r[k]] for r in rows]) for k in range(len(rows[0]))] if rows else []
        return [("prof header", lines[:2])] + cols
    out = []
    for ln in lines:
        if ln and not _number(ln[0]):
            if out and not out[-1][1]:   # consecutive keyword lines: one header
                out[-1] = (out[-1][0] + " | " + " ".join(ln), [])
            else:
                out.append((" ".join(ln), []))
        elif ln:
            if not out:
                out.append(("", []))
            out[-1][1].append(ln)
    return out


def _number(t):
    try:
        float(t)
        return True
    except ValueError:
        return False


# absolute floors = the parity tests' tolerances for the same quantities (test_gpu_parity.py):
# positions 1e-12 m, velocities 1e-9 m/s, accelerations ~1e-9 of O(1) m/s^2, elastic tensors at
# rest (stress 1e-8 Pa, strain 1e-13); .prof columns: 1-6 positions, 7-9 velocities
FLOORS = {"POINTS": 1e-12, "displacement": 1e-12, "velocity": 1e-9, "accel": 1e-9, "stress": 1e-8,
          "strain": 1e-13, "prof col 1": 1e-12, "prof col 2": 1e-12, "prof col 3": 1e-12,
          "prof col 4": 1e-12, "prof col 5": 1e-12, "prof col 6": 1e-12, "prof col 7": 1e-9,
          "prof col 8": 1e-9, "prof col 9": 1e-9}


def compare_numeric(a_path, b_path):
    """Integers exactly; %e numbers to one unit of the 7th digit (2e-6 relative) plus a roundoff
    floor of 1e-9 of the section's largest magnitude (the parity tests' relative floors)."""
    sa, sb = sections(a_path), sections(b_path)
    assert [h for h, _ in sa] == [h for h, _ in sb], a_path
    for (h, ra), (_, rb) in zip(sa, sb):
        ta = [t for r in ra for t in r]
        tb = [t for r in rb for t in r]
        assert len(ta) == len(tb), (a_path, h)
        ints = [x.lstrip("-").isdigit() and y.lstrip("-").isdigit() for x, y in zip(ta, tb)]
        assert all(x == y for x, y, i in zip(ta, tb, ints) if i), (a_path, h)
        a = np.array([float(x) for x, i in zip(ta, ints) if not i])
        b = np.array([float(y) for y, i in zip(tb, ints) if not i])
        if not a.size:
            continue
        floor = FLOORS.get(next((k for k in FLOORS if k in h), ""), 1e-30)
        tol = 2e-6 * np.abs(b) + 1e-9 * float(np.max(np.abs(b))) + floor
        bad = np.abs(a - b) > tol
        assert not bad.any(), (a_path, h, a[bad][:3], b[bad][:3])


def test_reference_executable_runs(tmp_path):
    """CPU half of the comparison (also checks the harness builds of oracle/_ref are sane)."""
    if not os.path.exists(REF_EXE):
        pytest.skip("oracle/_ref/mph_reference_2d_bar not built (needs /root/reference)")
    d = str(tmp_path / "ref")
    os.makedirs(d)
    write_case(d)
    files = run(REF_EXE, d)
    assert "output.vtk" in files and "dam000.prof" in files and len(files) >= 6, files


@pytest.mark.gpu
@pytest.mark.parametrize("case", sorted(VARIANTS))
def test_driver_matches_reference_executable(tmp_path, case):
    exe, dim, module = VARIANTS[case]
    exe = os.path.join(REF_DIR, exe)
    if not os.path.exists(exe):
        pytest.skip("oracle/_ref reference executable not built (needs /root/reference)")
    assert os.path.exists(DRIVER), "mph_explicit not built"
    dr, dg = str(tmp_path / "ref"), str(tmp_path / "gpu")
    os.makedirs(dr)
    os.makedirs(dg)
    write_case(dr, case)
    write_case(dg, case)
    files_ref = run(exe, dr)
    # MPH_PHASE_TIMING=1: the reference's timing buckets (opt-in; the steps then run as direct
    # launches with HIP events instead of graph replays)
    env = dict(os.environ, MPH_DIM=dim, MPH_MODULE=module, MPH_PHASE_TIMING="1")
    files_gpu = run(DRIVER, dg, env)
    assert files_gpu == files_ref
    with open(os.path.join(dr, "output.vtk"), "rb") as a, open(os.path.join(dg, "output.vtk"), "rb") as b:
        assert a.read() == b.read()
    for f in files_ref:
        if f != "output.vtk":
            compare_numeric(os.path.join(dg, f), os.path.join(dr, f))
    # the reference's timing report (main.cpp:695-700): the same four buckets and two totals, the
    # GPU ones from HIP events around the directly launched steps, "other" the rest of the loop's
    # wall time; the GPU buckets must fit inside the wall times they are part of
    log = open(os.path.join(dg, "dam.log")).read()
    vals = {}
    for key in ("neighbor search:", "explicit calculation:", "virial calculation:", "other calculation:",
                "total (check):", "step loop (wall):"):
        line = next(ln for ln in log.splitlines() if ln.startswith(key))
        vals[key] = float(line[len(key):].split()[0])
    nb, ex, vi = vals["neighbor search:"], vals["explicit calculation:"], vals["virial calculation:"]
    assert nb > 0 and ex > 0 and vi > 0, vals
    assert vals["other calculation:"] >= 0.0, vals
    assert nb + ex + vi <= vals["total (check):"], vals
    assert nb + ex <= vals["step loop (wall):"] + 1e-4, vals   # GPU time of the steps inside their wall time
    # without MPH_PHASE_TIMING the driver replays the step graphs and reports no GPU buckets
    dd = str(tmp_path / "gpu_default")
    os.makedirs(dd)
    write_case(dd, case)
    assert run(DRIVER, dd, dict(os.environ, MPH_DIM=dim, MPH_MODULE=module)) == files_ref
    log = open(os.path.join(dd, "dam.log")).read()
    assert "neighbor search:" not in log and "step loop (wall):" in log


# case -> (MPH_DIM, MPH_MODULE, slab ranks) of the multi-rank driver runs
SLAB_RUNS = {"dam2d": ("2", "bar", 4), "gate2d_sub": ("2", "dam", 2)}


@pytest.mark.gpu
@pytest.mark.parametrize("case", sorted(SLAB_RUNS))
def test_driver_slab_ranks_match_single_gpu(tmp_path, case):
    """mph_explicit as N slab ranks (MPH_SLABS: forked ranks, host transport over socket pairs,
    all on the test box's one GPU) writes the files of the single-GPU driver: the same names,
    output.vtk byte for byte (the initial state), and every .prof / .vtk of the run within the
    printed precision (compare_numeric) -- the owned records of every rank gathered on rank 0 in
    original order, the virial over owned particles with the ghosts' post-step state."""
    dim, module, nslabs = SLAB_RUNS[case]
    assert os.path.exists(DRIVER), "mph_explicit not built"
    d1, dn = str(tmp_path / "one"), str(tmp_path / "slabs")
    os.makedirs(d1)
    os.makedirs(dn)
    write_case(d1, case)
    write_case(dn, case)
    env = dict(os.environ, MPH_DIM=dim, MPH_MODULE=module)
    files_one = run(DRIVER, d1, env)
    files_n = run(DRIVER, dn, dict(env, MPH_SLABS=str(nslabs), MPH_SLAB_TRANSPORT="host", MPH_SLAB_SHARE_DEVICE="1"))
    assert files_n == files_one and len(files_one) >= 6, files_n
    identical = 0
    for f in files_one:
        a, b = open(os.path.join(dn, f), "rb").read(), open(os.path.join(d1, f), "rb").read()
        if f == "output.vtk":
            assert a == b
        identical += a == b
        if a != b:
            compare_numeric(os.path.join(dn, f), os.path.join(d1, f))
    print("%s: %d of %d files byte-identical" % (case, identical, len(files_one)))
    assert identical >= 2   # output.vtk and the first .prof at least


@pytest.mark.gpu
@pytest.mark.parametrize("fail_rank", ["1", "0"])
def test_driver_slab_rank_failure_ends_the_run(tmp_path, fail_rank):
    """A slab rank that fails mid-run ends the whole run with a non-zero status instead of leaving
    the others blocked in their exchange: rank 1 failing makes rank 0 kill the other
    ranks and exit 1 (SIGCHLD); rank 0 failing takes the other ranks down with it
    (PR_SET_PDEATHSIG).  Either way every process holding the output pipes is gone within the
    timeout (subprocess.run waits for the pipes' EOF)."""
    assert os.path.exists(DRIVER), "mph_explicit not built"
    d = str(tmp_path / "fail")
    os.makedirs(d)
    write_case(d, "dam2d")
    env = dict(os.environ, MPH_DIM="2", MPH_MODULE="bar", MPH_SLABS="3", MPH_SLAB_TRANSPORT="host",
               MPH_SLAB_SHARE_DEVICE="1", MPH_FAIL_RANK=fail_rank)
    cmd = [DRIVER, "dam.data", "dam.grid", "dam%03d.prof", "dam%03d.vtk", "dam.log", "4"]
    r = subprocess.run(cmd, cwd=d, env=env, capture_output=True, text=True, timeout=120)
    assert r.returncode != 0, (r.stdout[-500:], r.stderr[-500:])
    assert "fault injection" in r.stderr or "slab rank failed" in r.stderr, r.stderr[-1000:]
