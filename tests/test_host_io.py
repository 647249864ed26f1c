"""Host layer (no device): the C ABI library loads and exports every declared symbol; the
reference's file formats (.data, .grid, .prof, .vtk) and derived constants are reproduced."""
import ctypes
import gzip
import hashlib
import os
import re
import sys
import tempfile

import numpy as np
import pytest

from golden_utils import Golden
from particlemethod_fsi_amd import cases, mphio, solver

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "mph_gpu.h")


def declared_symbols():
    txt = open(HEADER).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    return sorted(set(re.findall(r"\b(mph_[a-z0-9_]+)\s*\(", txt)))


def test_library_exports_every_declared_symbol():
    L = solver.load_library()
    names = declared_symbols()
    assert len(names) >= 20
    for name in names:
        assert hasattr(L, name), name
    assert sorted(solver.EXPORTED_SYMBOLS) == names


def test_config_struct_layout_matches_header():
    # offsets of the ctypes mirror equal the C struct (checked through mph_config_default)
    L = solver.load_library()
    cfg = mphio.MphConfig()
    assert L.mph_config_default(ctypes.byref(cfg), 3, 1) == 0
    assert cfg.dim == 3 and cfg.module == 1 and cfg.dt == 1e100 and cfg.elastic_dt == 1e100
    assert ctypes.sizeof(mphio.MphConfig) == 8 + 8 * (8 + 7 * 6 + 36 + 3 + 3 * 18 + 2 + 6) + 8
    assert ctypes.sizeof(mphio.MphConfig) == L.mph_config_sizeof()


def _write_case(case, tmp):
    c = cases.get(case)
    dp, gp = os.path.join(tmp, "c.data"), os.path.join(tmp, "c.grid")
    open(dp, "w").write(cases.data_text(c.data()))
    open(gp, "w").write(c.grid_text())
    return c, dp, gp


@pytest.mark.parametrize("case", ["dam2d", "gate2d", "box3d"])
def test_cpp_reader_matches_python_reader(case):
    with tempfile.TemporaryDirectory() as tmp:
        c, dp, gp = _write_case(case, tmp)
        cfg_c, p_c = solver.read_case_files(dp, gp, c.dim, c.module)
        cfg_p = mphio.config_default(c.dim, c.module)
        mphio.read_data_file(dp, cfg_p)
        p_p = mphio.read_grid_file(gp, cfg_p)
        assert bytes(cfg_c) == bytes(cfg_p)
        for a, b in ((p_c.property, p_p.property), (p_c.position, p_p.position),
                     (p_c.initial_position, p_p.initial_position), (p_c.velocity, p_p.velocity)):
            assert np.array_equal(a, b)
        # and both equal the in-memory case the benchmarks use
        cfg_m, p_m = c.build()
        assert bytes(cfg_m) == bytes(cfg_c)
        assert np.array_equal(p_m.position, p_c.position)


@pytest.mark.parametrize("case", ["dam2d", "gate2d", "bar2d", "box3d", "gate3d"])
def test_derived_constants_bit_identical_to_reference(case):
    cfg, _ = cases.get(case).build()
    assert np.array_equal(solver.derive_scalars(cfg), Golden(case).z["scalars"])


def test_generator_reproduces_reference_dam_grid():
    ref = "/root/reference/results/Dam/dam.grid"
    txt = cases.get("dam2d").grid_text()
    if os.path.exists(ref):
        assert txt == open(ref).read()
    # independent of /root/reference: the golden .prof at step 0 holds the same particles
    prof = gzip.open(os.path.join(ROOT, "tests", "golden", "dam2d_000.prof.gz")).read().decode()
    body_grid = [l.split() for l in txt.splitlines()[2:]]
    body_prof = [l.split() for l in prof.splitlines()[2:]]
    assert len(body_grid) == len(body_prof) == 6650
    assert all(float(a[1]) == float(b[1]) and a[0] == b[0] for a, b in zip(body_grid, body_prof))


def test_prof_and_vtk_writers_byte_identical_at_step0():
    g = Golden("dam2d")
    cfg, p = cases.get("dam2d").build()
    n = p.n
    L = solver.load_library()
    zeros3 = np.zeros((n, 3))
    zeros9 = np.zeros((n, 3, 3))
    isnc = np.zeros(n, np.int32)
    nc = np.ascontiguousarray(g.get(0, "NeighborCount"), np.int32)
    with tempfile.TemporaryDirectory() as tmp:
        vtk = os.path.join(tmp, "output.vtk")
        rc = L.mph_write_vtk_arrays(vtk.encode(), n, p.property.ctypes.data, p.position.ctypes.data,
                                    p.initial_position.ctypes.data, p.velocity.ctypes.data,
                                    zeros3.ctypes.data, zeros3.ctypes.data, zeros9.ctypes.data,
                                    zeros9.ctypes.data, isnc.ctypes.data, nc.ctypes.data)
        assert rc == 0
        raw = open(vtk, "rb").read()
        assert hashlib.sha256(raw).digest() == bytes(g.z["sha256/output.vtk"])
        prof = os.path.join(tmp, "dam000.prof")
        rc = L.mph_write_prof_arrays(prof.encode(), ctypes.byref(cfg), 0.0, n, p.property.ctypes.data,
                                     p.position.ctypes.data, p.initial_position.ctypes.data,
                                     p.velocity.ctypes.data)
        assert rc == 0
        assert hashlib.sha256(open(prof, "rb").read()).digest() == bytes(g.z["sha256/dam000.prof"])


def test_data_reader_keeps_partial_lists_and_ignores_unknown_lines():
    with tempfile.TemporaryDirectory() as tmp:
        dp = os.path.join(tmp, "x.data")
        open(dp, "w").write("# c\nDt 2e-4\nDensity 1 2 3\nFoo 1 2\nGravity 0 -9.8 0\n"
                            "Wall6  Center 1 2 3 Velocity 4 5 6 Omega 7 8 9\n")
        cfg = mphio.MphConfig()
        L = solver.load_library()
        L.mph_config_default(ctypes.byref(cfg), 2, 0)
        assert L.mph_read_data_file(dp.encode(), ctypes.byref(cfg)) == 0
        cfg2 = mphio.config_default(2, 0)
        mphio.read_data_file(dp, cfg2)
        assert bytes(cfg) == bytes(cfg2)
        assert cfg.dt == 2e-4 and list(cfg.density)[:3] == [1.0, 2.0, 3.0]
        assert list(cfg.wall_omega[4]) == [7.0, 8.0, 9.0] and cfg.gravity[1] == -9.8


@pytest.mark.parametrize("case", ["bar2d", "gate2d", "gate3d"])
def test_structure_init_matches_reference(case):
    """calculateInitialNeighbor / Lamesconstant / Normalizer as done by mph_create (host)."""
    g = Golden(case)
    cfg, p = cases.get(case).build()
    n = p.n
    L = solver.load_library()
    isnc = np.zeros(n, np.int32)
    N = np.zeros((n, 3, 3))
    ll, lm = np.zeros(n), np.zeros(n)
    assert L.mph_structure_init(ctypes.byref(cfg), n, p.property.ctypes.data,
                                p.initial_position.ctypes.data, isnc.ctypes.data, N.ctypes.data,
                                ll.ctypes.data, lm.ctypes.data) == 0
    assert np.array_equal(isnc, g.get(0, "InitialStructureNeighborCount"))
    assert np.array_equal(ll[g.solid], g.get(0, "LambdaLames"))
    assert np.array_equal(lm[g.solid], g.get(0, "MuLames"))
    ref = g.get(0, "Normalizer")
    # neighbour sums in slot order instead of the reference's cell-scan order: reassociation only
    assert np.max(np.abs(N[g.solid] - ref)) <= 1e-12 * np.max(np.abs(ref))


def _vtk_reference_format(n, prop, pos, pos0, vel, acc, force, stress, strain, isnc, nc):
    """writeVtkFile's byte layout (main.cpp:984-1189) restated in Python (test-only), for sizes
    where the library formats the sections in parallel."""
    f32 = lambda a: a.astype(np.float32).astype(np.float64)
    out = []
    v3 = lambda a: "".join("%e %e %e\n" % tuple(r) for r in f32(a).reshape(n, 3).tolist())
    out.append("# vtk DataFile Version 2.0\nUnstructured Grid Example\nASCII\nDATASET UNSTRUCTURED_GRID\n")
    out.append("POINTS %d float\n" % n + v3(pos))
    out.append("CELLS %d %d\n" % (n, 2 * n) + "".join("1 %d " % i for i in range(n)) + "\n")
    out.append("CELL_TYPES %d\n" % n + "1 " * n + "\n\n")
    out.append("POINT_DATA %d\nSCALARS label float 1\nLOOKUP_TABLE default\n" % n)
    out.append("".join("%d\n" % t for t in prop.tolist()) + "\n\n")
    out.append("VECTORS displacement float\n" + v3(pos - pos0))
    for m, tag in ((stress, "stress"), (strain, "strain")):
        mm = f32(m).reshape(n, 9)
        for a in range(3):
            for b in range(3):
                out.append("\n SCALARS %s%d%d float \nLOOKUP_TABLE default\n" % (tag, a, b))
                out.append("".join("%e\n" % x for x in mm[:, 3 * a + b].tolist()))
    out.append("VECTORS velocity float\n" + v3(vel) + "\n")
    out.append("VECTORS accel float\n" + v3(acc) + "\n")
    out.append("SCALARS Initialneighbor float 1\nLOOKUP_TABLE default\n" + "".join("%d\n" % t for t in isnc.tolist()))
    out.append("SCALARS neighbor float 1\nLOOKUP_TABLE default\n" + "".join("%d\n" % t for t in nc.tolist()))
    out.append("VECTORS velocity float\n" + v3(vel) + "\n")
    out.append("VECTORS force float\n" + v3(force) + "\n")
    return "".join(out).encode()


def test_vtk_writer_parallel_sections_byte_identical():
    """Above 2 x 65536 particles mph_write_vtk_arrays formats each section on several threads; the
    file must still be the reference's sequential byte stream."""
    n = 150_000
    rng = np.random.default_rng(7)
    prop = rng.integers(0, 6, n).astype(np.int32)
    arrs = [rng.normal(size=(n, 3)) * 10.0 ** rng.integers(-6, 3, (n, 1)) for _ in range(5)]
    pos, pos0, vel, acc, force = arrs
    stress, strain = rng.normal(size=(n, 3, 3)) * 1e4, rng.normal(size=(n, 3, 3)) * 1e-4
    isnc = rng.integers(0, 40, n).astype(np.int32)
    nc = rng.integers(0, 90, n).astype(np.int32)
    L = solver.load_library()
    with tempfile.TemporaryDirectory() as tmp:
        path = os.path.join(tmp, "big.vtk")
        rc = L.mph_write_vtk_arrays(path.encode(), n, prop.ctypes.data, pos.ctypes.data, pos0.ctypes.data,
                                    vel.ctypes.data, acc.ctypes.data, force.ctypes.data, stress.ctypes.data,
                                    strain.ctypes.data, isnc.ctypes.data, nc.ctypes.data)
        assert rc == 0
        raw = open(path, "rb").read()
    assert raw == _vtk_reference_format(n, prop, pos, pos0, vel, acc, force, stress, strain, isnc, nc)


@pytest.mark.parametrize("case", ["dam2d", "gate3d", "bar2d"])
def test_binary_grid_roundtrip(case):
    """mph_write_grid_binary -> mph_read_grid_header/_particles (magic-detected) returns exactly
    what the ASCII .grid gave, so a binary grid is a drop-in for the reference's input file."""
    with tempfile.TemporaryDirectory() as tmp:
        c, dp, gp = _write_case(case, tmp)
        cfg_t, p_t = solver.read_case_files(dp, gp, c.dim, c.module)
        gb = os.path.join(tmp, "c.gridb")
        solver.write_grid_binary(gb, cfg_t, p_t)
        cfg_b, p_b = solver.read_case_files(dp, gb, c.dim, c.module)
        assert bytes(cfg_b) == bytes(cfg_t)
        for a, b in ((p_t.property, p_b.property), (p_t.position, p_b.position),
                     (p_t.initial_position, p_b.initial_position), (p_t.velocity, p_b.velocity)):
            assert np.array_equal(a, b)
        assert os.path.getsize(gb) == 80 + 4 * (p_t.n + (p_t.n & 1)) + 72 * p_t.n


def test_vtu_writer_roundtrip():
    """mph_write_vtu_arrays (binary VTK XML): every field of the ASCII writer,
    read back with solver.read_vtu, equals its float32 / int32 value exactly; the XML header
    declares one VTK_VERTEX cell per particle."""
    n = 1000
    rng = np.random.default_rng(3)
    prop = rng.integers(0, 6, n).astype(np.int32)
    pos, pos0, vel, acc, force = [rng.normal(size=(n, 3)) for _ in range(5)]
    stress, strain = rng.normal(size=(n, 3, 3)) * 1e4, rng.normal(size=(n, 3, 3)) * 1e-4
    isnc = rng.integers(0, 40, n).astype(np.int32)
    nc = rng.integers(0, 90, n).astype(np.int32)
    L = solver.load_library()
    with tempfile.TemporaryDirectory() as tmp:
        path = os.path.join(tmp, "out.vtu")
        rc = L.mph_write_vtu_arrays(path.encode(), n, prop.ctypes.data, pos.ctypes.data, pos0.ctypes.data,
                                    vel.ctypes.data, acc.ctypes.data, force.ctypes.data, stress.ctypes.data,
                                    strain.ctypes.data, isnc.ctypes.data, nc.ctypes.data)
        assert rc == 0
        d = solver.read_vtu(path)
        head = open(path, "rb").read(2048)
    assert b'NumberOfPoints="1000" NumberOfCells="1000"' in head
    f32 = lambda a: a.astype(np.float32)  # noqa: E731
    np.testing.assert_array_equal(d["Points"], f32(pos))
    np.testing.assert_array_equal(d["displacement"], f32(pos - pos0))
    np.testing.assert_array_equal(d["stress"], f32(stress.reshape(n, 9)))
    np.testing.assert_array_equal(d["strain"], f32(strain.reshape(n, 9)))
    for k, a in (("velocity", vel), ("accel", acc), ("force", force)):
        np.testing.assert_array_equal(d[k], f32(a))
    np.testing.assert_array_equal(d["label"], prop)
    np.testing.assert_array_equal(d["Initialneighbor"], isnc)
    np.testing.assert_array_equal(d["neighbor"], nc)
    np.testing.assert_array_equal(d["connectivity"], np.arange(n))
    np.testing.assert_array_equal(d["offsets"], np.arange(1, n + 1))
    assert (d["types"] == 1).all()


def test_generator_tool(tmp_path):
    """tools/generate.py: the ASCII .grid is the case's generator text, and the
    binary grid reads back to the same particles."""
    import subprocess
    import sys
    tool = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools", "generate.py")
    g, gb, dp = str(tmp_path / "c.grid"), str(tmp_path / "c.gridb"), str(tmp_path / "c.data")
    for extra in ([g, "--data", dp], [gb, "--binary"]):
        r = subprocess.run([sys.executable, tool, "--case", "gate2d"] + extra, capture_output=True, text=True)
        assert r.returncode == 0, r.stderr
    c = cases.get("gate2d")
    assert open(g).read() == c.grid_text()
    _, p_t = solver.read_case_files(dp, g, c.dim, c.module)
    _, p_b = solver.read_case_files(dp, gb, c.dim, c.module)
    for a, b in ((p_t.property, p_b.property), (p_t.position, p_b.position), (p_t.velocity, p_b.velocity)):
        np.testing.assert_array_equal(a, b)


# --- generator shapes (generator.cpp:154-175 parsing, 654-835 lattices) -------------------------

BOID_DIR = os.path.join(ROOT, "tests", "golden", "boid")
REF_GEN = os.path.join(ROOT, "oracle", "_ref", "mph_reference_generator")


@pytest.mark.parametrize("name", ["shapes2d.boid", "shapes3d.boid"])
def test_generator_shapes_byte_identical(name):
    """Every shape of the reference generator (Cuboid, Cuboid2, Cyboid, Cyboid2, Recboid,
    Recboid2; interleaved in the file, emitted grouped by shape like genparticle): the .grid text
    of mphio equals the reference generator's -- against the committed digest of its output
    (tests/golden/make_generator_golden.py) and, where it is built here, against a live run."""
    import json
    text = open(os.path.join(BOID_DIR, name)).read()
    spacing, lower, upper, blocks = mphio.parse_boid(text)
    assert {b.kind for b in blocks} == set(mphio.SHAPES)
    grid = mphio.format_grid(mphio.generate(blocks), spacing, lower, upper)
    gold = json.load(open(os.path.join(ROOT, "tests", "golden", "generator_grids.json")))[name]
    assert int(grid.splitlines()[1].split()[0]) == gold["n"]
    assert hashlib.sha256(grid.encode()).hexdigest() == gold["sha256"]
    if os.path.exists(REF_GEN):
        sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))
        from make_generator_golden import reference_grid
        assert grid == reference_grid(os.path.join(BOID_DIR, name))


def test_generator_shapes_slab_window_and_planes():
    """Slab-local creation of the non-cuboid shapes: the window's particles and their original
    indices are those of the full set, and the plane counts add up to it."""
    _, _, _, blocks = mphio.parse_boid(open(os.path.join(BOID_DIR, "shapes3d.boid")).read())
    full = mphio.generate(blocks)
    parts, ids, n = mphio.generate_window(blocks, 2, -0.01, 0.02, -0.1, 0.2)
    assert n == full.n and len(ids) == parts.n > 0
    np.testing.assert_array_equal(parts.position, full.position[ids])
    z = full.position[:, 2]
    assert parts.n == int(((z >= -0.01) & (z < 0.02)).sum())
    v, c = mphio.plane_counts(blocks, 2, -0.1, 0.2)
    assert int(c.sum()) == full.n and np.all(np.diff(v) > 0)


@pytest.mark.parametrize("bad,msg", [
    ("StartSphere\n Spacing 0.001\nEndSphere\n", "unknown block"),
    ("StartCuboid\n Spacing 0.001\n Type 1\n RigidType 0\n Lower 0 0 0\n Upper 1 1 1\n Velocity 0 0 0\n"
     "EndCuboid\n", "missing Enthalpy"),
    ("StartCyboid2\n Spacing 0.001\n Type 1\n Colour 3\nEndCyboid2\n", "no such indication"),
    ("StartRecboid\n Spacing 0.001\n", "without EndRecboid"),
])
def test_boid_parser_refuses_what_the_generator_would_drop(bad, msg):
    """The reference generator silently skips an unknown Start* block and stops reading at a
    malformed one (writing the particles read so far); parse_boid raises instead."""
    head = "ParticleDistance 0.001\nLowerDomain 0 0 0\nUpperDomain 1 1 1\n"
    with pytest.raises(mphio.BoidError, match=msg):
        mphio.parse_boid(head + bad)


def test_search_uncounted_loads_land_before_use(tmp_path):
    """The search issues its start[] loads in inline asm, which hipcc does not count
    (mph_kernels.hip start_load2): on every control-flow path from such a load to the next
    s_waitcnt vmcnt(0) no instruction may read, copy or overwrite its destination register
    (tools/asm_load_audit.py over the gfx950 assembly of every k_neighbors instantiation)."""
    import shutil
    import subprocess
    hipcc = shutil.which("hipcc") or "/opt/rocm/bin/hipcc"
    if not os.path.exists(hipcc):
        pytest.skip("hipcc not available")
    csrc = os.path.join(ROOT, "particlemethod_fsi_amd", "csrc")
    asm = str(tmp_path / "kernels.s")
    subprocess.run([hipcc, "-O3", "-std=c++17", "-I" + os.path.join(ROOT, "include"), "--offload-arch=gfx950",
                    "-munsafe-fp-atomics", "--cuda-device-only", "-S", os.path.join(csrc, "mph_kernels.hip"),
                    "-o", asm], check=True, capture_output=True, timeout=600)
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "asm_load_audit.py"), asm, "k_neighbors"],
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0 and "clean" in r.stdout, r.stdout[-2000:]
