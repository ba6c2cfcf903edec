"""TOML front end on the reference's own input files (fixtures in
tests/golden/res/). CPU only, except the last test.

Each supported file must give exactly the scene the reference's parse_params +
setup_simulation build -- compared node for node with the Python restatements of the
setupGeometry builders (which the oracle KATs pin) -- and each file the reference rejects
must be rejected with the reference's reason."""
import ctypes as C
import math
import os

import numpy as np
import pytest

from rsmcrt_amd import abi, builders, scene
from rsmcrt_amd.engine import SmcrtError
from rsmcrt_amd.job import Job

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
RES = os.path.join(GOLDEN, "res")


def res(name):
    return os.path.join(RES, name)


def node_bytes(arr, n):
    return [bytes(memoryview(arr[i]).cast("B")) for i in range(n)]


def same_scene(job, sc):
    assert job.desc.n_nodes == len(sc.nodes) and job.desc.n_top == sc.n_top
    assert list(job.top[:job.desc.n_top]) == list(sc.top)
    assert node_bytes(job.nodes, job.desc.n_nodes) == node_bytes(sc.node_array(), len(sc.nodes))


def same_struct(a, b):
    return bytes(memoryview(a).cast("B")) == bytes(memoryview(b).cast("B"))


def test_scat_test():  # res/scat_test.toml
    j = Job(res("scat_test.toml"))
    same_scene(j, builders.setup_scat_test(10.0))
    d = j.desc
    assert (d.grid.nx, d.grid.ny, d.grid.nz, d.grid.xmax) == (200, 200, 200, 1.0)
    assert d.n_photons == 100000 and d.seed == 123456789 and d.source.kind == abi.SRC_POINT
    assert d.flags == abi.FLAG_PATHLENGTH and d.overwrite == 1 and j.experiment == "scat_test"


def test_scat_test2_pencil():
    j = Job(res("scat_test2.toml"))
    same_scene(j, builders.setup_scat_test2(10.0, 0.9))  # hgg = [0.9] -> hgg%   1
    s = j.desc.source
    assert s.kind == abi.SRC_PENCIL and list(s.dir) == [0.0, 0.0, 1.0] and list(s.pos) == [0.0, 0.0, 0.0]
    assert j.desc.grid.xmax == 100.0


def test_aptran_uniform_vector_direction():
    j = Job(res("aptran.toml"))
    same_scene(j, builders.setup_tran_and_jacques())
    s = j.desc.source
    # the vector direction is applied and the corners read (the reference returns early
    # here and crashes later, parse_source.f90:145-159)
    assert s.kind == abi.SRC_UNIFORM and list(s.dir) == [0.0, 0.0, -1.0]
    assert list(s.p1) == [-0.25, 0.0, 0.99999] and list(s.p2) == [0.5, 0.0, 0.0] and list(s.p3) == [0.0, 0.0, 0.0]


def test_validation1_box_and_circle_detectors():
    j = Job(res("validation1.toml"))
    same_scene(j, builders.setup_box(90.0, 10.0, 0.75, 1.0, (100.0, 100.0, 0.02), (100.0, 100.0, 0.03)))
    want = [scene.circle_dect((0.0, 0.0, -0.01), (0.0, 0.0, -1.0), 1, 20.0, 100),
            scene.circle_dect((0.0, 0.0, 0.01), (0.0, 0.0, 1.0), 1, 20.0, 100)]
    assert all(same_struct(a, b) for a, b in zip(j.detectors, want))
    assert j.desc.flags == abi.FLAG_PATHLENGTH | abi.FLAG_RENDER_SOURCE


def test_detector_kinds_and_grouping():
    j = Job(res("test_dects.toml"))
    same_scene(j, builders.setup_scat_test(10.0))
    want = [scene.circle_dect((-1.0, 0.0, 0.0), (-1.0, 0.0, 0.0), 4, 0.5, 10),
            scene.annulus_dect((-1.0, 0.0, 0.0), (-1.0, 0.0, 0.0), 3, 0.5, 1.0, 10),
            scene.camera((-1.0, -1.0, -1.0), (0.0, 2.0, 0.0), (0.0, 0.0, 2.0), 2, 10, 5000.0)]
    assert all(same_struct(a, b) for a, b in zip(j.detectors, want))
    # parse_detectors.f90:100-115 orders circles, annuli, fibres, cameras
    kinds = [d.kind for d in Job(res("default.toml")).detectors]
    assert kinds == sorted(kinds)


def test_omg_csg_model():
    same_scene(Job(res("omg.toml")), builders.setup_omg_sdf())


def test_sphere_scene_build_defined_list():
    j = Job(res("sphere.toml"))
    assert j.desc.n_top == 41 and j.experiment == "sphere_scene"
    spheres = []
    for i in range(40):
        nd = j.nodes[i]
        r = nd.param[0]
        c = (-nd.transform[3], -nd.transform[7], -nd.transform[11])
        assert 0.001 <= r < 0.25 and all(-1.0 + r <= x <= 1.0 - r for x in c)
        spheres.append((r, *c))
    same_scene(j, builders.setup_sphere_scene(spheres))
    assert Job(res("sphere.toml")).nodes[7].param[0] == j.nodes[7].param[0]  # deterministic


def test_egg_revolution_modifiers():
    """egg_test.toml: setup_egg (setupGeometry.f90:149-248), two Moss eggs revolved about the
    y axis (the revolution modifier, sdfModifiers.f90:286-303), a yolk sphere and a bounding
    box; numOptProp = 3 with the default mus = 1, mua = 0, hgg = 0, n = 1 of each layer."""
    j = Job(res("egg_test.toml"))
    assert j.experiment == "egg" and j.desc.n_top == 4
    same_scene(j, builders.setup_egg([1.0] * 3, [0.0] * 3, [0.0] * 3, [1.0] * 3, (0.0, 0.0, 0.0), (5.0, 5.0, 5.0),
                                     2.0, 1.5, 1.4, 0.02, 1.0))
    assert [j.nodes[i].kind for i in range(6)] == [abi.SDF_SPHERE, abi.SDF_REVOLUTION, abi.SDF_REVOLUTION, abi.SDF_BOX,
                                                   abi.SDF_EGG, abi.SDF_EGG]
    meta = dict(l.split(" = ", 1) for l in j.metadata().strip().splitlines())
    assert meta["BottomSphereRadius"] == "2.0" and meta["ShellThickness"] == "0.02" and meta["YolkRadius"] == "1.0"


def _vessel_case(tmp_path, n_nodes, extra_edges, seed=7):
    from tests.golden.make_vessel_data import write_vessel_data
    edges, nodes, radii = write_vessel_data(tmp_path, n_nodes, seed, extra_edges)
    read = np.zeros_like(nodes)
    n_read = min(len(edges), len(nodes))  # setupGeometry.f90:615 loops to the edge count
    read[:n_read] = nodes[:n_read]
    return Job(str(tmp_path / "vessels.toml")), builders.get_vessels(edges, read, radii), edges, nodes


@pytest.mark.parametrize("extra_edges", [0, 9])
def test_vessels_get_vessels(tmp_path, extra_edges):
    """res/vessels.toml with a data set beside it (tests/golden/make_vessel_data.py): get_vessels
    (setupGeometry.f90:552-652) gives one capsule per edge plus the .32 x .18 x .26 dermis box,
    node for node equal to builders.get_vessels on the values the reference's reads leave. A
    tree (E = N - 1) leaves the last node unread (the :615 bound); with extra edges every node
    is read. The file mixes blank and comma separators, d exponents and a record split."""
    j, sc, edges, nodes = _vessel_case(tmp_path, 40, extra_edges)
    same_scene(j, sc)
    assert j.experiment == "vessels" and j.desc.n_top == len(edges) + 1
    caps = [j.nodes[i] for i in range(len(edges))]
    assert all(c.kind == abi.SDF_CAPSULE and c.layer == 1 and (c.mus, c.mua, c.hgg, c.n) == (94.0, 231.0, 0.9, 1.37)
               for c in caps)
    bx = j.nodes[len(edges)]
    assert bx.kind == abi.SDF_BOX and bx.layer == 2 and list(bx.param[:3]) == [0.16, 0.09, 0.13]
    assert (bx.mus, bx.mua) == (357.0, 0.458)
    # the rescale of :629-639, checked on one capsule end by hand
    mx = np.abs(nodes[:min(len(edges), len(nodes))]).max(axis=0)
    e1 = int(edges[0][0]) - 1
    want = [(nodes[e1][k] / mx[k] - 0.5) * mx[k] * 0.001 if e1 < len(edges) else -0.5 * mx[k] * 0.001
            for k in range(3)]
    assert list(caps[0].param[:3]) == want
    s = j.desc.source
    assert s.kind == abi.SRC_UNIFORM and list(s.dir) == [0.0, 0.0, -1.0] and list(s.p1) == [-0.16, -0.09, 0.129999]
    if extra_edges == 0:  # the unread last node sits at -max/2 * res on every axis
        last = len(nodes) - 1
        ends = [c for c, (a, b) in zip(caps, edges) if b - 1 == last]
        assert ends and list(ends[0].param[3:6]) == [-0.5 * mx[k] * 0.001 for k in range(3)]


def test_vessels_missing_or_bad_data(tmp_path):
    """Without the data files the front end names the file it could not read; a bad edge
    index (an out-of-bounds read in the reference) is refused."""
    with pytest.raises(SmcrtError) as e:
        Job(res("vessels.toml"))
    assert abi.STATUS_NAMES[abi.ERR_INVALID_ARG] in str(e.value) and "edges.dat" in str(e.value)
    from tests.golden.make_vessel_data import write_vessel_data
    write_vessel_data(tmp_path, 10, 3)
    with open(tmp_path / "edges.dat", "a") as f:
        f.write("1 11\n")
    with pytest.raises(SmcrtError, match="outside 1..10"):
        Job(str(tmp_path / "vessels.toml"))
    (tmp_path / "radii.dat").unlink()
    with pytest.raises(SmcrtError, match="radii.dat"):
        Job(str(tmp_path / "vessels.toml"))


@pytest.mark.gpu
def test_vessels_job_runs_bit_exact(tmp_path):
    """The vessels scene get_vessels builds, run through the HIP engine at 64^3 with
    res/vessels.toml's uniform source, bit-exact against the oracle."""
    from oracle import pyoracle as O
    from rsmcrt_amd.engine import Engine
    j, _, _, _ = _vessel_case(tmp_path, 40, 0)
    d = j.desc
    sc = scene.Scene([])
    sc.nodes = [j.nodes[i] for i in range(d.n_nodes)]
    sc.top = list(j.top[:d.n_top])
    g = scene.grid(64, 64, 64, d.grid.xmax, d.grid.ymax, d.grid.zmax)
    n = 3000
    with Engine(sc, g) as eng:
        gpu = eng.run(d.source, n, seed=d.seed, records=True)
    cpu = O.run(sc, g, d.source, n, seed=d.seed, records=True)
    assert gpu.counters_dict() == cpu.counters_dict()
    assert np.array_equal(gpu.records, cpu.records)
    assert np.array_equal(gpu.absorb, cpu.absorb)
    np.testing.assert_allclose(gpu.jmean, cpu.jmean, rtol=1e-12, atol=1e-15)
    assert cpu.counter("absorbed") > 0


@pytest.mark.parametrize("name,code,why", [
    ("logo.toml", abi.ERR_UNSUPPORTED, "svg"),
    # resdir//"test/parse/test.png" does not exist under res/ (parse_spectrum.f90:87-92)
    ("test_spectra_2D.toml", abi.ERR_INVALID_ARG, "Error reading file"),
    # rejected by the reference itself:
    ("skin.toml", abi.ERR_INVALID_ARG, "Uniform source requires point1"),   # parse_source.f90:183-186
    ("exp.toml", abi.ERR_INVALID_ARG, "position"),                          # annulus without position
    ("slab_test.toml", abi.ERR_INVALID_ARG, "position"),
    ("input.toml", abi.ERR_INVALID_ARG, "no such routine"),                 # setup.f90:58-59
    ("jacques.toml", abi.ERR_INVALID_ARG, "no such routine"),
])
def test_rejections(name, code, why):
    with pytest.raises(SmcrtError) as e:
        Job(res(name))
    assert abi.STATUS_NAMES[code] in str(e.value) and why in str(e.value)


def test_annulus_source_thin_barrier():
    """thinBarrier.toml: besselAnnulus source rotated onto +x (parse_source.f90:67-91, 230-247)."""
    j = Job(res("thinBarrier.toml"))
    s = j.desc.source
    assert s.kind == abi.SRC_ANNULUS and s.beam == abi.BEAM_BESSEL
    assert list(s.pos) == [-1.5, 0.0, 0.0] and list(s.rotation) == [1.0, 0.0, 0.0]
    assert (s.rlo, s.rhi, s.sigma, s.focal_length) == (0.48, 0.52, 0.05, 1.5)
    meta = dict(l.split(" = ", 1) for l in j.metadata().strip().splitlines())
    assert meta['"rotation%x"'] == "1.0" and meta["annulus_type"] == '"besselAnnulus"'


def test_fibre_detectors():
    """validateFibreDect.toml: ten fibre detectors (handle_fibre_collection_dect,
    parse_detectors.f90:233-294; init_fibre_dect detectors.f90:246-329)."""
    j = Job(res("validateFibreDect.toml"))
    assert len(j.detectors) == 10 and all(d.kind == abi.DET_FIBRE for d in j.detectors)
    d = j.detectors[5]
    f1, f2, a1, a2, front, back, f2pin, pin2b, pinap, acc, core = d.fibre
    assert (f1, f2, a1, a2, front, back) == (2.0, 200.0, 3.0, 3.0, 0.0, 200.0)
    assert (f2pin, pin2b, pinap, core) == (2.0, 200.0, 200.0, 1.0)
    assert acc == 90.0  # the file's "acceptAngle" is not the key the reference reads
    assert d.nbins == 101 and d.bin_wid == 1.0 / 2 / 100
    assert list(d.pos) == [0.0, 0.0, 2.0] and list(d.dir) == [0.0, 0.0, 1.0]


def test_spectrum_1d_blood():
    """test_spectra_1D.toml: the 1-D spectrum file (blood.dat) read in single precision
    (parse_spectrum.f90:59-66)."""
    j = Job(res("test_spectra_1D.toml"))
    sp = j.desc.source.spectrum.contents
    assert sp.kind == abi.SPEC_1D and sp.n == 376
    arr = np.ctypeslib.as_array(sp.array, shape=(2 * sp.n,))
    assert arr[0] == 250.0 and arr[sp.n] == 106112.0
    assert np.all(arr == arr.astype(np.float32))


def test_spectrum_2d_png(tmp_path):
    """A 2-D spectrum from a PNG (stb_image's first channel; parse_spectrum.f90:67-112)."""
    import shutil
    shutil.copy(os.path.join(GOLDEN, "test", "parse", "test.png"), tmp_path / "img.png")
    text = open(res("test_spectra_2D.toml")).read().replace('"test/parse/test.png"', '"img.png"')
    text = text.replace('name = "point"', 'name = "slm"\nrotation = [0.0, 0.0, 1.0]\ndirection = "-z"')
    (tmp_path / "slm.toml").write_text(text)
    j = Job(str(tmp_path / "slm.toml"))
    s = j.desc.source
    sp = s.spectrum.contents
    assert s.kind == abi.SRC_SLM and sp.kind == abi.SPEC_2D and (sp.width, sp.height) == (200, 200)
    img = np.ctypeslib.as_array(sp.image, shape=(200 * 200,)).reshape(200, 200, order="F")
    want = np.load(os.path.join(GOLDEN, "slm_test_png.npz"))["first_channel"]
    assert np.array_equal(img, want.astype(np.float64))


def test_metadata_dict():
    meta = Job(res("validation1.toml")).metadata()
    lines = dict(l.split(" = ", 1) for l in meta.strip().splitlines())
    assert lines["nphotons"] == "1000000" and lines['"mus%   1"'] == "90.0"
    assert lines["source"] == '"pencil"' and lines["experiment"] == '"box"' and lines["units"] == '"cm"'
    assert lines['"BoxDimensions%   3"'] == "0.02"


@pytest.mark.gpu
def test_job_run_scat_test(tmp_path, kats):
    """default_MCRT on res/scat_test.toml: the reference's KAT and its output files."""
    from tests.test_writers import read_nrrd_like_reference
    j = Job(res("scat_test.toml"))
    nscatt = j.run(tmp_path)
    k = kats["scat_test_nscatt"]
    assert abs(nscatt / j.desc.n_photons - k["value"]) <= k["thr"]
    data, hdr = read_nrrd_like_reference(tmp_path / "jmean" / "fluence.nrrd")
    assert data.shape == (200, 200, 200) and data.dtype == np.float32 and hdr["experiment"] == '"scat_test"'
    assert (tmp_path / "absorb" / "absorb.nrrd").exists() and (tmp_path / "emission" / "source_render.nrrd").exists()
    # the same photons through the Python engine API, normalised the same way
    from rsmcrt_amd import output
    from rsmcrt_amd.engine import Engine
    d = j.desc
    with Engine(builders.setup_scat_test(10.0), d.grid) as eng:
        r = eng.run(d.source, d.n_photons, seed=d.seed)
    # (the job runs checkpoint_every_n-photon batches: fp64 sums in another order)
    np.testing.assert_allclose(output.normalise_fluence(r.jmean.astype(np.float32), d.grid, d.n_photons), data,
                               rtol=1e-6, atol=0)


# ------------------------- the escape / inverse build variants --------
def test_escape_mode_symmetry_table():
    """res/default.toml under -DescapeFunction: parse_symmetry (parse.f90:188-340)."""
    j = Job(res("default.toml"), mode="escape")
    c = j.escape_config()
    assert c.symmetry == abi.SYM_ROTATIONAL_360
    assert list(c.n) == [100, 500, 200] and list(c.max) == [60.0, 360.0, 30.0]
    assert list(c.pos) == [0.0, 0.0, 0.0] and list(c.dir) == [1.0, 0.0, 0.0] and c.rotation == 0.0
    assert j.desc.n_photons == 100000  # escapenphotons replaces nphotons
    assert 'symmetryType = "360rotational"' in j.metadata()
    assert j.targets() == [-1.0] * 11
    # the default build neither parses nor records the table
    d = Job(res("default.toml"))
    assert d.desc.n_photons == 1000000 and "symmetryType" not in d.metadata()
    with pytest.raises(SmcrtError):
        d.escape_config()


def test_escape_mode_defaults_without_table():
    """No [symmetry] table: symmetry none, 10^3 grid of half-size 1, 1e5 photons (:313-339)."""
    j = Job(res("scat_test.toml"), mode="escape")
    c = j.escape_config()
    assert c.symmetry == abi.SYM_NONE and list(c.n) == [10, 10, 10] and list(c.max) == [1.0, 1.0, 1.0]
    assert list(c.dir) == [0.0, 0.0, 1.0] and j.desc.n_photons == 100000


def test_inverse_mode_table():
    """res/thinBarrier.toml under -DinverseMCRT: parse_inverse (parse.f90:343-413)."""
    j = Job(res("thinBarrier.toml"), mode="inverse")
    c = j.inverse_config()
    assert c.layer == 1 and c.max_steps == 30000
    assert (c.max_step_size, c.grad_step_size, c.accuracy) == (1.0, 0.0005, 0.001)
    assert c.flags == abi.INVERSE_FIND_MUA | abi.INVERSE_FIND_MUS
    meta = j.metadata()
    for k in ("maxStepSize", "gradStepSize", "accuracy", "maxNumSteps", "Findmua", "Findmus", "Findg", "Findn",
              "inverseLayer"):
        assert k + " = " in meta
    with pytest.raises(SmcrtError, match="Need inverse table"):
        Job(res("default.toml"), mode="inverse")


def test_escape_mode_bad_symmetry(tmp_path):
    text = open(res("scat_test.toml")).read()
    for extra, why in (('[symmetry]\nsymmetryType = "cubic"\n', "Unrecognised symmetry type"),
                       ('[symmetry]\nrotation = 360.0\n', "rotation for symmetry"),
                       ('[symmetry]\ndirection = [0.0, 0.0, 0.0]\n', "non-zero direction"),
                       ('[symmetry]\nGridSize = [1, 2]\n', "grid size")):
        p = tmp_path / "s.toml"
        p.write_text(text + "\n" + extra)
        with pytest.raises(SmcrtError, match=why):
            Job(str(p), mode="escape")


@pytest.mark.gpu
def test_job_run_escape_files(tmp_path):
    """escape_Function on res/default.toml (360rotational symmetry, 11 annulus detectors) with
    a smaller symmetry grid, fluence grid and photon count: write_escape's files hold the
    arrays of the batched escape run (smcrt_escape_run on the same scene)."""
    from tests.test_writers import read_nrrd_like_reference
    from rsmcrt_amd.engine import Engine
    text = open(res("default.toml")).read()
    text = (text.replace("GridSize = [100,500,200]", "GridSize = [4,3,5]")
            .replace("escapenphotons = 100000", "escapenphotons = 300")
            .replace("nxg = 200", "nxg = 20").replace("nyg = 110", "nyg = 11").replace("nzg = 100", "nzg = 10"))
    p = tmp_path / "esc.toml"
    p.write_text(text)
    j = Job(str(p), mode="escape")
    out = tmp_path / "out"
    j.run_escape(out)
    d = j.desc
    sc = scene.Scene([])
    sc.nodes = [j.nodes[i] for i in range(d.n_nodes)]
    sc.top = list(j.top[:d.n_top])
    with Engine(sc, d.grid, j.detectors) as eng:
        es, e, _ = eng.escape(j.escape_config(), d.n_photons, source=d.source, seed=d.seed)
    assert es.max() > 0
    for i, det_id in enumerate([f"Offset{k}mm" for k in range(1, 12)]):
        a, hdr = read_nrrd_like_reference(out / "escape" / f"dectID_{det_id}__escape{i + 1}.nrrd")
        b, _ = read_nrrd_like_reference(out / "escape" / f"dectID_{det_id}__escapeSym{i + 1}.nrrd")
        assert np.array_equal(a, e[i].T) and np.array_equal(b, es[i].T)  # (the reader gives z, y, x)
    assert (out / "jmean" / "fluence.nrrd").exists() and (out / "detectors" / "detector_1.dat").exists()


@pytest.mark.gpu
def test_job_run_inverse(tmp_path):
    """inverse_MCRT on res/thinBarrier.toml (with a target detector added, fewer steps and
    photons, searching g only): guesses inside AdaLIPO's bounds, every step's error identical (the reference
    reruns the original layer), and a different error per step with the trial applied."""
    text = open(res("thinBarrier.toml")).read()
    # (a 0.5-thick barrier: the file's zero-thickness box never scatters)
    text = (text.replace("maxNumSteps = 30000", "maxNumSteps = 3").replace("nphotons = 10000000", "nphotons = 2000")
            .replace("BoxDimensions = [0.0,2.0,2.0]", "BoxDimensions = [0.5,2.0,2.0]")
            .replace("Findmua = true", "Findmua = false").replace("Findmus = true", "Findmus = false")
            .replace("Findg = false", "Findg = true")
            + '\n[[detectors]]\ntype = "circle"\nID = "T"\nposition = [1.49, 0.0, 0.0]\ndirection = [1.0, 0.0, 0.0]\n'
            'radius = 1.0\nnbins = 10\nlayer = 2\ninverseTarget = 0.2\n')
    p = tmp_path / "inv.toml"
    p.write_text(text)
    j = Job(str(p), mode="inverse")
    assert j.targets() == [0.2]
    g = j.run_inverse()
    assert g.shape == (3, 5)
    assert np.all((g[:, 2] >= -1) & (g[:, 2] <= 1)) and len(set(g[:, 2])) == 3  # only g is searched
    assert np.all(g[:, 0] == g[0, 0]) and np.all(g[:, 1] == 0.075) and np.all(g[:, 3] == 1.0)
    assert np.all(g[:, 4] == g[0, 4]) and g[0, 4] < 0
    t = j.run_inverse(apply_trial=True)
    assert np.array_equal(t[:, :4], g[:, :4]) and len(set(t[:, 4])) > 1


@pytest.mark.gpu
def test_job_checkpoint_write_and_resume(tmp_path):
    """run_MCRT's checkpoints (kernelsMod.f90:1865, writer.f90:426-457) hold exactly the
    tally of photons [0, j); default_MCRT's load_checkpoint (:51-71) reruns the remaining
    photons with iseed*101 from zeroed tallies (the reference's second setup() zeroes them)."""
    from rsmcrt_amd import output
    from rsmcrt_amd.engine import Engine
    base = open(res("scat_test.toml")).read()
    t1 = base.replace("nphotons = 100000", "nphotons = 30000").replace("checkpoint_every_n=10000",
                                                                       "checkpoint_every_n=20000")
    assert t1 != base
    (tmp_path / "ck.toml").write_text(t1)
    out = tmp_path / "run1"
    j = Job(str(tmp_path / "ck.toml"))
    j.run(out)
    raw = (out / "check.ckpt").read_bytes()
    hdr = b"tomlfile=ck.toml\nphotons_run=20000\n"
    assert raw.startswith(hdr)
    ck = np.frombuffer(raw[len(hdr):], dtype=np.float32)
    d = j.desc
    with Engine(builders.setup_scat_test(10.0), d.grid) as eng:
        r = eng.run(d.source, 20000, seed=d.seed)
    np.testing.assert_allclose(ck, r.jmean.astype(np.float32).reshape(-1), rtol=1e-6, atol=0)
    # resume: load_checkpoint = true with the same relative checkpoint_file, which names the
    # file under the output directory for the read as for the write
    t2 = t1.replace("load_checkpoint=false", "load_checkpoint=true")
    assert "load_checkpoint=true" in t2 and 'checkpoint_file="check.ckpt"' in t2
    (tmp_path / "resume.toml").write_text(t2)
    out2 = out
    Job(str(tmp_path / "resume.toml")).run(out2)
    from tests.test_writers import read_nrrd_like_reference
    data, _ = read_nrrd_like_reference(out2 / "jmean" / "fluence.nrrd")
    with Engine(builders.setup_scat_test(10.0), d.grid) as eng:
        r2 = eng.run(d.source, 10000, seed=d.seed * 101)
    np.testing.assert_allclose(output.normalise_fluence(r2.jmean.astype(np.float32), d.grid, 10000), data,
                               rtol=1e-6, atol=0)
