"""The reference-side binding (bindings/fortran/smcrt_mod.f90): the module compiles with the
image's Fortran compiler, its bind(C) types have the C layout of include/smcrt.h, and the
example driver (the reference's scat_test KAT, test/end_to_end/test_scat.f90:33-38) links
against libsmcrt.so -- and, on a GPU, reproduces the KAT through the HIP engine."""
import ctypes as C
import os
import re
import shutil
import subprocess

import pytest

from rsmcrt_amd import abi

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
FDIR = os.path.join(ROOT, "bindings", "fortran")
FC = os.environ.get("AMDFLANG", "/opt/rocm/bin/amdflang")

pytestmark = pytest.mark.skipif(not os.path.exists(FC), reason="no Fortran compiler in this image")

TYPES = {"smcrt_sdf_node": abi.SdfNode, "smcrt_grid": abi.Grid, "smcrt_source": abi.Source,
         "smcrt_spectrum": abi.Spectrum,
         "smcrt_detector": abi.Detector, "smcrt_run_config": abi.RunConfig, "smcrt_tallies": abi.Tallies,
         "smcrt_device_tallies": abi.DeviceTallies, "smcrt_kernel_times": abi.KernelTimes,
         "smcrt_escape_config": abi.EscapeConfig, "smcrt_inverse_config": abi.InverseConfig,
         "smcrt_pack_layout": abi.PackLayout, "smcrt_spectral": abi.Spectral, "smcrt_optprops": abi.OptProps}


def _build_module(tmp):
    shutil.copy(os.path.join(FDIR, "smcrt_mod.f90"), tmp)
    subprocess.run([FC, "-O2", "-c", "smcrt_mod.f90"], cwd=tmp, check=True)


def test_bindc_layout_matches_c(lib_path, tmp_path):
    _build_module(tmp_path)
    lines = ["program sizes", "use smcrt_mod", "implicit none"]
    for t in TYPES:
        lines.append(f"type({t}) :: v_{t}")
    for t in TYPES:
        lines.append(f"print '(a,1x,i0)', '{t}', c_sizeof(v_{t})")
    lines.append("end program sizes")
    (tmp_path / "sizes.f90").write_text("\n".join(lines) + "\n")
    libdir = os.path.dirname(lib_path)
    subprocess.run([FC, "-o", "sizes", "sizes.f90", "smcrt_mod.o", f"-L{libdir}", "-lsmcrt", f"-Wl,-rpath,{libdir}"],
                   cwd=tmp_path, check=True)
    out = subprocess.run([str(tmp_path / "sizes")], capture_output=True, text=True, check=True).stdout
    got = {l.split()[0]: int(l.split()[1]) for l in out.splitlines() if l.strip()}
    for t, cls in TYPES.items():
        assert got[t] == C.sizeof(cls), (t, got[t], C.sizeof(cls))


def test_example_links_against_engine(lib_path, tmp_path):
    _build_module(tmp_path)
    shutil.copy(os.path.join(FDIR, "example_scat_test.f90"), tmp_path)
    libdir = os.path.dirname(lib_path)
    subprocess.run([FC, "-O2", "-o", "example", "example_scat_test.f90", "smcrt_mod.o", f"-L{libdir}", "-lsmcrt",
                    f"-Wl,-rpath,{libdir}"], cwd=tmp_path, check=True)
    nm = subprocess.run(["nm", str(tmp_path / "example")], capture_output=True, text=True, check=True).stdout
    for sym in ("smcrt_scene_create", "smcrt_run", "smcrt_normalise_fluence", "smcrt_scene_destroy",
                "smcrt_multi_create", "smcrt_multi_run", "smcrt_multi_destroy"):
        assert re.search(rf"\bU {sym}\b", nm), sym


@pytest.mark.gpu
def test_example_reproduces_scat_test_kat(lib_path, tmp_path, kats):
    _build_module(tmp_path)
    shutil.copy(os.path.join(FDIR, "example_scat_test.f90"), tmp_path)
    libdir = os.path.dirname(lib_path)
    subprocess.run([FC, "-O2", "-o", "example", "example_scat_test.f90", "smcrt_mod.o", f"-L{libdir}", "-lsmcrt",
                    f"-Wl,-rpath,{libdir}"], cwd=tmp_path, check=True)
    out = subprocess.run([str(tmp_path / "example"), "100000"], capture_output=True, text=True, timeout=300,
                         check=True).stdout
    v = float(re.search(r"nscatt/photon =\s*([0-9.]+)", out).group(1))
    k = kats["scat_test_nscatt"]
    assert abs(v - k["value"]) <= k["thr"], out
    assert re.search(r"photons = 100000\b", out), out


def test_module_binds_every_multi_gpu_entry_point(lib_path, tmp_path):
    """smcrt_mod declares the multi-GPU and communicator entry points of include/smcrt.h, each
    bound to a symbol the library exports."""
    src = open(os.path.join(FDIR, "smcrt_mod.f90")).read()
    names = set(re.findall(r'bind\(C, name="(smcrt_\w+)"\)', src))
    want = {"smcrt_multi_create", "smcrt_multi_info", "smcrt_multi_scene", "smcrt_multi_run", "smcrt_multi_accumulate",
            "smcrt_multi_collect", "smcrt_multi_device_photons", "smcrt_multi_destroy", "smcrt_comm_unique_id",
            "smcrt_comm_init_rank", "smcrt_comm_destroy", "smcrt_reduce_device_tallies", "smcrt_scene_fence",
            "smcrt_pack_size", "smcrt_pack_host", "smcrt_unpack_host"}
    assert want <= names, want - names
    lib = C.CDLL(lib_path)
    for n in names:
        assert hasattr(lib, n), n


@pytest.mark.gpu
def test_example_multi_gpu_matches_single(lib_path, tmp_path):
    """run_MCRT's n_gpus path from Fortran: the example through smcrt_multi_run on one device
    prints the same counters and nscatt as through smcrt_run, bit for bit (jmean to fp64 fold
    order)."""
    _build_module(tmp_path)
    shutil.copy(os.path.join(FDIR, "example_scat_test.f90"), tmp_path)
    libdir = os.path.dirname(lib_path)
    subprocess.run([FC, "-O2", "-o", "example", "example_scat_test.f90", "smcrt_mod.o", f"-L{libdir}", "-lsmcrt",
                    f"-Wl,-rpath,{libdir}"], cwd=tmp_path, check=True)
    outs = [subprocess.run([str(tmp_path / "example"), "50000", g], capture_output=True, text=True, timeout=300,
                           check=True).stdout for g in ("0", "1")]
    def parse(o):
        ctr = re.findall(r"counter (\d+) = (\d+)", o)
        return dict(ctr), re.search(r"nscatt =\s*(\S+)", o).group(1), float(re.search(r"jmean normalised\) =\s*(\S+)", o).group(1))
    (c0, n0, j0), (c1, n1, j1) = parse(outs[0]), parse(outs[1])
    assert len(c0) == 16 and n0 == n1, outs
    # (the engine counters, abi.ENGINE_COUNTERS, describe the schedule, not the photons)
    eng = {str(abi.CTR[k]) for k in abi.ENGINE_COUNTERS}
    assert {k: v for k, v in c0.items() if k not in eng} == {k: v for k, v in c1.items() if k not in eng}, outs
    assert abs(j0 - j1) <= 1e-9 * abs(j0)


# ---- the conversion glue (bindings/fortran/smcrt_glue.f90) ----------
GLUE_SCENES = ("scat_test", "aptran", "validation1", "omg", "test_dects", "egg_test")
SRC_FIELDS = ("pos", "dir", "p1", "p2", "p3", "radius", "beam_size", "focal_length", "rlo", "rhi", "sigma", "rotation")


def _read_glue(path):
    """One glue_scenes.f90 output: counts, node table, top, detectors, source fields."""
    import numpy as np
    raw = open(path, "rb").read()
    n_nodes, n_top, n_dets = np.frombuffer(raw[:12], dtype=np.int32)
    off = 12
    nodes = (abi.SdfNode * int(n_nodes)).from_buffer_copy(raw[off:off + n_nodes * C.sizeof(abi.SdfNode)])
    off += n_nodes * C.sizeof(abi.SdfNode)
    top = np.frombuffer(raw[off:off + 4 * n_top], dtype=np.int32)
    off += 4 * n_top
    dets = (abi.Detector * max(1, int(n_dets))).from_buffer_copy(
        raw[off:off + n_dets * C.sizeof(abi.Detector)] + b"\0" * (0 if n_dets else C.sizeof(abi.Detector)))
    off += n_dets * C.sizeof(abi.Detector)
    kind, beam = np.frombuffer(raw[off:off + 8], dtype=np.int32)
    vals = np.frombuffer(raw[off + 8:], dtype=np.float64)
    sizes = (3, 3, 3, 3, 3, 1, 1, 1, 1, 1, 1, 3)
    src, k = {"kind": int(kind), "beam": int(beam)}, 0
    for name, n in zip(SRC_FIELDS, sizes):
        src[name] = list(vals[k:k + n])
        k += n
    assert k == len(vals)
    return int(n_nodes), list(top), nodes, [dets[i] for i in range(n_dets)], src


def _fields(struct):
    out = {}
    for name, _ in struct._fields_:
        if name.startswith("reserved"):
            continue
        v = getattr(struct, name)
        out[name] = list(v) if hasattr(v, "__len__") else v
    return out


def test_glue_tables_match_the_toml_front_end(lib_path, tmp_path):
    """smcrt_glue's constructors, flattening, detector and source conversion (driven by
    glue_scenes.f90 as setupGeometry.f90 / parse_detectors.f90 / parse_source.f90 would) give
    the same node, top, detector and source tables, field for field and bit for bit, as the
    C++ front end's smcrt_job_scene on the same res/*.toml files."""
    from rsmcrt_amd.job import Job
    libdir = os.path.dirname(lib_path)
    for f in ("smcrt_mod.f90", "smcrt_glue.f90", "glue_scenes.f90"):
        shutil.copy(os.path.join(FDIR, f), tmp_path)
    subprocess.run([FC, "-O2", "-c", "smcrt_mod.f90"], cwd=tmp_path, check=True)
    subprocess.run([FC, "-O2", "-c", "smcrt_glue.f90"], cwd=tmp_path, check=True)
    subprocess.run([FC, "-O2", "-o", "glue_scenes", "glue_scenes.f90", "smcrt_glue.o", "smcrt_mod.o",
                    f"-L{libdir}", "-lsmcrt", f"-Wl,-rpath,{libdir}"], cwd=tmp_path, check=True)
    # get_vessels' data (tests/golden/make_vessel_data.py): the glue reads it with the Fortran
    # runtime's list-directed reads, the front end with its own reader
    from tests.golden.make_vessel_data import write_vessel_data
    vdir = tmp_path / "vessels"
    write_vessel_data(vdir, 40, 7)
    subprocess.run([str(tmp_path / "glue_scenes"), str(tmp_path), str(vdir)], check=True)
    for name in GLUE_SCENES + ("vessels",):
        n_nodes, top, nodes, dets, src = _read_glue(tmp_path / f"{name}.bin")
        j = Job(str(vdir / "vessels.toml") if name == "vessels" else
                os.path.join(ROOT, "tests", "golden", "res", f"{name}.toml"))
        d = j.desc
        assert n_nodes == d.n_nodes and len(top) == d.n_top and len(dets) == d.n_dets, name
        assert top == list(j.top[:d.n_top]), name
        for i in range(n_nodes):
            assert _fields(nodes[i]) == _fields(j.nodes[i]), (name, "node", i)
        for i, det in enumerate(dets):
            assert _fields(det) == _fields(j.dets[i]), (name, "detector", i)
        assert src["kind"] == d.source.kind and src["beam"] == d.source.beam, name
        for k in SRC_FIELDS:
            want = getattr(d.source, k)
            assert src[k] == (list(want) if hasattr(want, "__len__") else [want]), (name, "source", k)


def test_fortran_spectral_unit_test(lib_path, tmp_path):
    """test_opticalprops.f90:81-142 written against the binding (bindings/fortran/
    example_spectral.f90: the reference's tables with their default-real literals, spectral()
    then 10^4 updates in the test's bounds); its first 100 samples equal the restatement's."""
    import numpy as np
    from oracle import pyoracle as O
    from test_opticalprops import reference_tables
    for f in ("smcrt_mod.f90", "smcrt_glue.f90", "example_spectral.f90"):
        shutil.copy(os.path.join(FDIR, f), tmp_path)
    libdir = os.path.dirname(lib_path)
    subprocess.run([FC, "-O2", "-c", "smcrt_mod.f90"], cwd=tmp_path, check=True)
    subprocess.run([FC, "-O2", "-c", "smcrt_glue.f90"], cwd=tmp_path, check=True)
    subprocess.run([FC, "-O2", "-o", "example_spectral", "example_spectral.f90", "smcrt_glue.o", "smcrt_mod.o",
                    f"-L{libdir}", "-lsmcrt", f"-Wl,-rpath,{libdir}"], cwd=tmp_path, check=True)
    r = subprocess.run([str(tmp_path / "example_spectral"), str(tmp_path / "s.bin")], capture_output=True, text=True)
    assert r.returncode == 0 and "spectral OK" in r.stdout, r.stdout + r.stderr
    got = np.fromfile(tmp_path / "s.bin", dtype=np.float64).reshape(100, 5)
    tabs = reference_tables()
    _, d = O.spectral_sample(tabs, abi.SPECTRAL_INIT, 1234569, 0)
    for i in range(100):
        ref, d = O.spectral_sample(tabs, abi.SPECTRAL_UPDATE, 1234569, d)
        assert list(got[i]) == [ref["wavelength"], ref["mus"], ref["mua"], ref["hgg"], ref["n"]], i
