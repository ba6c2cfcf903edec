"""CPU checks of the C ABI boundary: the HIP library builds for gfx950, loads, exports
exactly the entry points include/smcrt.h declares, and its struct layouts match the
ctypes mirror. No compute call is made (there is no GPU here)."""
import ctypes as C
import os
import re
import subprocess
import textwrap

import pytest

from rsmcrt_amd import abi
from rsmcrt_amd import build as B

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "smcrt.h")


def header_functions():
    txt = open(HEADER).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    return sorted(set(re.findall(r"\b(smcrt_[a-z_0-9]+)\s*\(", txt)))


def test_header_and_mirror_agree():
    assert header_functions() == sorted(abi.EXPORTED_SYMBOLS)


def test_exports(lib_path):
    out = subprocess.run(["nm", "-D", "--defined-only", lib_path], capture_output=True, text=True, check=True).stdout
    exported = {l.split()[-1] for l in out.splitlines() if " T " in l}
    for fn in header_functions():
        assert fn in exported, fn


def test_abi_version_matches_header():
    """The header, the ctypes mirror and the Fortran module agree on the version; version 4 is
    the 56-byte smcrt_kernel_times (lean_hazards), version 5 the node flags and the spectral
    optical properties."""
    txt = open(HEADER).read()
    assert int(re.search(r"#define SMCRT_ABI_VERSION (\d+)", txt).group(1)) == abi.SMCRT_ABI_VERSION == 5
    f90 = open(os.path.join(ROOT, "bindings", "fortran", "smcrt_mod.f90")).read()
    assert int(re.search(r"SMCRT_MOD_ABI_VERSION = (\d+)", f90).group(1)) == abi.SMCRT_ABI_VERSION
    assert C.sizeof(abi.KernelTimes) == 56


def test_load_and_version(lib_path):
    from rsmcrt_amd import engine
    L = engine.load_library(lib_path)
    assert L.smcrt_abi_version() == abi.SMCRT_ABI_VERSION
    n = C.c_int32(-1)
    assert L.smcrt_device_count(C.byref(n)) == 0 and n.value >= 0


def test_errors_without_compute(lib_path):
    """Invalid arguments fail with a status code and a message, never an abort."""
    from rsmcrt_amd import engine
    L = engine.load_library(lib_path)
    h = C.c_void_p()
    st = L.smcrt_scene_create(None, 0, None, 0, None, None, 0, 0, C.byref(h))
    assert st == abi.ERR_INVALID_ARG and L.smcrt_last_error()
    assert L.smcrt_run(None, None, None, None) == abi.ERR_INVALID_ARG


STRUCTS = {
    "smcrt_sdf_node": (abi.SdfNode, ["kind", "op", "n_children", "flags", "reserved", "transform", "param", "k",
                                     "mus", "n"]),
    "smcrt_spectral": (abi.Spectral, ["n_mus", "n_flux", "mus", "mua", "hgg", "n", "flux"]),
    "smcrt_optprops": (abi.OptProps, ["mus", "g2", "albedo", "wavelength", "node_flags"]),
    "smcrt_grid": (abi.Grid, ["nx", "nz", "xmax", "zmax"]),
    "smcrt_source": (abi.Source, ["kind", "pos", "dir", "p1", "p3", "beam", "radius", "sigma", "rotation",
                                  "spectrum"]),
    "smcrt_spectrum": (abi.Spectrum, ["kind", "wavelength", "n", "array", "width", "image", "cell_height"]),
    "smcrt_detector": (abi.Detector, ["kind", "nbins", "pos", "e2", "radius", "bin_wid_y", "fibre"]),
    "smcrt_run_config": (abi.RunConfig, ["n_photons", "seed", "flags"]),
    "smcrt_photon_record": (abi.PhotonRecord, ["pos", "weight", "cell", "draws", "status"]),
    "smcrt_tallies": (abi.Tallies, ["jmean", "jmean_f64", "det_bins", "counters", "records"]),
    "smcrt_device_tallies": (abi.DeviceTallies, ["jmean", "det_bins", "records"]),
    "smcrt_kernel_times": (abi.KernelTimes, ["transport_ms", "deposit_ms", "launches", "lean_launches", "far_steps",
                                             "fold_cu_ms", "lean_hazards"]),
    "smcrt_pack_layout": (abi.PackLayout, ["n_voxels", "n_det_bins", "fields"]),
    "smcrt_escape_config": (abi.EscapeConfig, ["symmetry", "n", "max", "pos", "dir", "rotation"]),
    "smcrt_inverse_config": (abi.InverseConfig, ["layer", "flags", "max_steps", "max_step_size", "accuracy", "seed"]),
}


def test_struct_layout(tmp_path):
    lines = ['#include <stdio.h>', '#include <stddef.h>', f'#include "{HEADER}"', 'int main(void){']
    for s, (_, fields) in STRUCTS.items():
        lines.append(f'printf("{s} %zu\\n", sizeof({s}));')
        for f in fields:
            lines.append(f'printf("{s}.{f} %zu\\n", offsetof({s}, {f}));')
    lines.append("return 0;}")
    src = tmp_path / "layout.c"
    src.write_text("\n".join(lines))
    exe = tmp_path / "layout"
    subprocess.run(["gcc", "-o", str(exe), str(src)], check=True)
    got = dict(l.rsplit(" ", 1) for l in subprocess.run([str(exe)], capture_output=True, text=True).stdout.splitlines())
    for s, (cls, fields) in STRUCTS.items():
        assert int(got[s]) == C.sizeof(cls), s
        for f in fields:
            assert int(got[f"{s}.{f}"]) == getattr(cls, f).offset, (s, f)
    assert abi.record_dtype().itemsize == C.sizeof(abi.PhotonRecord)


def test_no_oracle_in_product():
    """The product path never imports, loads or links the oracle (test infrastructure)."""
    pat = re.compile(r"(from\s+oracle|import\s+oracle|pyoracle|liboracle|smcrt_oracle\.c|oracle_run)")
    for dp, _, files in os.walk(os.path.join(ROOT, "rsmcrt_amd")):
        for f in files:
            if f.endswith((".py", ".hip", ".h", ".cpp")):
                txt = open(os.path.join(dp, f)).read()
                assert not pat.search(txt), f


def _nested(levels):
    """One top: `levels` models nested in each other around two spheres, plus a medium box."""
    from rsmcrt_amd.scene import Scene, box, invert, model, mono, sphere, translate
    o = mono(5.0, 0.1, 0.8, 1.0)
    s = model([sphere(0.3, o, 1), sphere(0.2, o, 1, transform=invert(translate((0.2, 0.0, 0.0))))], abi.OP_UNION)
    for _ in range(levels - 1):
        s = model([s, sphere(0.1, o, 1, transform=invert(translate((0.0, 0.3, 0.0))))], abi.OP_SMOOTH_UNION, 0.05)
    return Scene([s, box((1.0, 1.0, 1.0), mono(1.0, 0.01, 0.0, 1.0), 2)])


def test_nested_model_depth_checked_before_the_device(lib_path):
    """Nested models (eval_model's recursion, sdf_base.f90:146-161) are accepted up to 32
    levels (geometry.h PROG_MAX_DEPTH, node_value's explicit stack); a 33rd level is rejected
    with UNSUPPORTED before any device call, so both are checkable without a GPU."""
    from rsmcrt_amd import engine, scene
    L = engine.load_library(lib_path)
    g = scene.grid(8, 8, 8, 1, 1, 1)
    for levels, want in ((3, (abi.OK, abi.ERR_NO_DEVICE)), (32, (abi.OK, abi.ERR_NO_DEVICE)),
                         (33, (abi.ERR_UNSUPPORTED,))):
        sc = _nested(levels)
        h = C.c_void_p()
        st = L.smcrt_scene_create(sc.node_array(), len(sc.nodes), sc.top_array(), sc.n_top, C.byref(g), None, 0, 0,
                                  C.byref(h))
        assert st in want, (levels, st, L.smcrt_last_error())
        if st == abi.OK:
            L.smcrt_scene_destroy(h)
        if levels == 33:
            assert b"nested" in L.smcrt_last_error()
