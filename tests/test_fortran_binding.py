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
         "smcrt_escape_config": abi.EscapeConfig, "smcrt_inverse_config": abi.InverseConfig}


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
    for sym in ("smcrt_scene_create", "smcrt_run", "smcrt_normalise_fluence", "smcrt_scene_destroy"):
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
