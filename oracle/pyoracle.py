"""ORACLE — test infrastructure only (see smcrt_oracle.c header).

ctypes front end of liboracle.so, the CPU restatement of the reference hot path. Imported
only by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess
import threading

import numpy as np

from rsmcrt_amd import abi
from rsmcrt_amd.scene import detector_array
from rsmcrt_amd.tallies import Result

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "liboracle.so")
_lock = threading.Lock()
_lib = None


def build(force: bool = False) -> str:
    src = os.path.join(HERE, "smcrt_oracle.c")
    if force or not os.path.exists(LIB_PATH) or os.path.getmtime(LIB_PATH) < os.path.getmtime(src):
        subprocess.run(["make", "-C", HERE, "-s", "liboracle.so"], check=True)
    return LIB_PATH


def lib():
    global _lib
    with _lock:
        if _lib is None:
            build()
            L = C.CDLL(LIB_PATH)
            L.oracle_philox4x32_10.argtypes = [C.POINTER(C.c_uint32), C.POINTER(C.c_uint32), C.POINTER(C.c_uint32)]
            L.oracle_uniform.argtypes = [C.c_uint64, C.c_uint64, C.c_uint32]
            L.oracle_uniform.restype = C.c_double
            L.oracle_log.argtypes = [C.c_double]
            L.oracle_log.restype = C.c_double
            L.oracle_sincos.argtypes = [C.c_double, C.POINTER(C.c_double), C.POINTER(C.c_double)]
            L.oracle_spectrum_sample.argtypes = [C.POINTER(abi.Source), C.c_uint64, C.c_uint64, C.c_int64,
                                                 C.POINTER(C.c_double), C.POINTER(C.c_double),
                                                 C.POINTER(C.c_uint32)]
            L.oracle_atan.argtypes = [C.c_double]
            L.oracle_atan.restype = C.c_double
            L.oracle_emit.argtypes = [C.POINTER(abi.Grid), C.POINTER(abi.Source), C.c_uint64, C.c_uint64, C.c_int64,
                                      C.POINTER(C.c_double), C.POINTER(C.c_double), C.POINTER(C.c_int32),
                                      C.POINTER(C.c_uint32)]
            L.oracle_fresnel.argtypes = [C.POINTER(C.c_double), C.POINTER(C.c_double), C.c_double, C.c_double]
            L.oracle_fresnel.restype = C.c_double
            L.oracle_reflect_refract.argtypes = [C.POINTER(C.c_double), C.POINTER(C.c_double), C.c_double,
                                                 C.c_double, C.c_double, C.POINTER(C.c_int)]
            L.oracle_sdf_eval.argtypes = [C.POINTER(abi.SdfNode), C.c_int32, C.c_int32, C.POINTER(C.c_double),
                                          C.c_int64, C.POINTER(C.c_double)]
            L.oracle_calc_normal.argtypes = [C.POINTER(abi.SdfNode), C.c_int32, C.c_int32, C.POINTER(C.c_double),
                                             C.POINTER(C.c_double)]
            L.oracle_run.argtypes = [C.POINTER(abi.SdfNode), C.c_int32, C.POINTER(C.c_int32), C.c_int32,
                                     C.POINTER(abi.Grid), C.POINTER(abi.Detector), C.c_int32,
                                     C.POINTER(abi.Source), C.POINTER(abi.RunConfig), C.POINTER(abi.Tallies)]
            L.oracle_record_hit.argtypes = [C.POINTER(abi.Detector), C.POINTER(C.c_double), C.POINTER(C.c_double),
                                            C.c_double, C.c_int32, C.c_double, C.POINTER(C.c_double),
                                            C.POINTER(C.c_uint64)]
            L.oracle_spectral_sample.argtypes = [C.POINTER(abi.Spectral), C.c_int32, C.c_uint64,
                                                 C.POINTER(C.c_uint64), C.POINTER(C.c_double)]
            _lib = L
    return _lib


def _dp(a):
    return a.ctypes.data_as(C.POINTER(C.c_double))


def philox(ctr, key):
    c = (C.c_uint32 * 4)(*ctr)
    k = (C.c_uint32 * 2)(*key)
    o = (C.c_uint32 * 4)()
    lib().oracle_philox4x32_10(c, k, o)
    return list(o)


def uniform(seed, pid, draw):
    return lib().oracle_uniform(seed, pid, draw)


def log(x):
    return lib().oracle_log(float(x))


def atan(x):
    return lib().oracle_atan(float(x))


def spectral_sample(tables, mode, seed, draw=0):
    """The restatement of init_spectral / updateSpectral (opticalProperties.f90:127-201) on
    five (n, 2) tables (mus, mua, hgg, n, flux): (dict of mus, mua, hgg, g2, n, kappa, albedo,
    wavelength; the stream position after it)."""
    arrs = [np.asfortranarray(np.asarray(a, dtype=np.float64)) for a in tables]
    sp = abi.Spectral()
    for name, a in zip(("mus", "mua", "hgg", "n", "flux"), arrs):
        setattr(sp, "n_" + name, a.shape[0])
        setattr(sp, name, _dp(a))
    d = C.c_uint64(draw)
    out = np.zeros(8)
    st = lib().oracle_spectral_sample(C.byref(sp), mode, seed, C.byref(d), _dp(out))
    if st != 0:
        raise RuntimeError(f"oracle_spectral_sample failed: {abi.STATUS_NAMES.get(st, st)}")
    keys = ("mus", "mua", "hgg", "g2", "n", "kappa", "albedo", "wavelength")
    return dict(zip(keys, out.tolist())), d.value


def spectrum_sample(source, n, seed=123456789, first=0):
    """n draws of source.spectrum (photon p uses its own stream, from draw 0): x, y, draws."""
    x = np.zeros(n); y = np.zeros(n); dr = np.zeros(n, dtype=np.uint32)
    st = lib().oracle_spectrum_sample(C.byref(source), seed, first, n, _dp(x), _dp(y),
                                      dr.ctypes.data_as(C.POINTER(C.c_uint32)))
    if st != 0:
        raise RuntimeError(f"oracle_spectrum_sample failed: {abi.STATUS_NAMES.get(st, st)}")
    return x, y, dr


def emit(grid, source, n, seed=123456789, first=0):
    """One emission of photons [first, first+n) (no re-emission loop): pos (n,3), dir (n,3),
    cells (n,3), draws (n)."""
    pos = np.zeros((n, 3)); d = np.zeros((n, 3))
    cells = np.zeros((n, 3), dtype=np.int32); draws = np.zeros(n, dtype=np.uint32)
    st = lib().oracle_emit(C.byref(grid), C.byref(source), seed, first, n, _dp(pos), _dp(d),
                           cells.ctypes.data_as(C.POINTER(C.c_int32)),
                           draws.ctypes.data_as(C.POINTER(C.c_uint32)))
    if st != 0:
        raise RuntimeError(f"oracle_emit failed: {abi.STATUS_NAMES.get(st, st)}")
    return pos, d, cells, draws


def sincos(x):
    s, c = C.c_double(), C.c_double()
    lib().oracle_sincos(float(x), C.byref(s), C.byref(c))
    return s.value, c.value


def fresnel(I, N, n1, n2):
    i = (C.c_double * 3)(*I)
    n = (C.c_double * 3)(*N)
    return lib().oracle_fresnel(i, n, n1, n2)


def reflect_refract(I, N, n1, n2, xi):
    i = (C.c_double * 3)(*I)
    n = (C.c_double * 3)(*N)
    r = C.c_int()
    lib().oracle_reflect_refract(i, n, n1, n2, xi, C.byref(r))
    return list(i), bool(r.value)


def sdf_eval(scene, pts, which=0):
    """Evaluate top-level SDF `which` of `scene` at points pts (n,3)."""
    pts = np.ascontiguousarray(pts, dtype=np.float64).reshape(-1, 3)
    out = np.empty(len(pts))
    nodes = scene.node_array()
    st = lib().oracle_sdf_eval(nodes, len(scene.nodes), scene.top[which], _dp(pts), len(pts), _dp(out))
    assert st == 0
    return out


def calc_normal(scene, p, which=0):
    nodes = scene.node_array()
    pp = (C.c_double * 3)(*p)
    n = (C.c_double * 3)()
    lib().oracle_calc_normal(nodes, len(scene.nodes), scene.top[which], pp, n)
    return list(n)


def record_hit(det, start, direction, point_sep, layer=1, weight=1.0):
    """One record_hit on one detector: returns (bins, hits)."""
    n = det.nbins * det.nbins if det.kind == abi.DET_CAMERA else det.nbins
    bins = np.zeros(n)
    hits = C.c_uint64()
    s = (C.c_double * 3)(*start)
    d = (C.c_double * 3)(*direction)
    lib().oracle_record_hit(C.byref(det), s, d, point_sep, layer, weight, _dp(bins), C.byref(hits))
    return bins, hits.value


def run(scene, grid, source, n_photons, seed=123456789, flags=abi.FLAG_PATHLENGTH, dets=(),
        first_photon=0, records=False, result=None):
    dets = list(dets)
    res = result if result is not None else Result(grid, dets, n_photons, records)
    res.n_photons += n_photons
    cfg = abi.RunConfig()
    cfg.n_photons, cfg.first_photon, cfg.seed = n_photons, first_photon, seed
    cfg.flags = flags | (abi.FLAG_RECORD_PHOTONS if records else 0)
    nodes = scene.node_array()
    top = scene.top_array()
    darr = detector_array(dets)
    t = res.tallies()
    st = lib().oracle_run(nodes, len(scene.nodes), top, scene.n_top, C.byref(grid), darr, len(dets),
                          C.byref(source), C.byref(cfg), C.byref(t))
    if st != 0:
        raise RuntimeError(f"oracle_run failed: {abi.STATUS_NAMES.get(st, st)}")
    return res
