"""Output files of the reference (src/writer.f90) through libsmcrt.so's writer entry points:
NRRD / raw volumes, detector .dat streams, checkpoints. Host-side; no GPU needed.

Arrays use the package's grid convention, shape (nz, ny, nx), which is the memory image of
the reference's Fortran jmean(nx, ny, nz).
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from . import abi
from .engine import SmcrtError, load_library

_declared = False


def _lib():
    global _declared
    L = load_library()
    if not _declared:
        common = [C.c_char_p, C.c_void_p, C.c_int32, C.c_int32, C.c_int32, C.c_char_p, C.c_char_p, C.c_int32,
                  C.c_char_p, C.c_int32]
        L.smcrt_write_data_f32.argtypes = common
        L.smcrt_write_data_f64.argtypes = common
        L.smcrt_write_detector.argtypes = [C.c_char_p, C.POINTER(abi.Detector), C.POINTER(C.c_double), C.c_char_p,
                                           C.c_int64]
        L.smcrt_write_checkpoint.argtypes = [C.c_char_p, C.c_char_p, C.c_int64, C.POINTER(C.c_float),
                                             C.POINTER(abi.Grid), C.c_int32, C.c_char_p, C.c_int32]
        _declared = True
    return L


def _check(st):
    if st != abi.OK:
        raise SmcrtError(f"{abi.STATUS_NAMES.get(st, st)}: {load_library().smcrt_last_error().decode(errors='replace')}")


def _b(s):
    return None if s is None else str(s).encode()


def write_data(filename, array, metadata: str | None = None, dect_id: str | None = None,
               overwrite: bool = True) -> str:
    """write_data, writer.f90:162-226: .nrrd / .raw / .dat chosen by extension. `array` is
    float32 or float64 of shape (nz, ny, nx). Returns the file name actually written."""
    a = np.ascontiguousarray(array)
    if a.ndim != 3:
        raise ValueError("array must be 3-D (nz, ny, nx)")
    nz, ny, nx = a.shape
    fn = {np.dtype(np.float32): "smcrt_write_data_f32", np.dtype(np.float64): "smcrt_write_data_f64"}.get(a.dtype)
    if fn is None:
        raise TypeError("array must be float32 or float64")
    out = C.create_string_buffer(4096)
    _check(getattr(_lib(), fn)(_b(filename), a.ctypes.data_as(C.c_void_p), nx, ny, nz, _b(metadata), _b(dect_id),
                               1 if overwrite else 0, out, len(out)))
    return out.value.decode()


def write_detector(filename, det: abi.Detector, data, dect_id: str, nphotons: int) -> None:
    """write_detected_photons, writer.f90:55-138, for one detector."""
    d = np.ascontiguousarray(data, dtype=np.float64)
    _check(_lib().smcrt_write_detector(_b(filename), C.byref(det), d.ctypes.data_as(C.POINTER(C.c_double)),
                                       _b(dect_id), int(nphotons)))


def write_checkpoint(filename, toml_filename: str, photons_run: int, jmean, grid: abi.Grid,
                     overwrite: bool = True) -> str:
    """checkpoint, writer.f90:419-455."""
    a = np.ascontiguousarray(jmean, dtype=np.float32)
    out = C.create_string_buffer(4096)
    _check(_lib().smcrt_write_checkpoint(_b(filename), _b(toml_filename), int(photons_run),
                                         a.ctypes.data_as(C.POINTER(C.c_float)), C.byref(grid),
                                         1 if overwrite else 0, out, len(out)))
    return out.value.decode()


def normalise_fluence(jmean, grid: abi.Grid, nphotons: int) -> np.ndarray:
    """normalise_fluence, writer.f90:25-52, on an fp32 copy (the reference's array kind)."""
    a = np.array(jmean, dtype=np.float32, copy=True, order="C")
    _check(load_library().smcrt_normalise_fluence(a.ctypes.data_as(C.POINTER(C.c_float)), C.byref(grid),
                                                  int(nphotons)))
    return a
