"""TOML front end (include/smcrt.h smcrt_job_*): a res/*.toml file -> the scene, grid,
source, detectors and settings the reference's parse_params + setup_simulation produce, and
default_MCRT's run + finalise on the GPU (src/kernelsMod.f90:14-82, 2321-2416)."""
from __future__ import annotations

import ctypes as C

from . import abi
from .engine import SmcrtError, load_library

_declared = False


def _lib():
    global _declared
    L = load_library()
    if not _declared:
        L.smcrt_job_load.argtypes = [C.c_char_p, C.POINTER(C.c_void_p)]
        L.smcrt_job_destroy.argtypes = [C.c_void_p]
        L.smcrt_job_destroy.restype = None
        L.smcrt_job_info.argtypes = [C.c_void_p, C.POINTER(abi.JobDesc)]
        L.smcrt_job_scene.argtypes = [C.c_void_p, C.POINTER(abi.SdfNode), C.POINTER(C.c_int32),
                                      C.POINTER(abi.Detector)]
        L.smcrt_job_metadata.argtypes = [C.c_void_p, C.c_char_p, C.c_int32]
        L.smcrt_job_run.argtypes = [C.c_void_p, C.c_int32, C.c_char_p, C.POINTER(C.c_double)]
        _declared = True
    return L


def _check(st):
    if st != abi.OK:
        raise SmcrtError(f"{abi.STATUS_NAMES.get(st, st)}: {load_library().smcrt_last_error().decode(errors='replace')}")


class Job:
    """A parsed input file (smcrt_job_load)."""

    def __init__(self, toml_path):
        L = _lib()
        h = C.c_void_p()
        _check(L.smcrt_job_load(str(toml_path).encode(), C.byref(h)))
        self._h = h
        self.desc = abi.JobDesc()
        _check(L.smcrt_job_info(self._h, C.byref(self.desc)))
        d = self.desc
        self.nodes = (abi.SdfNode * max(1, d.n_nodes))()
        self.top = (C.c_int32 * max(1, d.n_top))()
        self.dets = (abi.Detector * max(1, d.n_dets))()
        _check(L.smcrt_job_scene(self._h, self.nodes, self.top, self.dets))

    def close(self):
        if getattr(self, "_h", None):
            _lib().smcrt_job_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    @property
    def experiment(self) -> str:
        return self.desc.experiment.decode()

    @property
    def detectors(self):
        return [self.dets[i] for i in range(self.desc.n_dets)]

    def metadata(self) -> str:
        buf = C.create_string_buffer(1 << 16)
        _check(_lib().smcrt_job_metadata(self._h, buf, len(buf)))
        return buf.value.decode()

    def run(self, outdir, device: int = 0) -> float:
        """default_MCRT without checkpoint loading; returns the total scatter count."""
        ns = C.c_double()
        _check(_lib().smcrt_job_run(self._h, device, str(outdir).encode(), C.byref(ns)))
        return ns.value
