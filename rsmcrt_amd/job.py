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
        L.smcrt_job_load_mode.argtypes = [C.c_char_p, C.c_int32, C.POINTER(C.c_void_p)]
        L.smcrt_job_escape_config.argtypes = [C.c_void_p, C.POINTER(abi.EscapeConfig)]
        L.smcrt_job_inverse_config.argtypes = [C.c_void_p, C.POINTER(abi.InverseConfig)]
        L.smcrt_job_targets.argtypes = [C.c_void_p, C.POINTER(C.c_double)]
        L.smcrt_job_run_escape.argtypes = [C.c_void_p, C.c_int32, C.c_char_p]
        L.smcrt_job_run_inverse.argtypes = [C.c_void_p, C.c_int32, C.c_int32, C.POINTER(C.c_double)]
        _declared = True
    return L


def _check(st):
    if st != abi.OK:
        raise SmcrtError(f"{abi.STATUS_NAMES.get(st, st)}: {load_library().smcrt_last_error().decode(errors='replace')}")


class Job:
    """A parsed input file (smcrt_job_load_mode). mode: "default", "escape" (the
    -DescapeFunction build: [symmetry]) or "inverse" (-DinverseMCRT: [inverse])."""

    MODES = {"default": abi.JOB_DEFAULT, "escape": abi.JOB_ESCAPE, "inverse": abi.JOB_INVERSE}

    def __init__(self, toml_path, mode: str = "default"):
        L = _lib()
        h = C.c_void_p()
        self.mode = mode
        _check(L.smcrt_job_load_mode(str(toml_path).encode(), self.MODES[mode], C.byref(h)))
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

    def targets(self):
        """inverseTarget of each detector (-1: none)."""
        t = (C.c_double * max(1, self.desc.n_dets))()
        _check(_lib().smcrt_job_targets(self._h, t))
        return [t[i] for i in range(self.desc.n_dets)]

    def escape_config(self) -> abi.EscapeConfig:
        c = abi.EscapeConfig()
        _check(_lib().smcrt_job_escape_config(self._h, C.byref(c)))
        return c

    def inverse_config(self) -> abi.InverseConfig:
        c = abi.InverseConfig()
        _check(_lib().smcrt_job_inverse_config(self._h, C.byref(c)))
        return c

    def run_escape(self, outdir, device: int = 0):
        """escape_Function: the batched escape run, write_escape and finalise under outdir."""
        _check(_lib().smcrt_job_run_escape(self._h, device, str(outdir).encode()))

    def run_inverse(self, device: int = 0, apply_trial: bool = False):
        """inverse_MCRT: gradDescentData (maxNumSteps, 5) as a numpy array."""
        import numpy as np
        m = self.inverse_config().max_steps
        out = np.zeros((5, m))  # Fortran (maxNumSteps, 5): column c contiguous
        _check(_lib().smcrt_job_run_inverse(self._h, device, 1 if apply_trial else 0,
                                            out.ctypes.data_as(C.POINTER(C.c_double))))
        return out.T.copy()
