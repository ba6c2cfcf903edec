"""Python front end of the HIP engine (rsmcrt_amd/libsmcrt.so, C ABI include/smcrt.h).

`Engine` mirrors the reference seam run_MCRT (src/kernelsMod.f90:1790-1898): build it once
per scene (the SDF table, grid and detectors go to the GPU and stay resident), then call
`run` for a batch of photons; tallies accumulate like the reference's module globals
jmean/absorb/emission, nscatt and the detector data.

There is no CPU fallback: if the library is missing or no GPU is visible, construction
raises.
"""
from __future__ import annotations

import ctypes as C
import os
import threading

from . import abi
from .scene import detector_array
from .tallies import Result

LIB_PATH = os.environ.get("SMCRT_LIB") or os.path.join(os.path.dirname(os.path.abspath(__file__)), "libsmcrt.so")
_lock = threading.Lock()
_lib = None


class SmcrtError(RuntimeError):
    pass


def load_library(path: str = LIB_PATH):
    """Load libsmcrt.so and declare its prototypes. Raises if it is absent."""
    global _lib
    with _lock:
        if _lib is not None:
            return _lib
        if not os.path.exists(path):
            raise SmcrtError(f"HIP engine library not built: {path} (run __graft_entry__.build())")
        L = C.CDLL(path)
        L.smcrt_abi_version.restype = C.c_int
        L.smcrt_device_count.argtypes = [C.POINTER(C.c_int32)]
        L.smcrt_last_error.restype = C.c_char_p
        L.smcrt_scene_create.argtypes = [C.POINTER(abi.SdfNode), C.c_int32, C.POINTER(C.c_int32), C.c_int32,
                                         C.POINTER(abi.Grid), C.POINTER(abi.Detector), C.c_int32, C.c_int32,
                                         C.POINTER(C.c_void_p)]
        L.smcrt_scene_destroy.argtypes = [C.c_void_p]
        L.smcrt_scene_destroy.restype = None
        L.smcrt_scene_det_bins.argtypes = [C.c_void_p, C.POINTER(C.c_int64)]
        L.smcrt_scene_set_optprops.argtypes = [C.c_void_p, C.c_int32, C.c_double, C.c_double, C.c_double,
                                               C.c_double]
        L.smcrt_run.argtypes = [C.c_void_p, C.POINTER(abi.Source), C.POINTER(abi.RunConfig), C.POINTER(abi.Tallies)]
        L.smcrt_run_device.argtypes = [C.c_void_p, C.POINTER(abi.Source), C.POINTER(abi.RunConfig),
                                       C.POINTER(abi.DeviceTallies), C.c_void_p]
        L.smcrt_scene_set_timing.argtypes = [C.c_void_p, C.c_int32]
        L.smcrt_scene_kernel_times.argtypes = [C.c_void_p, C.POINTER(abi.KernelTimes)]
        L.smcrt_normalise_fluence.argtypes = [C.POINTER(C.c_float), C.POINTER(abi.Grid), C.c_uint64]
        if L.smcrt_abi_version() != abi.SMCRT_ABI_VERSION:
            raise SmcrtError("libsmcrt.so ABI version mismatch")
        _lib = L
        return L


def _check(st: int):
    if st != abi.OK:
        msg = load_library().smcrt_last_error().decode(errors="replace")
        raise SmcrtError(f"{abi.STATUS_NAMES.get(st, st)}: {msg}")


def device_count() -> int:
    n = C.c_int32()
    _check(load_library().smcrt_device_count(C.byref(n)))
    return n.value


class Engine:
    """A scene resident on one GPU (smcrt_scene_create)."""

    def __init__(self, scene, grid, dets=(), device: int = 0):
        L = load_library()
        self.scene, self.grid, self.dets, self.device = scene, grid, list(dets), device
        self._nodes = scene.node_array()
        self._top = scene.top_array()
        self._darr = detector_array(self.dets)
        h = C.c_void_p()
        _check(L.smcrt_scene_create(self._nodes, len(scene.nodes), self._top, scene.n_top, C.byref(grid),
                                    self._darr, len(self.dets), device, C.byref(h)))
        self._h = h

    def close(self):
        if getattr(self, "_h", None):
            load_library().smcrt_scene_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def set_optprops(self, top_index: int, mus, mua, hgg, n):
        _check(load_library().smcrt_scene_set_optprops(self._h, top_index, mus, mua, hgg, n))

    @staticmethod
    def config(n_photons, seed=123456789, flags=abi.FLAG_PATHLENGTH, first_photon=0) -> abi.RunConfig:
        cfg = abi.RunConfig()
        cfg.n_photons, cfg.first_photon, cfg.seed, cfg.flags = int(n_photons), int(first_photon), int(seed), int(flags)
        return cfg

    def run(self, source, n_photons, seed=123456789, flags=abi.FLAG_PATHLENGTH, first_photon=0,
            records=False, result: Result | None = None) -> Result:
        """Synchronous run_MCRT: returns host tallies (accumulated into `result` if given)."""
        res = result if result is not None else Result(self.grid, self.dets, n_photons, records)
        res.n_photons += int(n_photons)
        cfg = self.config(n_photons, seed, flags | (abi.FLAG_RECORD_PHOTONS if records else 0), first_photon)
        t = res.tallies()
        _check(load_library().smcrt_run(self._h, C.byref(source), C.byref(cfg), C.byref(t)))
        return res

    def run_device(self, source, cfg: abi.RunConfig, dev: abi.DeviceTallies, stream: int = 0):
        """Asynchronous launch into caller-owned device buffers on `stream` (hipStream_t)."""
        _check(load_library().smcrt_run_device(self._h, C.byref(source), C.byref(cfg), C.byref(dev),
                                               C.c_void_p(stream)))

    def set_timing(self, enable: bool = True):
        """Record HIP events around each kernel group of later launches."""
        _check(load_library().smcrt_scene_set_timing(self._h, 1 if enable else 0))

    def kernel_times(self) -> dict:
        """Device ms per kernel group since the previous call (waits for those launches)."""
        t = abi.KernelTimes()
        _check(load_library().smcrt_scene_kernel_times(self._h, C.byref(t)))
        return {"transport_ms": t.transport_ms, "deposit_ms": t.deposit_ms, "launches": t.launches}
