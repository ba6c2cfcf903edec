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

import numpy as np

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
        L.smcrt_scene_fence.argtypes = [C.c_void_p, C.c_void_p]
        L.smcrt_scene_check.argtypes = [C.c_void_p]
        L.smcrt_scene_kernel_times.argtypes = [C.c_void_p, C.POINTER(abi.KernelTimes)]
        L.smcrt_normalise_fluence.argtypes = [C.POINTER(C.c_float), C.POINTER(abi.Grid), C.c_uint64]
        L.smcrt_scene_info.argtypes = [C.c_void_p, C.POINTER(abi.Grid), C.POINTER(C.c_int32), C.POINTER(C.c_int32)]
        L.smcrt_run_origins.argtypes = [C.c_void_p, C.POINTER(abi.Source), C.POINTER(C.c_double), C.c_int64,
                                        C.POINTER(abi.RunConfig), C.POINTER(C.c_double), C.POINTER(abi.Tallies)]
        L.smcrt_scene_classify.argtypes = [C.c_void_p, C.POINTER(C.c_double), C.c_int64, C.POINTER(C.c_int32),
                                           C.POINTER(C.c_double)]
        L.smcrt_scene_get_optprops.argtypes = [C.c_void_p, C.c_int32, C.POINTER(C.c_int32)] + [C.POINTER(C.c_double)] * 4
        L.smcrt_inverse_run.argtypes = [C.c_void_p, C.POINTER(abi.Source), C.POINTER(abi.InverseConfig),
                                        C.POINTER(abi.RunConfig), C.POINTER(C.c_double), C.POINTER(C.c_double),
                                        C.POINTER(abi.Tallies)]
        L.smcrt_escape_sym_dims.argtypes = [C.POINTER(abi.EscapeConfig), C.POINTER(C.c_int32)]
        L.smcrt_escape_cells.argtypes = [C.POINTER(abi.EscapeConfig), C.POINTER(C.c_int64), C.POINTER(C.c_int32),
                                         C.POINTER(C.c_double)]
        L.smcrt_escape_map.argtypes = [C.POINTER(abi.EscapeConfig), C.POINTER(abi.Grid), C.c_int32,
                                       C.POINTER(C.c_float), C.POINTER(C.c_float)]
        L.smcrt_escape_run.argtypes = [C.c_void_p, C.POINTER(abi.Source), C.POINTER(abi.EscapeConfig),
                                       C.POINTER(abi.RunConfig), C.POINTER(C.c_float), C.POINTER(C.c_float),
                                       C.POINTER(abi.Tallies)]
        L.smcrt_pack_size.argtypes = [C.POINTER(abi.PackLayout), C.POINTER(C.c_int64)]
        L.smcrt_pack_host.argtypes = [C.POINTER(abi.PackLayout), C.POINTER(abi.Tallies), C.POINTER(C.c_double)]
        L.smcrt_unpack_host.argtypes = [C.POINTER(abi.PackLayout), C.POINTER(C.c_double), C.POINTER(abi.Tallies)]
        L.smcrt_comm_unique_id.argtypes = [C.POINTER(C.c_uint8)]
        L.smcrt_comm_init_rank.argtypes = [C.POINTER(C.c_uint8), C.c_int32, C.c_int32, C.c_int32,
                                           C.POINTER(C.c_void_p)]
        L.smcrt_comm_info.argtypes = [C.c_void_p, C.POINTER(C.c_int32), C.POINTER(C.c_int32), C.POINTER(C.c_int32)]
        L.smcrt_comm_destroy.argtypes = [C.c_void_p]
        L.smcrt_comm_destroy.restype = None
        L.smcrt_reduce_device_tallies.argtypes = [C.c_void_p, C.c_void_p, C.POINTER(abi.DeviceTallies), C.c_int32,
                                                  C.c_void_p]
        L.smcrt_multi_create.argtypes = [C.POINTER(abi.SdfNode), C.c_int32, C.POINTER(C.c_int32), C.c_int32,
                                         C.POINTER(abi.Grid), C.POINTER(abi.Detector), C.c_int32,
                                         C.POINTER(C.c_int32), C.c_int32, C.POINTER(C.c_void_p)]
        L.smcrt_multi_info.argtypes = [C.c_void_p, C.POINTER(C.c_int32)]
        L.smcrt_multi_scene.argtypes = [C.c_void_p, C.c_int32]
        L.smcrt_multi_scene.restype = C.c_void_p
        L.smcrt_multi_run.argtypes = [C.c_void_p, C.POINTER(abi.Source), C.POINTER(abi.RunConfig),
                                      C.POINTER(abi.Tallies)]
        L.smcrt_multi_accumulate.argtypes = [C.c_void_p, C.POINTER(abi.Source), C.POINTER(abi.RunConfig)]
        L.smcrt_multi_collect.argtypes = [C.c_void_p, C.POINTER(abi.Tallies)]
        L.smcrt_multi_device_photons.argtypes = [C.c_void_p, C.POINTER(C.c_uint64)]
        L.smcrt_multi_destroy.argtypes = [C.c_void_p]
        L.smcrt_multi_destroy.restype = None
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

    def set_spectral(self, top_index: int, sp, mode: int = abi.SPECTRAL_UPDATE) -> float:
        """Re-sample spectral layer `sp` (rsmcrt_amd.spectral.Spectral; updateSpectral by
        default) into top-level SDF `top_index` (smcrt_scene_set_spectral); returns the
        wavelength. sp's stream position and current values advance with it."""
        from .spectral import _lib
        d = C.c_uint64(sp.draw)
        out = abi.OptProps()
        _check(_lib().smcrt_scene_set_spectral(self._h, top_index, C.byref(sp.struct()), int(mode), sp.seed,
                                               C.byref(d), C.byref(out)))
        sp.draw, sp.props = d.value, out
        return out.wavelength

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

    def run_origins(self, origins, n_photons, source=None, seed=123456789, flags=abi.FLAG_PATHLENGTH,
                    first_photon=0, result: Result | None = None):
        """Photons [first_photon, first_photon + n_photons) from an isotropic point source at each
        of `origins` (k, 3), in one batched launch (smcrt_run_origins). Returns (totals (k, n_dets),
        Result of all origins' tallies)."""
        org = np.ascontiguousarray(origins, dtype=np.float64).reshape(-1, 3)
        k = len(org)
        res = result if result is not None else Result(self.grid, self.dets, 0)
        res.n_photons += int(n_photons) * k
        tot = np.zeros((k, max(1, len(self.dets))))
        cfg = self.config(n_photons, seed, flags, first_photon)
        t = res.tallies()
        _check(load_library().smcrt_run_origins(self._h, C.byref(source) if source is not None else None,
                                                org.ctypes.data_as(C.POINTER(C.c_double)), k, C.byref(cfg),
                                                tot.ctypes.data_as(C.POINTER(C.c_double)), C.byref(t)))
        return tot[:, :len(self.dets)], res

    def classify(self, points):
        """(layer, kappa) of each point: maxloc(ds, mask=ds<0) over the top-level SDFs."""
        pts = np.ascontiguousarray(points, dtype=np.float64).reshape(-1, 3)
        lay = np.zeros(len(pts), dtype=np.int32)
        kap = np.zeros(len(pts))
        _check(load_library().smcrt_scene_classify(self._h, pts.ctypes.data_as(C.POINTER(C.c_double)), len(pts),
                                                   lay.ctypes.data_as(C.POINTER(C.c_int32)),
                                                   kap.ctypes.data_as(C.POINTER(C.c_double))))
        return lay, kap

    def escape(self, cfg: abi.EscapeConfig, n_photons, source=None, seed=123456789, flags=abi.FLAG_PATHLENGTH,
               result: Result | None = None):
        """The escape function (smcrt_escape_run): (escape_sym (n_dets, n0, n1, n2), escape
        (n_dets, nx, ny, nz), Result). Arrays are fp32 in the reference's index order."""
        from .escape import sym_dims
        n0, n1, n2 = sym_dims(cfg)
        nd = len(self.dets)
        es = np.zeros((n2, n1, n0, max(nd, 1)), dtype=np.float32)
        e = np.zeros((self.grid.nz, self.grid.ny, self.grid.nx, max(nd, 1)), dtype=np.float32)
        res = result if result is not None else Result(self.grid, self.dets, 0)
        rc = self.config(n_photons, seed, flags, 0)
        t = res.tallies()
        _check(load_library().smcrt_escape_run(self._h, C.byref(source) if source is not None else None, C.byref(cfg),
                                               C.byref(rc), es.ctypes.data_as(C.POINTER(C.c_float)),
                                               e.ctypes.data_as(C.POINTER(C.c_float)), C.byref(t)))
        return es.transpose(3, 2, 1, 0)[:nd], e.transpose(3, 2, 1, 0)[:nd], res

    def get_optprops(self, top_index: int):
        """(layer, mus, mua, hgg, n) as the reference's getters return them (mus = kappa - mua)."""
        lay = C.c_int32()
        v = [C.c_double() for _ in range(4)]
        _check(load_library().smcrt_scene_get_optprops(self._h, top_index, C.byref(lay), *[C.byref(x) for x in v]))
        return (lay.value, *[x.value for x in v])

    def inverse(self, source, cfg: abi.InverseConfig, n_photons, targets, seed=123456789,
                flags=abi.FLAG_PATHLENGTH, result: Result | None = None):
        """inverse_MCRT on the resident scene: gradDescentData (max_steps, 5)."""
        m = cfg.max_steps
        out = np.zeros((5, m))
        tg = np.ascontiguousarray(targets, dtype=np.float64)
        rc = self.config(n_photons, seed, flags, 0)
        t = result.tallies() if result is not None else None
        _check(load_library().smcrt_inverse_run(self._h, C.byref(source), C.byref(cfg), C.byref(rc),
                                                tg.ctypes.data_as(C.POINTER(C.c_double)),
                                                out.ctypes.data_as(C.POINTER(C.c_double)),
                                                C.byref(t) if t is not None else None))
        return out.T.copy()

    def run_device(self, source, cfg: abi.RunConfig, dev: abi.DeviceTallies, stream: int = 0):
        """Asynchronous launch into caller-owned device buffers on `stream` (hipStream_t)."""
        _check(load_library().smcrt_run_device(self._h, C.byref(source), C.byref(cfg), C.byref(dev),
                                               C.c_void_p(stream)))

    def reduce_device_tallies(self, comm: "Comm", dev: abi.DeviceTallies, root: int = -1, stream: int = 0):
        """Sum this rank's device tallies over `comm` with one packed RCCL collective
        (all-reduce for root < 0, else reduce onto rank `root`), asynchronously on `stream`."""
        _check(load_library().smcrt_reduce_device_tallies(self._h, comm._h, C.byref(dev), int(root),
                                                          C.c_void_p(stream)))

    def fence(self, stream: int = 0):
        """Make `stream` wait for the deposit folds of FLAG_ASYNC_FOLD launches."""
        _check(load_library().smcrt_scene_fence(self._h, C.c_void_p(stream)))

    def check(self):
        """Wait for the scene's launches and folds; raise SmcrtError (DEVICE_FAULT, naming the
        wait site) if the watchdog fired in any of them (smcrt_scene_check)."""
        _check(load_library().smcrt_scene_check(self._h))

    def set_timing(self, enable: bool = True):
        """Record HIP events around each kernel group of later launches."""
        _check(load_library().smcrt_scene_set_timing(self._h, 1 if enable else 0))

    def kernel_times(self) -> dict:
        """Device ms per kernel group since the previous call (waits for those launches)."""
        t = abi.KernelTimes()
        _check(load_library().smcrt_scene_kernel_times(self._h, C.byref(t)))
        return {"transport_ms": t.transport_ms, "deposit_ms": t.deposit_ms, "launches": t.launches,
                "lean_launches": t.lean_launches, "far_steps": t.far_steps,
                "fold_cu_ms": t.fold_cu_ms, "lean_hazards": t.lean_hazards}


def pack_layout(grid, n_det_bins: int, fields: int) -> abi.PackLayout:
    lay = abi.PackLayout()
    lay.n_voxels, lay.n_det_bins, lay.fields = grid.nx * grid.ny * grid.nz, int(n_det_bins), int(fields)
    return lay


def pack_result(res: Result, fields: int) -> np.ndarray:
    """A host Result as the packed fp64 buffer of the multi-GPU reduction (smcrt_pack_host)."""
    L = load_library()
    lay = pack_layout(res.grid, sum(res.det_sizes), fields)
    n = C.c_int64()
    _check(L.smcrt_pack_size(C.byref(lay), C.byref(n)))
    buf = np.zeros(n.value)
    t = res.tallies()
    _check(L.smcrt_pack_host(C.byref(lay), C.byref(t), buf.ctypes.data_as(C.POINTER(C.c_double))))
    return buf


def unpack_into(res: Result, buf: np.ndarray, fields: int) -> Result:
    """Accumulate a packed buffer into a host Result (smcrt_unpack_host)."""
    L = load_library()
    lay = pack_layout(res.grid, sum(res.det_sizes), fields)
    b = np.ascontiguousarray(buf, dtype=np.float64)
    t = res.tallies()
    _check(L.smcrt_unpack_host(C.byref(lay), b.ctypes.data_as(C.POINTER(C.c_double)), C.byref(t)))
    return res


class Comm:
    """An RCCL communicator of one process per GPU (smcrt_comm_init_rank). Rank 0 makes the
    id with `unique_id()`; the caller hands it to the other ranks out of band."""

    @staticmethod
    def unique_id() -> bytes:
        buf = (C.c_uint8 * abi.UNIQUE_ID_BYTES)()
        _check(load_library().smcrt_comm_unique_id(buf))
        return bytes(buf)

    def __init__(self, uid: bytes, n_ranks: int, rank: int, device: int):
        buf = (C.c_uint8 * abi.UNIQUE_ID_BYTES).from_buffer_copy(uid)
        h = C.c_void_p()
        _check(load_library().smcrt_comm_init_rank(buf, int(n_ranks), int(rank), int(device), C.byref(h)))
        self._h = h

    def info(self) -> dict:
        """The communicator's rank count and rank as RCCL reports them, and its device."""
        n, r, d = C.c_int32(), C.c_int32(), C.c_int32()
        _check(load_library().smcrt_comm_info(self._h, C.byref(n), C.byref(r), C.byref(d)))
        return {"n_ranks": n.value, "rank": r.value, "device": d.value}

    @property
    def n_ranks(self) -> int:
        return self.info()["n_ranks"]

    def close(self):
        if getattr(self, "_h", None):
            load_library().smcrt_comm_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class MultiEngine:
    """One process driving several GPUs (smcrt_multi_*): photon chunks handed to whichever
    device is free, accumulated on the devices, one packed RCCL reduce per `collect`. `run`
    (= accumulate + collect) has Engine.run's semantics (without photon records)."""

    def __init__(self, scene, grid, dets=(), devices=None):
        L = load_library()
        self.scene, self.grid, self.dets = scene, grid, list(dets)
        self._nodes = scene.node_array()
        self._top = scene.top_array()
        self._darr = detector_array(self.dets)
        devs = None if devices is None else (C.c_int32 * len(devices))(*devices)
        h = C.c_void_p()
        _check(L.smcrt_multi_create(self._nodes, len(scene.nodes), self._top, scene.n_top, C.byref(grid),
                                    self._darr, len(self.dets), devs, len(devices) if devices else 0, C.byref(h)))
        self._h = h
        n = C.c_int32()
        _check(L.smcrt_multi_info(h, C.byref(n)))
        self.n_devices = n.value
        self._pending = 0  # photons accumulated on the devices, not collected yet

    def close(self):
        if getattr(self, "_h", None):
            load_library().smcrt_multi_destroy(self._h)
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

    def run(self, source, n_photons, seed=123456789, flags=abi.FLAG_PATHLENGTH, first_photon=0,
            result: Result | None = None) -> Result:
        res = result if result is not None else Result(self.grid, self.dets, n_photons)
        res.n_photons += int(n_photons) + self._pending
        self._pending = 0
        cfg = Engine.config(n_photons, seed, flags, first_photon)
        t = res.tallies()
        _check(load_library().smcrt_multi_run(self._h, C.byref(source), C.byref(cfg), C.byref(t)))
        return res

    def accumulate(self, source, n_photons, seed=123456789, flags=abi.FLAG_PATHLENGTH, first_photon=0):
        """Launch photons [first_photon, +n_photons) over the devices; nothing is waited for."""
        cfg = Engine.config(n_photons, seed, flags, first_photon)
        try:
            _check(load_library().smcrt_multi_accumulate(self._h, C.byref(source), C.byref(cfg)))
        except SmcrtError:
            self._pending = 0  # (the library discarded everything since the last collect)
            raise
        self._pending += int(n_photons)

    def device_photons(self):
        """Photons each device ran since the last collect."""
        out = (C.c_uint64 * self.n_devices)()
        _check(load_library().smcrt_multi_device_photons(self._h, out))
        return list(out)

    def collect(self, result: Result | None = None) -> Result:
        """One packed RCCL reduce of everything accumulated since the last collect."""
        res = result if result is not None else Result(self.grid, self.dets, 0)
        held = sum(self.device_photons())  # the library's own count of what the accumulators hold
        if held != self._pending:  # (before any tally is reduced or normalised with it)
            raise SmcrtError(f"multi-device photon count mismatch: the devices hold {held} photons, "
                             f"{self._pending} were accumulated since the last collect")
        res.n_photons += held
        self._pending = 0
        t = res.tallies()
        _check(load_library().smcrt_multi_collect(self._h, C.byref(t)))
        return res
