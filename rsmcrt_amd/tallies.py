"""Host-side tally containers (numpy views laid out as include/smcrt.h expects)."""
from __future__ import annotations

import ctypes as C

import numpy as np

from . import abi
from .scene import det_sizes


def _dp(a):
    return a.ctypes.data_as(C.POINTER(C.c_double))


class Result:
    """Tallies of one or more runs, accumulated in fp64.

    Grids are numpy arrays of shape (nz, ny, nx): the C view of the reference's Fortran
    jmean(nx, ny, nz) (x fastest, src/iarray.f90:12-16)."""

    def __init__(self, grid, dets=(), n_photons=0, records=False):
        shape = (grid.nz, grid.ny, grid.nx)
        self.grid = grid
        self.jmean = np.zeros(shape)
        self.absorb = np.zeros(shape)
        self.emission = np.zeros(shape)
        self.det_sizes = det_sizes(list(dets))
        self.det_bins = np.zeros(max(1, sum(self.det_sizes)))
        self.nscatt = np.zeros(1)
        self.moments = np.zeros(24)
        self.counters = np.zeros(abi.NCOUNTERS, dtype=np.uint64)
        self.records = np.zeros(n_photons if records else 0, dtype=abi.record_dtype())
        self.n_photons = 0

    def tallies(self) -> abi.Tallies:
        t = abi.Tallies()
        t.jmean_f64 = _dp(self.jmean)
        t.absorb_f64 = _dp(self.absorb)
        t.emission_f64 = _dp(self.emission)
        t.det_bins = _dp(self.det_bins)
        t.nscatt = _dp(self.nscatt)
        t.moments = _dp(self.moments)
        t.counters = self.counters.ctypes.data_as(C.POINTER(C.c_uint64))
        if self.records.size:
            t.records = self.records.ctypes.data_as(C.POINTER(abi.PhotonRecord))
        return t

    def counter(self, name: str) -> int:
        return int(self.counters[abi.CTR[name]])

    def counters_dict(self, engine: bool = False):
        """Counter name -> value; engine diagnostics (abi.ENGINE_COUNTERS) only if `engine`."""
        return {n: int(v) for n, v in zip(abi.COUNTER_NAMES, self.counters)
                if engine or n not in abi.ENGINE_COUNTERS}

    def merge(self, other: "Result") -> "Result":
        """Add another Result of the same grid/detectors (disjoint photon ranges)."""
        for f in ("jmean", "absorb", "emission", "det_bins", "nscatt", "moments", "counters"):
            getattr(self, f)[...] += getattr(other, f)
        self.n_photons += other.n_photons
        return self

    def detector(self, i: int) -> np.ndarray:
        off = sum(self.det_sizes[:i])
        return self.det_bins[off:off + self.det_sizes[i]]

    def normalised_fluence(self) -> np.ndarray:
        """normalise_fluence (writer.f90:25-52): jmean * nx*ny*nz / nphotons, in fp64."""
        g = self.grid
        f = (2.0 * g.xmax * 2.0 * g.ymax * 2.0 * g.zmax) / (
            self.n_photons * (2.0 * g.xmax / g.nx) * (2.0 * g.ymax / g.ny) * (2.0 * g.zmax / g.nz))
        return self.jmean * f
