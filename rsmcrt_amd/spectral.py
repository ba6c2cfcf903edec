"""Spectral optical properties: the reference's `spectral` type (opticalProperties.f90:51-55,
127-201) over five piecewise1D tables (piecewise.f90:109-168).

    optProp = spectral(mus_a, mua_a, hgg_a, n_a, flux)     ! init_spectral
    call optProp%update(wave)                               ! updateSpectral

becomes

    sp = spectral(mus_a, mua_a, hgg_a, n_a, flux, seed=...)  # Spectral, current values set
    wave = sp.update()

Each table is an (n, 2) array as the reference takes it (column 1 the wavelength, column 2 the
value). The sampling runs in libsmcrt.so (smcrt_spectral_sample, include/smcrt.h ABI 5) on a
host Philox stream keyed by `seed`; `draw` is the position in it. A Spectral can stand where an
SDF constructor takes its optical properties (scene.sphere(1.0, sp, 1)): the node takes the
current values and the albedo rule they need. Engine.set_spectral re-samples a resident
scene's layer between runs.
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from . import abi


def _lib():
    from .engine import load_library
    L = load_library()
    if not getattr(L, "_spectral_declared", False):
        L.smcrt_spectral_sample.argtypes = [C.POINTER(abi.Spectral), C.c_int32, C.c_uint64, C.POINTER(C.c_uint64),
                                            C.POINTER(abi.OptProps)]
        L.smcrt_scene_set_spectral.argtypes = [C.c_void_p, C.c_int32, C.POINTER(abi.Spectral), C.c_int32,
                                               C.c_uint64, C.POINTER(C.c_uint64), C.POINTER(abi.OptProps)]
        L._spectral_declared = True
    return L


class Spectral:
    """A spectral layer: its tables, its stream position and its current properties."""

    NAMES = ("mus", "mua", "hgg", "n", "flux")

    def __init__(self, mus, mua, hgg, n, flux, seed: int = 123456789, mode: int = abi.SPECTRAL_INIT):
        self.tables = {}
        for name, a in zip(self.NAMES, (mus, mua, hgg, n, flux)):
            a = np.asarray(a, dtype=np.float64)
            if a.ndim != 2 or a.shape[1] != 2 or a.shape[0] < 2:  # piecewise.f90:153
                raise ValueError(f"{name}: array must be size (n, 2) with n >= 2, got {a.shape}")
            self.tables[name] = np.asfortranarray(a)
        self.seed = int(seed)
        self.draw = 0
        self.props = abi.OptProps()
        self._sample(mode)

    def struct(self) -> abi.Spectral:
        sp = abi.Spectral()
        for name in self.NAMES:
            a = self.tables[name]
            setattr(sp, "n_" + name, a.shape[0])
            setattr(sp, name, a.ctypes.data_as(C.POINTER(C.c_double)))
        return sp

    def _sample(self, mode: int) -> float:
        from .engine import _check
        d = C.c_uint64(self.draw)
        out = abi.OptProps()
        _check(_lib().smcrt_spectral_sample(C.byref(self.struct()), int(mode), self.seed, C.byref(d), C.byref(out)))
        self.draw, self.props = d.value, out
        return out.wavelength

    def update(self) -> float:
        """updateSpectral (:171-201): a new wavelength and the properties there; returns it."""
        return self._sample(abi.SPECTRAL_UPDATE)

    # opticalProp_base's fields
    mus = property(lambda self: self.props.mus)
    mua = property(lambda self: self.props.mua)
    hgg = property(lambda self: self.props.hgg)
    g2 = property(lambda self: self.props.g2)
    n = property(lambda self: self.props.n)
    kappa = property(lambda self: self.props.kappa)
    albedo = property(lambda self: self.props.albedo)
    wavelength = property(lambda self: self.props.wavelength)
    flags = property(lambda self: self.props.node_flags)

    def mono(self):
        """The current values as a scene.Mono (with the albedo rule they need)."""
        from .scene import Mono
        p = self.props
        return Mono(p.mus, p.mua, p.hgg, p.n, p.node_flags)


def spectral(mus, mua, hgg, n, flux, seed: int = 123456789, mode: int = abi.SPECTRAL_INIT) -> Spectral:
    """init_spectral (opticalProperties.f90:127-156); mode abi.SPECTRAL_INIT_AS_WRITTEN samples
    as the compiled Fortran does (include/smcrt.h)."""
    return Spectral(mus, mua, hgg, n, flux, seed, mode)
