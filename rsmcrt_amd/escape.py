"""Escape function (kernelsMod.f90:85-1460, the reference's -DescapeFunction build): the
symmetry-grid config and the host-side steps of the C ABI (include/smcrt.h).

The GPU part is `Engine.escape` (all launch cells in one batched launch) and
`Engine.run_origins`; the functions here are host-only (launch cells, symmetry-grid shape,
interpolation onto the fluence grid) and run without a GPU.
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from . import abi
from .engine import _check, load_library


def escape_config(symmetry="none", grid_size=(10, 10, 10), max_values=(1.0, 1.0, 1.0), position=(0.0, 0.0, 0.0),
                  direction=(0.0, 0.0, 1.0), rotation=0.0) -> abi.EscapeConfig:
    """The [symmetry] table (parse.f90:188-340) with the parser's defaults."""
    c = abi.EscapeConfig()
    c.symmetry = abi.SYMMETRY_KINDS[symmetry] if isinstance(symmetry, str) else int(symmetry)
    for i in range(3):
        c.n[i] = int(grid_size[i])
        c.max[i] = float(max_values[i])
        c.pos[i] = float(position[i])
        c.dir[i] = float(direction[i])
    c.rotation = float(rotation)
    return c


def sym_dims(cfg: abi.EscapeConfig):
    d = (C.c_int32 * 3)()
    _check(load_library().smcrt_escape_sym_dims(C.byref(cfg), d))
    return tuple(d)


def cells(cfg: abi.EscapeConfig):
    """Launch cells in the reference's loop order: (indices (k, 3) 1-based, positions (k, 3))."""
    L = load_library()
    n = C.c_int64()
    _check(L.smcrt_escape_cells(C.byref(cfg), C.byref(n), None, None))
    idx = np.zeros((n.value, 3), dtype=np.int32)
    pos = np.zeros((n.value, 3))
    _check(L.smcrt_escape_cells(C.byref(cfg), C.byref(n), idx.ctypes.data_as(C.POINTER(C.c_int32)),
                                pos.ctypes.data_as(C.POINTER(C.c_double))))
    return idx, pos


def map_to_grid(cfg: abi.EscapeConfig, grid: abi.Grid, escape_sym):
    """escapeSymmetry (n_dets, n0, n1, n2) -> escape (n_dets, nx, ny, nz), both fp32."""
    es = np.asarray(escape_sym, dtype=np.float32)
    nd = es.shape[0]
    src = np.ascontiguousarray(es.transpose(3, 2, 1, 0))  # Fortran order, detector fastest
    out = np.zeros((grid.nz, grid.ny, grid.nx, max(nd, 1)), dtype=np.float32)
    _check(load_library().smcrt_escape_map(C.byref(cfg), C.byref(grid), nd, src.ctypes.data_as(C.POINTER(C.c_float)),
                                           out.ctypes.data_as(C.POINTER(C.c_float))))
    return out.transpose(3, 2, 1, 0)[:nd]
