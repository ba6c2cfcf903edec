"""Scene description: SDF primitives, CSG models, grid, sources and detectors.

Host-side mirror of the reference's object constructors, so a scene is assembled the way
the Fortran builders assemble it and then flattened into the POD node table of
include/smcrt.h:

  SDF constructors      src/sdfs/sdfs.f90:158-492       (box halves its lengths, :455)
  model                 src/sdfs/sdf_base.f90:104-144   (optical props of the first child)
  mono optical props    src/opticalProps/opticalProperties.f90:107-125
  transforms            src/sdfs/sdfHelpers.f90, src/mat_class.f90:154-207 (invert)
  cart_grid             src/grid.f90:119-159
  detectors             src/detectors/detectors.f90:122-145 (circle), 166-210 (annulus),
                        401-445 (camera)
  scene builders        src/setupGeometry.f90 (see rsmcrt_amd.builders)

All arithmetic on transforms is done in Python floats (IEEE binary64) in the reference's
operation order, so the transforms equal the Fortran ones.
"""
from __future__ import annotations

import ctypes as C
import math
from dataclasses import dataclass, field
from typing import List, Optional, Sequence

import numpy as np

from . import abi

Vec = Sequence[float]


# ------------------------------------------------------------------ 4x4 helpers --
# Matrices are Python lists m[r][c] with r, c in 0..3 (Fortran t(r+1, c+1)).

def identity():
    """sdfHelpers.f90:134-143"""
    return [[1.0 if r == c else 0.0 for c in range(4)] for r in range(4)]


def translate(o: Vec):
    """sdfHelpers.f90:160-171: column c has o(c) in row 4."""
    m = identity()
    m[3][0], m[3][1], m[3][2] = float(o[0]), float(o[1]), float(o[2])
    return m


def deg2rad(a: float) -> float:
    # fortran_utilities deg2rad (un-vendored dependency): a * pi / 180
    return a * math.pi / 180.0


def _cols(c1, c2, c3, c4):
    cols = [c1, c2, c3, c4]
    return [[float(cols[c][r]) for c in range(4)] for r in range(4)]


def rotate_x(angle: float):
    """sdfHelpers.f90:15-31"""
    a = deg2rad(angle); c = math.cos(a); s = math.sin(a)
    return _cols([1, 0, 0, 0], [0, c, -s, 0], [0, s, c, 0], [0, 0, 0, 1])


def rotate_y(angle: float):
    """sdfHelpers.f90:33-50"""
    a = deg2rad(angle); c = math.cos(a); s = math.sin(a)
    return _cols([c, 0, s, 0], [0, 1, 0, 0], [-s, 0, c, 0], [0, 0, 0, 1])


def rotate_z(angle: float):
    """sdfHelpers.f90:52-69"""
    a = deg2rad(angle); c = math.cos(a); s = math.sin(a)
    return _cols([c, -s, 0, 0], [s, c, 0, 0], [0, 0, 1, 0], [0, 0, 0, 1])


def invert(A):
    """Direct 4x4 inverse, term for term as mat_class.f90:154-207 (A(i,j) -> A[i-1][j-1])."""
    a = lambda i, j: A[i - 1][j - 1]  # noqa: E731
    detinv = 1.0 / (a(1, 1) * (a(2, 2) * (a(3, 3) * a(4, 4) - a(3, 4) * a(4, 3))
                               + a(2, 3) * (a(3, 4) * a(4, 2) - a(3, 2) * a(4, 4))
                               + a(2, 4) * (a(3, 2) * a(4, 3) - a(3, 3) * a(4, 2)))
                    - a(1, 2) * (a(2, 1) * (a(3, 3) * a(4, 4) - a(3, 4) * a(4, 3))
                                 + a(2, 3) * (a(3, 4) * a(4, 1) - a(3, 1) * a(4, 4))
                                 + a(2, 4) * (a(3, 1) * a(4, 3) - a(3, 3) * a(4, 1)))
                    + a(1, 3) * (a(2, 1) * (a(3, 2) * a(4, 4) - a(3, 4) * a(4, 2))
                                 + a(2, 2) * (a(3, 4) * a(4, 1) - a(3, 1) * a(4, 4))
                                 + a(2, 4) * (a(3, 1) * a(4, 2) - a(3, 2) * a(4, 1)))
                    - a(1, 4) * (a(2, 1) * (a(3, 2) * a(4, 3) - a(3, 3) * a(4, 2))
                                 + a(2, 2) * (a(3, 3) * a(4, 1) - a(3, 1) * a(4, 3))
                                 + a(2, 3) * (a(3, 1) * a(4, 2) - a(3, 2) * a(4, 1))))
    B = [[0.0] * 4 for _ in range(4)]
    B[0][0] = detinv * (a(2, 2) * (a(3, 3) * a(4, 4) - a(3, 4) * a(4, 3)) + a(2, 3) * (a(3, 4) * a(4, 2) - a(3, 2) * a(4, 4)) + a(2, 4) * (a(3, 2) * a(4, 3) - a(3, 3) * a(4, 2)))
    B[1][0] = detinv * (a(2, 1) * (a(3, 4) * a(4, 3) - a(3, 3) * a(4, 4)) + a(2, 3) * (a(3, 1) * a(4, 4) - a(3, 4) * a(4, 1)) + a(2, 4) * (a(3, 3) * a(4, 1) - a(3, 1) * a(4, 3)))
    B[2][0] = detinv * (a(2, 1) * (a(3, 2) * a(4, 4) - a(3, 4) * a(4, 2)) + a(2, 2) * (a(3, 4) * a(4, 1) - a(3, 1) * a(4, 4)) + a(2, 4) * (a(3, 1) * a(4, 2) - a(3, 2) * a(4, 1)))
    B[3][0] = detinv * (a(2, 1) * (a(3, 3) * a(4, 2) - a(3, 2) * a(4, 3)) + a(2, 2) * (a(3, 1) * a(4, 3) - a(3, 3) * a(4, 1)) + a(2, 3) * (a(3, 2) * a(4, 1) - a(3, 1) * a(4, 2)))
    B[0][1] = detinv * (a(1, 2) * (a(3, 4) * a(4, 3) - a(3, 3) * a(4, 4)) + a(1, 3) * (a(3, 2) * a(4, 4) - a(3, 4) * a(4, 2)) + a(1, 4) * (a(3, 3) * a(4, 2) - a(3, 2) * a(4, 3)))
    B[1][1] = detinv * (a(1, 1) * (a(3, 3) * a(4, 4) - a(3, 4) * a(4, 3)) + a(1, 3) * (a(3, 4) * a(4, 1) - a(3, 1) * a(4, 4)) + a(1, 4) * (a(3, 1) * a(4, 3) - a(3, 3) * a(4, 1)))
    B[2][1] = detinv * (a(1, 1) * (a(3, 4) * a(4, 2) - a(3, 2) * a(4, 4)) + a(1, 2) * (a(3, 1) * a(4, 4) - a(3, 4) * a(4, 1)) + a(1, 4) * (a(3, 2) * a(4, 1) - a(3, 1) * a(4, 2)))
    B[3][1] = detinv * (a(1, 1) * (a(3, 2) * a(4, 3) - a(3, 3) * a(4, 2)) + a(1, 2) * (a(3, 3) * a(4, 1) - a(3, 1) * a(4, 3)) + a(1, 3) * (a(3, 1) * a(4, 2) - a(3, 2) * a(4, 1)))
    B[0][2] = detinv * (a(1, 2) * (a(2, 3) * a(4, 4) - a(2, 4) * a(4, 3)) + a(1, 3) * (a(2, 4) * a(4, 2) - a(2, 2) * a(4, 4)) + a(1, 4) * (a(2, 2) * a(4, 3) - a(2, 3) * a(4, 2)))
    B[1][2] = detinv * (a(1, 1) * (a(2, 4) * a(4, 3) - a(2, 3) * a(4, 4)) + a(1, 3) * (a(2, 1) * a(4, 4) - a(2, 4) * a(4, 1)) + a(1, 4) * (a(2, 3) * a(4, 1) - a(2, 1) * a(4, 3)))
    B[2][2] = detinv * (a(1, 1) * (a(2, 2) * a(4, 4) - a(2, 4) * a(4, 2)) + a(1, 2) * (a(2, 4) * a(4, 1) - a(2, 1) * a(4, 4)) + a(1, 4) * (a(2, 1) * a(4, 2) - a(2, 2) * a(4, 1)))
    B[3][2] = detinv * (a(1, 1) * (a(2, 3) * a(4, 2) - a(2, 2) * a(4, 3)) + a(1, 2) * (a(2, 1) * a(4, 3) - a(2, 3) * a(4, 1)) + a(1, 3) * (a(2, 2) * a(4, 1) - a(2, 1) * a(4, 2)))
    B[0][3] = detinv * (a(1, 2) * (a(2, 4) * a(3, 3) - a(2, 3) * a(3, 4)) + a(1, 3) * (a(2, 2) * a(3, 4) - a(2, 4) * a(3, 2)) + a(1, 4) * (a(2, 3) * a(3, 2) - a(2, 2) * a(3, 3)))
    B[1][3] = detinv * (a(1, 1) * (a(2, 3) * a(3, 4) - a(2, 4) * a(3, 3)) + a(1, 3) * (a(2, 4) * a(3, 1) - a(2, 1) * a(3, 4)) + a(1, 4) * (a(2, 1) * a(3, 3) - a(2, 3) * a(3, 1)))
    B[2][3] = detinv * (a(1, 1) * (a(2, 4) * a(3, 2) - a(2, 2) * a(3, 4)) + a(1, 2) * (a(2, 1) * a(3, 4) - a(2, 4) * a(3, 1)) + a(1, 4) * (a(2, 2) * a(3, 1) - a(2, 1) * a(3, 2)))
    B[3][3] = detinv * (a(1, 1) * (a(2, 2) * a(3, 3) - a(2, 3) * a(3, 2)) + a(1, 2) * (a(2, 3) * a(3, 1) - a(2, 1) * a(3, 3)) + a(1, 3) * (a(2, 1) * a(3, 2) - a(2, 2) * a(3, 1)))
    return B


def _colmajor(m) -> List[float]:
    return [float(m[r][c]) for c in range(4) for r in range(4)]


# ------------------------------------------------------------ optical props ----
@dataclass(frozen=True)
class Mono:
    """mono optical properties (opticalProperties.f90:107-125). flags (smcrt_sdf_node.flags):
    abi.NODE_ALBEDO_UNGUARDED for properties that came from updateSpectral (:198-199), whose
    albedo has no mua < 1e-9 guard (rsmcrt_amd.spectral)."""
    mus: float
    mua: float
    hgg: float
    n: float
    flags: int = 0

    @property
    def kappa(self) -> float:
        return self.mus + self.mua

    @property
    def albedo(self) -> float:
        if self.flags & abi.NODE_ALBEDO_UNGUARDED:
            return self.mus / self.kappa
        return 1.0 if self.mua < 1e-9 else self.mus / self.kappa


def mono(mus, mua, hgg, n) -> Mono:
    return Mono(float(mus), float(mua), float(hgg), float(n))


def _set_opt(nd: abi.SdfNode, o) -> None:
    """A node's optical properties from a Mono (or anything with mus/mua/hgg/n, e.g. a
    rsmcrt_amd.spectral.Spectral's current values) and its derivation flags."""
    nd.mus, nd.mua, nd.hgg, nd.n = float(o.mus), float(o.mua), float(o.hgg), float(o.n)
    nd.flags = int(getattr(o, "flags", 0))


# ------------------------------------------------------------------ SDFs ----------
@dataclass
class SDF:
    kind: int
    opt: Mono
    layer: int
    param: List[float]
    transform: Optional[list] = None  # 4x4, default identity

    def node(self) -> abi.SdfNode:
        nd = abi.SdfNode()
        nd.kind = self.kind
        nd.layer = int(self.layer)
        t = _colmajor(self.transform if self.transform is not None else identity())
        for i, v in enumerate(t):
            nd.transform[i] = v
        for i, v in enumerate(self.param):
            nd.param[i] = float(v)
        _set_opt(nd, self.opt)
        return nd


def sphere(radius, opt, layer, transform=None):
    return SDF(abi.SDF_SPHERE, opt, layer, [radius], transform)


def box(lengths: Vec, opt, layer, transform=None):
    # box_init: out%lengths = .5_wp*lengths (sdfs.f90:455)
    return SDF(abi.SDF_BOX, opt, layer, [0.5 * float(v) for v in lengths], transform)


def torus(oradius, iradius, opt, layer, transform=None):
    return SDF(abi.SDF_TORUS, opt, layer, [oradius, iradius], transform)


def cylinder(a: Vec, b: Vec, radius, opt, layer, transform=None):
    return SDF(abi.SDF_CYLINDER, opt, layer, [*a, *b, radius], transform)


def triprism(h1, h2, opt, layer, transform=None):
    return SDF(abi.SDF_TRIPRISM, opt, layer, [h1, h2], transform)


def segment(a: Vec, b: Vec, opt, layer, transform=None):
    return SDF(abi.SDF_SEGMENT, opt, layer, [*a, *b], transform)


def capsule(a: Vec, b: Vec, r, opt, layer, transform=None):
    return SDF(abi.SDF_CAPSULE, opt, layer, [*a, *b, r], transform)


def cone(a: Vec, b: Vec, ra, rb, opt, layer, transform=None):
    return SDF(abi.SDF_CONE, opt, layer, [*a, *b, ra, rb], transform)


def egg(r1, r2, h, opt, layer, transform=None):
    return SDF(abi.SDF_EGG, opt, layer, [r1, r2, h], transform)


def plane(a: Vec, opt, layer, transform=None):
    return SDF(abi.SDF_PLANE, opt, layer, [*a], transform)


@dataclass
class Model:
    """CSG model: left fold of `op` over `children` (sdf_base.f90:104-161)."""
    children: List[SDF]
    op: int = abi.OP_UNION
    k: float = 0.0

    @property
    def opt(self) -> Mono:
        return self.children[0].opt

    @property
    def layer(self) -> int:
        return self.children[0].layer


def model(children, op=abi.OP_UNION, k=0.0) -> Model:
    return Model(list(children), op, float(k))


@dataclass
class Modifier:
    """A modifier of sdfModifiers.f90 wrapping one SDF (primitive, model or modifier). Like the
    reference's *_init functions it takes the layer and optics of what it wraps; its own
    transform is the identity and is never applied."""
    kind: int
    child: object
    param: List[float]

    @property
    def opt(self) -> Mono:
        return self.child.opt

    @property
    def layer(self) -> int:
        return self.child.layer


def revolution(prim, o, center=(0.0, 0.0, 0.0)) -> Modifier:
    """revolution_init(prim, o, center) sdfModifiers.f90:238-266."""
    return Modifier(abi.SDF_REVOLUTION, prim, [float(o), *map(float, center)])


def extrude(prim, h) -> Modifier:
    """extrude_init(prim, h) :143-159."""
    return Modifier(abi.SDF_EXTRUDE, prim, [float(h)])


def onion(prim, thickness) -> Modifier:
    """onion_init(prim, thickness) :268-284."""
    return Modifier(abi.SDF_ONION, prim, [float(thickness)])


def twist(prim, k) -> Modifier:
    """twist_init(prim, k) :126-141. Its k is a default (single precision) real, so the stored
    k is the float32 rounding of the value, widened."""
    return Modifier(abi.SDF_TWIST, prim, [float(np.float32(k))])


def bend(prim, k) -> Modifier:
    """bend_init(prim, k) :196-212."""
    return Modifier(abi.SDF_BEND, prim, [float(k)])


def elongate(prim, size: Vec) -> Modifier:
    """elongate_init(prim, size) :161-176."""
    return Modifier(abi.SDF_ELONGATE, prim, [float(v) for v in size])


def displacement_sine(prim, amplitude, freq: Vec) -> Modifier:
    """displacement_init(prim, func) :178-194 with the built-in f(p) = a sin(fx x) sin(fy y)
    sin(fz z) (smcrt.h SMCRT_DISP_SINE): the reference takes any procedure(primitive)."""
    return Modifier(abi.SDF_DISPLACEMENT, prim, [float(abi.DISP_SINE), float(amplitude), *map(float, freq)])


class Scene:
    """An ordered sdfs_array (reference index i+1 == tauint2 layer) flattened to nodes."""

    def __init__(self, sdfs):
        self.sdfs = list(sdfs)
        nodes: List[abi.SdfNode] = []
        top: List[int] = []
        # top-level nodes first, children after
        for s in self.sdfs:
            top.append(len(nodes))
            nodes.append(None)
        pending = list(zip(top, self.sdfs))
        while pending:
            idx, s = pending.pop(0)
            if isinstance(s, Modifier):
                nd = abi.SdfNode()
                nd.kind = int(s.kind)
                nd.layer = int(s.layer)
                for i, v in enumerate(_colmajor(identity())):
                    nd.transform[i] = v
                for i, v in enumerate(s.param):
                    nd.param[i] = float(v)
                _set_opt(nd, s.opt)
                nd.first_child = len(nodes)
                nd.n_children = 1
                nodes.append(None)
                pending.append((nd.first_child, s.child))
                nodes[idx] = nd
            elif isinstance(s, Model):
                nd = abi.SdfNode()
                nd.kind = abi.SDF_MODEL
                nd.layer = int(s.layer)
                nd.op = int(s.op)
                nd.k = s.k
                for i, v in enumerate(_colmajor(identity())):
                    nd.transform[i] = v
                _set_opt(nd, s.opt)
                nd.first_child = len(nodes)
                nd.n_children = len(s.children)
                first = len(nodes)
                nodes.extend([None] * len(s.children))
                for j, ch in enumerate(s.children):
                    pending.append((first + j, ch))
                nodes[idx] = nd
            else:
                nodes[idx] = s.node()
        self.nodes = nodes
        self.top = top

    @property
    def n_top(self) -> int:
        return len(self.top)

    def node_array(self):
        arr = (abi.SdfNode * len(self.nodes))()
        for i, nd in enumerate(self.nodes):
            arr[i] = nd
        return arr

    def top_array(self):
        return (C.c_int32 * len(self.top))(*self.top)


# ------------------------------------------------------------------ grid ----------
def grid(nx, ny, nz, xmax, ymax, zmax) -> abi.Grid:
    g = abi.Grid()
    g.nx, g.ny, g.nz = int(nx), int(ny), int(nz)
    g.xmax, g.ymax, g.zmax = float(xmax), float(ymax), float(zmax)
    return g


# ------------------------------------------------------------------ sources -------
def point_source(pos=(0.0, 0.0, 0.0)) -> abi.Source:
    s = abi.Source()
    s.kind = abi.SRC_POINT
    for i in range(3):
        s.pos[i] = float(pos[i])
    return s


def pencil_source(pos, direction) -> abi.Source:
    s = abi.Source()
    s.kind = abi.SRC_PENCIL
    for i in range(3):
        s.pos[i] = float(pos[i]); s.dir[i] = float(direction[i])
    return s


def uniform_source(p1, p2, p3, direction) -> abi.Source:
    s = abi.Source()
    s.kind = abi.SRC_UNIFORM
    for i in range(3):
        s.p1[i] = float(p1[i]); s.p2[i] = float(p2[i]); s.p3[i] = float(p3[i])
        s.dir[i] = float(direction[i])
    return s


def _src(kind, pos=(0.0, 0.0, 0.0), direction=(0.0, 0.0, 0.0)) -> abi.Source:
    s = abi.Source()
    s.kind = kind
    for i in range(3):
        s.pos[i] = float(pos[i]); s.dir[i] = float(direction[i])
    return s


def circular_source(pos, direction, radius) -> abi.Source:
    """circular (photon.f90:214-308): a uniform disc of `radius` centred on pos, facing direction."""
    s = _src(abi.SRC_CIRCULAR, pos, direction)
    s.radius = float(radius)
    return s


def focus_source(pos, rotation, focal_length=1.0, focus_type="gaussian", beam_size=0.5) -> abi.Source:
    """focus (photon.f90:361-563): a beam focused at focal_length, rotated onto `rotation`."""
    s = _src(abi.SRC_FOCUS, pos)
    s.beam = abi.BEAM_KINDS[focus_type]
    s.focal_length, s.beam_size = float(focal_length), float(beam_size)
    for i in range(3):
        s.rotation[i] = float(rotation[i])
    return s


def annulus_source(pos, rotation, focal_length=1.0, annulus_type="gaussian", rlo=0.5, rhi=0.6,
                   sigma=0.04) -> abi.Source:
    """annulus (photon.f90:850-1043): an annular beam (tophat, besselAnnulus or gaussian)."""
    s = _src(abi.SRC_ANNULUS, pos)
    s.beam = abi.BEAM_KINDS[annulus_type]
    s.focal_length, s.rlo, s.rhi, s.sigma = float(focal_length), float(rlo), float(rhi), float(sigma)
    for i in range(3):
        s.rotation[i] = float(rotation[i])
    return s


def slm_source(pos, direction, spectrum=None) -> abi.Source:
    """slm (photon.f90:159-212): (x, y) sampled from a 2-D spectrum (an image)."""
    s = _src(abi.SRC_SLM, pos, direction)
    if spectrum is not None:
        attach_spectrum(s, spectrum)
    return s


def dslit_source() -> abi.Source:
    """dslit (photon.f90:712-780): double-slit diffraction source."""
    return _src(abi.SRC_DSLIT)


def aperture_source() -> abi.Source:
    """aperture (photon.f90:782-848): square-aperture diffraction source."""
    return _src(abi.SRC_APERTURE)


def spectrum_constant(wavelength=500.0) -> abi.Spectrum:
    sp = abi.Spectrum()
    sp.kind, sp.wavelength = abi.SPEC_CONSTANT, float(wavelength)
    return sp


def spectrum_1d(array) -> abi.Spectrum:
    """piecewise1D (piecewise.f90:140-168) of an (n, 2) array: column 0 wavelengths, column 1
    the flux (the reference loads it in single precision, parse_spectrum.f90:61-64)."""
    a = np.asfortranarray(np.asarray(array, dtype=np.float64))
    assert a.ndim == 2 and a.shape[1] == 2
    sp = abi.Spectrum()
    sp.kind, sp.n = abi.SPEC_1D, a.shape[0]
    sp.array = a.ctypes.data_as(C.POINTER(C.c_double))
    sp._keep = a
    return sp


def spectrum_2d(image, cell_width, cell_height) -> abi.Spectrum:
    """piecewise2D (piecewise.f90:190-236) of image(width, height) (Fortran order: the first
    index is x)."""
    img = np.asfortranarray(np.asarray(image, dtype=np.float64))
    sp = abi.Spectrum()
    sp.kind = abi.SPEC_2D
    sp.width, sp.height = img.shape
    sp.image = img.ctypes.data_as(C.POINTER(C.c_double))
    sp.cell_width, sp.cell_height = float(cell_width), float(cell_height)
    sp._keep = img
    return sp


def attach_spectrum(source: abi.Source, spectrum: abi.Spectrum) -> abi.Source:
    """Point source.spectrum at `spectrum` (kept alive by the source object)."""
    source.spectrum = C.pointer(spectrum)
    source._spectrum = spectrum
    return source


DIRECTIONS = {"x": (1.0, 0.0, 0.0), "-x": (-1.0, 0.0, 0.0), "y": (0.0, 1.0, 0.0),
              "-y": (0.0, -1.0, 0.0), "z": (0.0, 0.0, 1.0), "-z": (0.0, 0.0, -1.0)}


# ------------------------------------------------------------------ detectors -----
def _norm(v):
    ln = math.sqrt(v[0] ** 2 + v[1] ** 2 + v[2] ** 2)
    return (v[0] / ln, v[1] / ln, v[2] / ln)


def circle_dect(pos, direction, layer, radius, nbins) -> abi.Detector:
    """init_circle_dect, detectors.f90:122-145 (direction normalised by the parser)."""
    d = abi.Detector()
    d.kind = abi.DET_CIRCLE
    d.nbins = int(nbins) + 1
    d.layer = int(layer)
    for i in range(3):
        d.pos[i] = float(pos[i]); d.dir[i] = float(direction[i])
    d.radius = float(radius)
    d.bin_wid = 1.0 if nbins == 0 else float(radius) / float(nbins)
    return d


def annulus_dect(pos, direction, layer, r1, r2, nbins) -> abi.Detector:
    """init_annulus_dect, detectors.f90:166-200."""
    d = abi.Detector()
    d.kind = abi.DET_ANNULUS
    d.nbins = int(nbins) + 1
    d.layer = int(layer)
    for i in range(3):
        d.pos[i] = float(pos[i]); d.dir[i] = float(direction[i])
    d.r1, d.r2 = float(r1), float(r2)
    d.bin_wid = 1.0 if nbins == 0 else (float(r2) - float(r1)) / float(nbins)
    return d


def camera(p1, p2, p3, layer, nbins, maxval) -> abi.Detector:
    """init_camera, detectors.f90:401-445: e1=p2-p1, e2=p3-p1, n=normalise(e2 x e1)."""
    d = abi.Detector()
    d.kind = abi.DET_CAMERA
    e1 = [float(p2[i]) - float(p1[i]) for i in range(3)]
    e2 = [float(p3[i]) - float(p1[i]) for i in range(3)]
    n = (e2[1] * e1[2] - e2[2] * e1[1], -e2[0] * e1[2] + e2[2] * e1[0], e2[0] * e1[1] - e2[1] * e1[0])
    ln = math.sqrt(n[0] * n[0] + n[1] * n[1] + n[2] * n[2])
    n = (n[0] / ln, n[1] / ln, n[2] / ln)
    for i in range(3):
        d.pos[i] = float(p1[i]); d.e1[i] = e1[i]; d.e2[i] = e2[i]; d.dir[i] = n[i]
    d.width = math.sqrt(e1[0] * e1[0] + e1[1] * e1[1] + e1[2] * e1[2])
    d.height = math.sqrt(e2[0] * e2[0] + e2[1] * e2[1] + e2[2] * e2[2])
    d.nbins = int(nbins) + 1
    d.layer = int(layer)
    if nbins == 0:
        d.bin_wid = d.bin_wid_y = 1.0
    else:
        d.bin_wid = float(maxval) / float(d.nbins)
        d.bin_wid_y = float(maxval) / float(d.nbins)
    return d


def fibre_dect(pos, direction, layer, nbins, focal1=1.0, focal2=1.0, f1_aperture=1.0, f2_aperture=1.0,
               front_offset=0.0, back_offset=None, front_to_pin=None, pin_to_back=None, pin_aperture=None,
               accept_angle=90.0, core_diameter=0.01) -> abi.Detector:
    """init_fibre_dect, detectors.f90:246-329, with the parser's defaults
    (parse_detectors.f90:262-280): back_offset and pin_to_back default to focal2,
    front_to_pin to focal1, pin_aperture to max(f1_aperture, f2_aperture)."""
    d = abi.Detector()
    d.kind = abi.DET_FIBRE
    d.nbins = int(nbins) + 1
    d.layer = int(layer)
    direction = _norm(direction)
    for i in range(3):
        d.pos[i] = float(pos[i]); d.dir[i] = float(direction[i])
    f = [focal1, focal2, f1_aperture, f2_aperture, front_offset,
         focal2 if back_offset is None else back_offset,
         focal1 if front_to_pin is None else front_to_pin,
         focal2 if pin_to_back is None else pin_to_back,
         max(f1_aperture, f2_aperture) if pin_aperture is None else pin_aperture,
         accept_angle, core_diameter]
    for i, v in enumerate(f):
        d.fibre[i] = float(v)
    d.bin_wid = 1.0 if nbins == 0 else float(core_diameter) / 2.0 / float(nbins)
    return d


def det_sizes(dets) -> List[int]:
    return [d.nbins * d.nbins if d.kind == abi.DET_CAMERA else d.nbins for d in dets]


def detector_array(dets):
    arr = (abi.Detector * max(1, len(dets)))()
    for i, d in enumerate(dets):
        arr[i] = d
    return arr
