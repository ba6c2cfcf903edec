"""ORACLE — test infrastructure only (see smcrt_oracle.c header).

Pure-Python restatement of the escape-function driver of the reference
(src/kernelsMod.f90:85-1460, src/grid.f90:50-117, src/interpolate.f90,
src/sdfs/sdfHelpers.f90:85-140, src/parse/parse.f90:188-340), for small symmetry grids.
The photon transport of each launch cell is the C restatement (pyoracle.run), called once
per cell exactly as the reference calls run_MCRT once per cell. Imported only by tests/.

Arrays use the reference's index order: escape_sym[d, m, n, o] (0-based here), values fp32
(iarray.f90:18), arithmetic in Python floats (IEEE fp64, libm sin/cos/atan2/sqrt).
"""
from __future__ import annotations

import math

import numpy as np

PI = 4.0 * math.atan(1.0)  # constants.f90
TWOPI = 2.0 * PI
CYL = ("noneRotational", "360rotational")


# ---- sdfHelpers / vector_class ------------------------------------------------------
def _identity():
    return [[1.0 if i == j else 0.0 for j in range(4)] for i in range(4)]


def _matmul(A, B):  # Fortran matmul, k ascending
    C = [[0.0] * 4 for _ in range(4)]
    for i in range(4):
        for j in range(4):
            s = 0.0
            for k in range(4):
                s = s + A[i][k] * B[k][j]
            C[i][j] = s
    return C


def _magnitude(v):  # vector_class.f90:392-402
    t = math.sqrt(v[0] * v[0] + v[1] * v[1] + v[2] * v[2])
    return (v[0] / t, v[1] / t, v[2] / t)


def rotation_align(a, b):
    """sdfHelpers.f90:114-140: I + [v]x + [v]x^2 / (1 + a.b), v = a x b; m[r][c] = t(r+1, c+1)."""
    v = (a[1] * b[2] - a[2] * b[1], -a[0] * b[2] + a[2] * b[0], a[0] * b[1] - a[1] * b[0])
    c = a[0] * b[0] + a[1] * b[1] + a[2] * b[2]
    k = 1.0 / (1.0 + c) if (1.0 + c) != 0.0 else math.inf
    vx = [[0.0] * 4 for _ in range(4)]
    vx[1][0] = -1.0 * v[2]; vx[2][0] = v[1]
    vx[0][1] = v[2]; vx[2][1] = -1.0 * v[0]
    vx[0][2] = -1.0 * v[1]; vx[1][2] = v[0]
    vx2 = _matmul(vx, vx)
    I = _identity()
    return [[(I[i][j] + vx[i][j]) + vx2[i][j] * k for j in range(4)] for i in range(4)]


def rotmat(axis, angle):
    """sdfHelpers.f90:85-112 (angle in degrees)."""
    a = _magnitude(axis)
    r = angle * PI / 180.0
    s, c = math.sin(r), math.cos(r)
    oc = 1.0 - c
    m = [[0.0] * 4 for _ in range(4)]
    m[0][0] = oc * a[0] * a[0] + c; m[1][0] = oc * a[0] * a[1] - a[2] * s; m[2][0] = oc * a[2] * a[0] + a[1] * s
    m[0][1] = oc * a[0] * a[1] + a[2] * s; m[1][1] = oc * a[1] * a[1] + c; m[2][1] = oc * a[1] * a[2] - a[0] * s
    m[0][2] = oc * a[2] * a[0] - a[1] * s; m[1][2] = oc * a[1] * a[2] + a[0] * s; m[2][2] = oc * a[2] * a[2] + c
    m[3][3] = 1.0
    return m


def vdotm(p, b):  # vec_dot_mat, vector_class.f90:292-304
    return (b[0][0] * p[0] + b[1][0] * p[1] + b[2][0] * p[2] + b[3][0] * 1.0,
            b[0][1] * p[0] + b[1][1] * p[1] + b[2][1] * p[2] + b[3][1] * 1.0,
            b[0][2] * p[0] + b[1][2] * p[1] + b[2][2] * p[2] + b[3][2] * 1.0)


# ---- the symmetry grid ----------------------------------------------------------------
class Sym:
    def __init__(self, symmetry, n, maxv, pos, direction, rotation):
        self.kind = symmetry
        self.n = tuple(int(x) for x in n)
        self.max = (float(maxv[0]), TWOPI if symmetry in CYL else float(maxv[1]), float(maxv[2]))
        self.pos = tuple(float(x) for x in pos)
        self.dir = _magnitude(direction)  # parse.f90:296
        z = (0.0, 0.0, 1.0)
        self.off = rotation_align(z, self.dir)  # kernelsMod.f90:190-194
        self.on = rotation_align(self.dir, z)
        self.off_z = rotmat(z, -rotation)
        self.on_z = rotmat(z, rotation)

    @property
    def cyl(self):
        return self.kind in CYL


def cart_c(i, n, mx):
    return ((((float(i) - 0.5) / n) * 2.0 * mx) - mx)


def rad_c(i, n, rmax):
    return ((float(i) - 0.5) / n) * rmax


def voxel_cart(S, p):  # grid.f90:50-78
    r = [math.floor(S.n[k] * (p[k] + S.max[k]) / (2.0 * S.max[k])) + 1 for k in range(3)]
    return [x if 1 <= x <= S.n[k] else -1 for k, x in enumerate(r)]


def polar(p):
    rad = math.sqrt(p[0] * p[0] + p[1] * p[1])
    if rad == 0:
        return rad, 0.0
    theta = math.atan2(p[1], p[0])
    if theta < 0.0:
        theta = theta + 2 * math.atan2(0.0, -1.0)
    return rad, theta


def voxel_cyl(S, p):  # grid.f90:80-117
    rad, theta = polar(p)
    r = [math.floor(S.n[0] * (rad / S.max[0])) + 1, math.floor(S.n[1] * ((theta) / S.max[1])) + 1,
         math.floor(S.n[2] * (p[2] + S.max[2]) / (2.0 * S.max[2])) + 1]
    return [x if 1 <= x <= S.n[k] else -1 for k, x in enumerate(r)]


def launch_cells(S):
    """(m, n, o) in the loop order of escape_Function's symmetry branches (:177-453)."""
    n0, n1, n2 = S.n
    if S.kind in ("none", "noneRotational"):
        return [(m, n, o) for m in range(1, n0 + 1) for n in range(1, n1 + 1) for o in range(1, n2 + 1)]
    if S.kind == "prism":
        idx = voxel_cart(S, (0.0, 0.0, 0.0))
        return [(m, n, idx[2]) for m in range(1, n0 + 1) for n in range(1, n1 + 1)]
    if S.kind == "flipped":
        return [(m, n, o) for m in range(1, n0 + 1) for n in range(1, n1 + 1) for o in range(1, min(n2 // 2 + 1, n2) + 1)]
    if S.kind == "uniformSlab":
        idx = voxel_cart(S, (0.0, 0.0, 0.0))
        return [(idx[0], idx[1], o) for o in range(1, n2 + 1)]
    if S.kind == "360rotational":
        return [(m, 1, o) for m in range(1, n0 + 1) for o in range(1, n2 + 1)]
    raise ValueError(S.kind)


def cell_position(S, m, n, o):
    """cart_calc_escape_sym :566-580 / cyl_calc_escape_sym :1004-1021."""
    if S.cyl:
        rad = rad_c(m, S.n[0], S.max[0])
        theta = ((float(n) - 0.5) / S.n[1]) * S.max[1]
        p = (rad * math.cos(theta), rad * math.sin(theta), cart_c(o, S.n[2], S.max[2]))
    else:
        p = (cart_c(m, S.n[0], S.max[0]), cart_c(n, S.n[1], S.max[1]), cart_c(o, S.n[2], S.max[2]))
    p = vdotm(p, S.off_z)
    p = vdotm(p, S.off)
    return (p[0] + S.pos[0], p[1] + S.pos[1], p[2] + S.pos[2])


# ---- interpolate.f90 --------------------------------------------------------------------
def lin1(x0, x1, v0, v1, p):
    xd = (p - x0) / (x1 - x0)
    return v0 * (1 - xd) + v1 * xd


def bilin(a, b, v, pa, pb):
    xd = (pa - a[0]) / (a[1] - a[0])
    yd = (pb - b[0]) / (b[1] - b[0])
    c0 = v[0][0] * (1 - xd) + v[1][0] * xd
    c1 = v[0][1] * (1 - xd) + v[1][1] * xd
    return c0 * (1 - yd) + c1 * yd


def trilin(x, y, z, v, px, py, pz):
    xd = (px - x[0]) / (x[1] - x[0])
    yd = (py - y[0]) / (y[1] - y[0])
    zd = (pz - z[0]) / (z[1] - z[0])
    c00 = v[0][0][0] * (1 - xd) + v[1][0][0] * xd
    c01 = v[0][0][1] * (1 - xd) + v[1][0][1] * xd
    c10 = v[0][1][0] * (1 - xd) + v[1][1][0] * xd
    c11 = v[0][1][1] * (1 - xd) + v[1][1][1] * xd
    c0 = c00 * (1 - yd) + c10 * yd
    c1 = c01 * (1 - yd) + c11 * yd
    return c0 * (1 - zd) + c1 * zd


def cyl_bilin(r, t, v, pr, pt):
    area = 0.5 * (t[1] - t[0]) * (r[1] * r[1] - r[0] * r[0])
    a00 = 0.5 * (t[1] - pt) * (r[1] * r[1] - pr * pr)
    a01 = 0.5 * (pt - t[0]) * (r[1] * r[1] - pr * pr)
    a10 = 0.5 * (t[1] - pt) * (pr * pr - r[0] * r[0])
    a11 = 0.5 * (pt - t[0]) * (pr * pr - r[0] * r[0])
    return (a00 / area) * v[0][0] + (a01 / area) * v[0][1] + (a10 / area) * v[1][0] + (a11 / area) * v[1][1]


def cyl_trilin(r, t, z, v, pr, pt, pz):
    volume = 0.5 * (t[1] - t[0]) * (r[1] * r[1] - r[0] * r[0]) * (z[1] - z[0])
    a00 = 0.5 * (t[1] - pt) * (r[1] * r[1] - pr * pr)
    a01 = 0.5 * (pt - t[0]) * (r[1] * r[1] - pr * pr)
    a10 = 0.5 * (t[1] - pt) * (pr * pr - r[0] * r[0])
    a11 = 0.5 * (pt - t[0]) * (pr * pr - r[0] * r[0])
    w = [a00 * (z[1] - pz) / volume, a00 * (pz - z[0]) / volume, a01 * (z[1] - pz) / volume,
         a01 * (pz - z[0]) / volume, a10 * (z[1] - pz) / volume, a10 * (pz - z[0]) / volume,
         a11 * (z[1] - pz) / volume, a11 * (pz - z[0]) / volume]
    c = [v[0][0][0], v[0][0][1], v[0][1][0], v[0][1][1], v[1][0][0], v[1][0][1], v[1][1][0], v[1][1][1]]
    s = w[0] * c[0]
    for i in range(1, 8):
        s = s + w[i] * c[i]
    return s


# ---- cart_map_escape_sym / cyl_map_escape_sym ---------------------------------------------
def _map_cart(S, E, p, nd):
    indx = voxel_cart(S, p)
    if -1 in indx:
        return [-1.0] * nd
    cx, cy, cz = cart_c(indx[0], S.n[0], S.max[0]), cart_c(indx[1], S.n[1], S.max[1]), cart_c(indx[2], S.n[2], S.max[2])
    xi = [indx[0] - 1, indx[0]] if cx > p[0] else [indx[0], indx[0] + 1]
    yi = [indx[1] - 1, indx[1]] if cy > p[1] else [indx[1], indx[1] + 1]
    zi = [indx[2] - 1, indx[2]] if cz > p[2] else [indx[2], indx[2] + 1]
    inx = not (xi[0] < 1 or xi[1] > S.n[0])
    iny = not (yi[0] < 1 or yi[1] > S.n[1])
    inz = not (zi[0] < 1 or zi[1] > S.n[2])
    X = [cart_c(i, S.n[0], S.max[0]) for i in xi]
    Y = [cart_c(i, S.n[1], S.max[1]) for i in yi]
    Z = [cart_c(i, S.n[2], S.max[2]) for i in zi]
    ii, jj, kk = (0 if xi[0] >= 1 else 1), (0 if yi[0] >= 1 else 1), (0 if zi[0] >= 1 else 1)
    out = []
    for d in range(nd):
        e = lambda m, n, o: float(E[d, m - 1, n - 1, o - 1])
        if inx and iny and inz:
            v = [[[e(xi[i], yi[j], zi[k]) for k in range(2)] for j in range(2)] for i in range(2)]
            r = trilin(X, Y, Z, v, p[0], p[1], p[2])
        elif inx and iny and not inz:
            r = bilin(X, Y, [[e(xi[i], yi[j], zi[kk]) for j in range(2)] for i in range(2)], p[0], p[1])
        elif inx and inz and not iny:
            r = bilin(X, Z, [[e(xi[i], yi[jj], zi[k]) for k in range(2)] for i in range(2)], p[0], p[2])
        elif iny and inz and not inx:
            r = bilin(Y, Z, [[e(xi[ii], yi[j], zi[k]) for k in range(2)] for j in range(2)], p[1], p[2])
        elif inx and not iny and not inz:
            r = lin1(X[0], X[1], e(xi[0], yi[jj], zi[kk]), e(xi[1], yi[jj], zi[kk]), p[0])
        elif iny and not inx and not inz:
            r = lin1(Y[0], Y[1], e(xi[ii], yi[0], zi[kk]), e(xi[ii], yi[1], zi[kk]), p[1])
        elif inz and not inx and not iny:
            r = lin1(Z[0], Z[1], e(xi[ii], yi[jj], zi[0]), e(xi[ii], yi[jj], zi[1]), p[2])
        else:
            r = e(indx[0], indx[1], indx[2])
        out.append(r)
    return out


def _map_cyl(S, E, p, nd):
    rad, theta = polar(p)
    indx = voxel_cyl(S, p)
    if -1 in indx:
        return [-1.0] * nd
    nr, nt, nz = S.n
    cr = rad_c(indx[0], nr, S.max[0])
    ct = ((float(indx[1]) - 0.5) / nt) * S.max[1]
    cz = cart_c(indx[2], nz, S.max[2])
    ri = [indx[0] - 1, indx[0]] if cr > rad else [indx[0], indx[0] + 1]
    ti = [indx[1] - 1, indx[1]] if ct > theta else [indx[1], indx[1] + 1]
    zi = [indx[2] - 1, indx[2]] if cz > p[2] else [indx[2], indx[2] + 1]
    tlo = ((float(ti[0]) - 0.5) / nt) * S.max[1]
    thi = ((float(ti[1]) - 0.5) / nt) * S.max[1]
    if ti[0] < 1:
        ti[0] = nt
    if ti[1] > nt:
        ti[1] = 1
    T = [tlo, thi]
    Z = [cart_c(zi[0], nz, S.max[2]), cart_c(zi[1], nz, S.max[2])]
    out = []
    for d in range(nd):
        e = lambda m, n, o: float(E[d, m - 1, n - 1, o - 1])

        def avg(o):
            s = 0.0
            for i in range(1, nt + 1):
                s = s + e(1, i, o)
            return s / nt

        if ri[0] < 1:  # :1215-1294
            r0 = ((0.5) / nr) * S.max[0]
            at = PI * (r0 * r0) * ((thi - tlo) / TWOPI)
            a1 = (0.5 * r0 * rad * math.sin(thi - theta))
            a2 = (0.5 * r0 * rad * math.sin(theta - tlo))
            a3 = (at - a1 - a2)
            a1, a2, a3 = a1 / at, a2 / at, a3 / at
            if zi[0] < 1:
                r = a1 * e(1, ti[0], 1) + a2 * e(1, ti[1], 1) + a3 * avg(1)
            elif zi[1] > nz:
                r = a1 * e(1, ti[0], nz) + a2 * e(1, ti[1], nz) + a3 * avg(nz)
            else:
                v = [a1 * e(1, ti[0], zi[k]) + a2 * e(1, ti[1], zi[k]) + a3 * avg(zi[k]) for k in range(2)]
                r = lin1(Z[0], Z[1], v[0], v[1], p[2])
        elif ri[1] > nr:  # :1296-1379
            if zi[0] < 1:
                r = lin1(tlo, thi, e(nr, ti[0], 1), e(nr, ti[1], 1), theta)
            elif zi[1] > nz:
                r = lin1(tlo, thi, e(nr, ti[0], nz), e(nr, ti[1], nz), theta)
            else:
                v = [[e(nr, ti[i], zi[k]) for k in range(2)] for i in range(2)]
                r = bilin(T, Z, v, theta, p[2])
        else:
            R = [rad_c(ri[0], nr, S.max[0]), rad_c(ri[1], nr, S.max[0])]
            if zi[0] < 1 or zi[1] > nz:  # :1381-1433
                zo = 1 if zi[0] < 1 else nz
                v = [[e(ri[i], ti[j], zo) for j in range(2)] for i in range(2)]
                r = cyl_bilin(R, T, v, rad, theta)
            else:
                v = [[[e(ri[i], ti[j], zi[k]) for k in range(2)] for j in range(2)] for i in range(2)]
                r = cyl_trilin(R, T, Z, v, rad, theta, p[2])
        out.append(r)
    return out


def map_to_grid(S, grid, E):
    """escape[d, i, j, k] on the fluence grid from escape_sym E[d, m, n, o] (fp32 in, fp32 out)."""
    nd = E.shape[0]
    out = np.zeros((nd, grid.nx, grid.ny, grid.nz), dtype=np.float32)
    for m in range(1, grid.nx + 1):
        for n in range(1, grid.ny + 1):
            for o in range(1, grid.nz + 1):
                y = ((((float(n) - 0.5) / grid.ny) * 2.0 * grid.ymax) - grid.ymax)
                x = ((((float(m) - 0.5) / grid.nx) * 2.0 * grid.xmax) - grid.xmax)
                z = ((((float(o) - 0.5) / grid.nz) * 2.0 * grid.zmax) - grid.zmax)
                p = (x - S.pos[0], y - S.pos[1], z - S.pos[2])
                p = vdotm(p, S.on)
                p = vdotm(p, S.on_z)
                vals = _map_cyl(S, E, p, nd) if S.cyl else _map_cart(S, E, p, nd)
                out[:, m - 1, n - 1, o - 1] = np.array(vals, dtype=np.float64).astype(np.float32)
    return out


def fill_symmetry(S, E):
    """The cells a symmetry copies from the launched ones (:255-262, 348-356, 399-405, 446-449)."""
    n0, n1, n2 = S.n
    if S.kind == "prism":
        o0 = voxel_cart(S, (0.0, 0.0, 0.0))[2]
        for o in range(1, n2 + 1):
            E[:, :, :, o - 1] = E[:, :, :, o0 - 1].copy()
    elif S.kind == "flipped":
        for m in range(n0):
            for n in range(n1):
                for o in range(1, min(n2 // 2 + 1, n2) + 1):
                    E[:, m, n, n2 - o] = E[:, m, n, o - 1]
    elif S.kind == "uniformSlab":
        i0, j0, _ = voxel_cart(S, (0.0, 0.0, 0.0))
        col = E[:, i0 - 1, j0 - 1, :].copy()
        for m in range(n0):
            for n in range(n1):
                E[:, m, n, :] = col
    elif S.kind == "360rotational":
        for n in range(n1):
            E[:, :, n, :] = E[:, :, 0, :].copy()
    return E


def escape_function(scene, grid, dets, S, n_photons, seed=123456789, flags=None, spectrum_source=None):
    """escape_Function end to end on the CPU restatement: (escape_sym, escape, Result of all
    cells' tallies). One pyoracle.run per launch cell, as the reference calls run_MCRT."""
    from oracle import pyoracle as O
    from rsmcrt_amd import abi, scene as scn
    flags = abi.FLAG_PATHLENGTH if flags is None else flags
    nd = len(dets)
    E = np.zeros((nd, *S.n), dtype=np.float32)
    res = None
    for (m, n, o) in launch_cells(S):
        p = cell_position(S, m, n, o)
        ds = [float(O.sdf_eval(scene, [p], which=i)[0]) for i in range(scene.n_top)]
        layer = 0  # maxloc(ds, mask=ds<0): the first maximum of the negative entries
        for i, d in enumerate(ds):
            if d < 0.0 and (layer == 0 or d > ds[layer - 1]):
                layer = i + 1
        if layer == 0:
            continue
        node = scene.nodes[scene.top[layer - 1]]
        if node.mus + node.mua == 0.0:  # getkappa() (init_mono: kappa = mus + mua)
            continue
        src = scn.point_source(p)
        if spectrum_source is not None and getattr(spectrum_source, "_spectrum", None) is not None:
            scn.attach_spectrum(src, spectrum_source._spectrum)
        r = O.run(scene, grid, src, n_photons, seed=seed, flags=flags, dets=dets)
        res = r if res is None else res.merge(r)
        for d in range(nd):
            E[d, m - 1, n - 1, o - 1] = np.float32(float(r.detector(d).sum()) / float(n_photons))
    fill_symmetry(S, E)
    return E, map_to_grid(S, grid, E), res
