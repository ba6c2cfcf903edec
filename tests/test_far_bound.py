"""The far-field march's error bound (far.h), tested instead of asserted.

The march's certificate (far.h header) needs every computed top-level SDF value within
fm_err of the true distance, and the rounding of each step p + d*dir within fm_step. The host
sets both from the scene's scale (smcrt.hip scene creation, "far-field march" block):
    ext     = xmax + ymax + zmax + 1
    scale   = max over tops of |t14| + |t24| + |t34| + sum |param[0..7]|
    fm_err  = 2^-44 (scale + ext),   fm_step = 2^-48 (scale + ext).
Here every far-eligible primitive kind (sphere, box, torus, segment, capsule under
translation-only transforms) is evaluated by the CPU restatement, whose fp64 operations are
the device's bit for bit (the GPU parity tests), at adversarial points: on and within
1e-15..1e-6 of the surfaces, on box faces, edges and corners, at the grid's corners and all
over the grid. The true value is the same formula in 60-digit decimal arithmetic on the
exact binary inputs (the translation applied exactly). The test asserts
|computed - true| <= fm_err / 2 (a factor-2 margin on the certificate's assumption) for the
scales of M2 (40 spheres + box, the far march's workload) and M4 (capsules + box, 0.16 cm
grid), plus a sphere, torus, segment and capsule at each scale, sdfs.f90:494-648.
"""
import decimal
from decimal import Decimal as D

import numpy as np
import pytest

import bench
from oracle import pyoracle as O
from rsmcrt_amd import abi, scene
from rsmcrt_amd.scene import Scene, invert, mono, translate

decimal.getcontext().prec = 60
FAR_KINDS = (abi.SDF_SPHERE, abi.SDF_BOX, abi.SDF_TORUS, abi.SDF_SEGMENT, abi.SDF_CAPSULE)


def node_scale(sc, i):
    """The operand magnitude a top contributes to the bound (smcrt.hip far_ok): a primitive's
    translation and parameters; a model's largest child, and its smooth-union k."""
    nd = sc.nodes[i]
    if nd.kind == abi.SDF_MODEL:
        m = nd.k if nd.op == abi.OP_SMOOTH_UNION else 0.0
        return max([m] + [node_scale(sc, nd.first_child + c) for c in range(nd.n_children)])
    m = abs(nd.transform[3]) + abs(nd.transform[7]) + abs(nd.transform[11])
    return m + sum(abs(nd.param[r]) for r in range(8))


def fm_bounds(sc, g):
    """fm_err, fm_step as the host computes them (smcrt.hip, far-field block)."""
    ext = g.xmax + g.ymax + g.zmax + 1.0
    scale = max(node_scale(sc, i) for i in sc.top)
    return np.ldexp(scale + ext, -44), np.ldexp(scale + ext, -48)


def _len(*c):
    return sum(x * x for x in c).sqrt()


def exact_sdf(nd, p):
    """The primitive's formula (sdfs.f90:494-648, as the restatement writes it) in decimal
    arithmetic on the exact point p - c of a translation-only transform."""
    t = nd.transform
    assert [t[i] for i in (0, 1, 2, 4, 5, 6, 8, 9, 10)] == [1.0, 0.0, 0.0, 0.0, 1.0, 0.0, 0.0, 0.0, 1.0]
    x, y, z = (D(float(p[0])) + D(t[3]), D(float(p[1])) + D(t[7]), D(float(p[2])) + D(t[11]))
    P = [D(v) for v in nd.param]
    k = nd.kind
    if k == abi.SDF_SPHERE:
        return _len(x, y, z) - P[0]
    if k == abi.SDF_BOX:
        q = (abs(x) - P[0], abs(y) - P[1], abs(z) - P[2])
        return _len(*(max(v, D(0)) for v in q)) + min(max(q), D(0))
    if k == abi.SDF_TORUS:
        return _len(_len(x, z) - P[0], y) - P[1]
    a, b = P[0:3], P[3:6]
    pa = (x - a[0], y - a[1], z - a[2])
    ba = (b[0] - a[0], b[1] - a[1], b[2] - a[2])
    h = sum(u * v for u, v in zip(pa, ba)) / sum(v * v for v in ba)
    h = min(max(h, D(0)), D(1))
    r = D(0.1) if k == abi.SDF_SEGMENT else P[6]  # (the segment's literal 0.1 as a double, sdfs.f90:624)
    return _len(*(u - v * h for u, v in zip(pa, ba))) - r


def adversarial_points(nd, g, rng, n=60):
    """Points on and near the primitive's surface (offsets 0 and +-1e-15 .. 1e-6), on box
    faces, edges and corners, at the grid's corners and uniformly over the grid."""
    t = nd.transform
    c = np.array([-t[3], -t[7], -t[11]])
    P = np.array(list(nd.param))
    offs = np.array([0.0, 1e-15, -1e-15, 1e-12, -1e-12, 1e-9, -1e-9, 1e-6, -1e-6])
    pts = []
    u = rng.normal(size=(n, 3))
    u /= np.linalg.norm(u, axis=1)[:, None]
    k = nd.kind
    for i in range(n):
        o = offs[i % len(offs)]
        if k == abi.SDF_SPHERE:
            pts.append(c + u[i] * (P[0] + o))
        elif k == abi.SDF_BOX:
            b = P[:3]
            q = rng.uniform(-b, b)
            ax = i % 3
            q[ax] = np.sign(u[i][ax]) * (b[ax] + o)
            if i % 4 == 1:  # an edge
                q[(ax + 1) % 3] = np.sign(u[i][(ax + 1) % 3]) * b[(ax + 1) % 3]
            if i % 4 == 2:  # a corner
                q = np.sign(u[i]) * (b + o)
            pts.append(c + q)
        elif k == abi.SDF_TORUS:
            ang = rng.uniform(0.0, 2.0 * np.pi)
            ring = np.array([np.cos(ang) * P[0], 0.0, np.sin(ang) * P[0]])
            pts.append(c + ring + u[i] * (P[1] + o))
        else:
            a, b = P[0:3], P[3:6]
            r = 0.1 if k == abi.SDF_SEGMENT else P[6]
            h = rng.uniform(-0.2, 1.2)
            ax = b - a
            perp = np.cross(ax, u[i])
            perp /= np.linalg.norm(perp)
            base = a + np.clip(h, 0.0, 1.0) * ax
            dirn = perp if 0.0 <= h <= 1.0 else u[i]
            pts.append(c + base + dirn * (r + o))
    m = np.array([g.xmax, g.ymax, g.zmax])
    corners = np.array([[sx, sy, sz] for sx in (-1, 1) for sy in (-1, 1) for sz in (-1, 1)]) * m
    pts.extend(corners)
    pts.extend(rng.uniform(-1.05 * m, 1.05 * m, size=(n, 3)))
    return np.array(pts)


def extra_tops(scale):
    """A sphere, a torus, a segment and a capsule at the scene's scale (far-eligible kinds the
    workload may not use)."""
    o = mono(1.0, 0.1, 0.9, 1.0)
    return [scene.sphere(0.3 * scale, o, 1, transform=invert(translate((-0.2 * scale, 0.1 * scale, 0.05)))),
            scene.torus(0.4 * scale, 0.1 * scale, o, 1, transform=invert(translate((0.1 * scale, -0.2 * scale, 0.3)))),
            scene.segment((-0.3 * scale, 0.0, 0.1 * scale), (0.2 * scale, 0.25 * scale, -0.1 * scale), o, 1,
                          transform=invert(translate((0.05, 0.0, -0.1 * scale)))),
            scene.capsule((0.1 * scale, -0.3 * scale, 0.0), (-0.2 * scale, 0.1 * scale, 0.2 * scale), 0.05 * scale, o, 1,
                          transform=invert(translate((-0.1 * scale, 0.05, 0.0))))]


@pytest.mark.parametrize("workload", ["m2", "m4"])
def test_far_field_error_bound(workload):
    sc, g, _, _, _, _ = bench.workload(workload, 32)
    scale = max(g.xmax, g.ymax, g.zmax)
    tops = [s for s in sc.sdfs]
    if workload == "m4":
        tops = tops[:48] + tops[-1:]  # (the box and a subset of the 512 capsules)
    full = Scene(tops + extra_tops(scale))
    fm_err, fm_step = fm_bounds(full, g)
    rng = np.random.Generator(np.random.Philox(7))
    worst = 0.0
    kinds = set()
    for which, i in enumerate(full.top):
        nd = full.nodes[i]
        assert nd.kind in FAR_KINDS
        kinds.add(nd.kind)
        pts = adversarial_points(nd, g, rng)
        got = O.sdf_eval(full, pts, which)
        for p, v in zip(pts, got):
            err = abs(D(float(v)) - exact_sdf(nd, p))
            worst = max(worst, float(err))
            assert err <= D(fm_err) / 2, (workload, which, nd.kind, p.tolist(), float(err), fm_err)
    assert kinds == set(FAR_KINDS)
    # the step's rounding: |RN(p + d dir) - (p + d dir)| <= ulp(|p| + d)/2, with |p|, d below
    # the grid's extent plus the scale
    assert np.spacing(g.xmax + g.ymax + g.zmax + scale) <= fm_step / 2
    # the bound's actual slack (measured: the worst error is ~1e-3 of fm_err at both scales)
    assert worst <= fm_err / 64, (worst, fm_err)


def exact_node(sc, i, p):
    """A far-eligible top in decimal arithmetic: a primitive (exact_sdf) or a model folded left
    to right with union / smooth union / subtraction / intersection (sdfModifiers.f90:428-491)."""
    nd = sc.nodes[i]
    if nd.kind != abi.SDF_MODEL:
        return exact_sdf(nd, p)
    acc = None
    k = D(nd.k)
    for c in range(nd.n_children):
        v = exact_node(sc, nd.first_child + c, p)
        if acc is None:
            acc = v
        elif nd.op == abi.OP_UNION:
            acc = min(acc, v)
        elif nd.op == abi.OP_SMOOTH_UNION:
            h = max(k - abs(acc - v), D(0)) / k
            acc = min(acc, v) - h * h * h * k * (D(1) / D(6))
        elif nd.op == abi.OP_SUBTRACTION:
            acc = max(-acc, v)
        else:
            acc = max(acc, v)
    return acc


@pytest.mark.parametrize("scale_of", ["m2", "m4"])
def test_far_field_error_bound_models(scale_of):
    """Round 4: a model of far-eligible primitives folded with union, smooth union,
    subtraction or intersection (two levels deep too) qualifies for the far-field march as a
    non-near top (smcrt.hip far_ok). Its computed value must be within the same bound:
    evaluated by the restatement at adversarial points of every child, against the fold in
    60-digit decimal arithmetic."""
    from rsmcrt_amd.scene import box, capsule, model, sphere, torus
    _, g, _, _, _, _ = bench.workload(scale_of, 32)
    s = max(g.xmax, g.ymax, g.zmax)
    o = mono(1.0, 0.1, 0.9, 1.0)
    t = lambda c: invert(translate(tuple(v * s for v in c)))  # noqa: E731
    kids = lambda: [sphere(0.2 * s, o, 1, transform=t((0.1, 0.0, 0.05))),  # noqa: E731
                    box((0.15 * s, 0.1 * s, 0.2 * s), o, 1, transform=t((0.2, -0.05, 0.0))),
                    capsule((0.0, -0.1 * s, 0.0), (0.2 * s, 0.1 * s, 0.1 * s), 0.05 * s, o, 1,
                            transform=t((-0.1, 0.1, 0.0)))]
    tops = [model(kids(), abi.OP_UNION), model(kids(), abi.OP_SMOOTH_UNION, 0.05 * s),
            model(kids(), abi.OP_SUBTRACTION), model(kids(), abi.OP_INTERSECTION),
            model([model(kids()[:2], abi.OP_SMOOTH_UNION, 0.03 * s),
                   torus(0.2 * s, 0.05 * s, o, 1, transform=t((0.0, 0.2, -0.1)))], abi.OP_UNION)]
    full = Scene(tops)
    fm_err, _ = fm_bounds(full, g)
    rng = np.random.Generator(np.random.Philox(11))
    worst = 0.0

    def prims(i):
        nd = full.nodes[i]
        if nd.kind != abi.SDF_MODEL:
            return [nd]
        return [q for c in range(nd.n_children) for q in prims(nd.first_child + c)]

    for which, i in enumerate(full.top):
        pts = np.concatenate([adversarial_points(nd, g, rng, n=27) for nd in prims(i)])
        got = O.sdf_eval(full, pts, which)
        for p, v in zip(pts, got):
            err = abs(D(float(v)) - exact_node(full, i, p))
            worst = max(worst, float(err))
            assert err <= D(fm_err) / 2, (scale_of, which, p.tolist(), float(err), fm_err)
    assert worst <= fm_err / 64, (worst, fm_err)
