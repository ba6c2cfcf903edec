"""Scene builders: the geometry setups of /root/reference/src/setupGeometry.f90.

Each returns the sdfs_array in the reference order (index i+1 is the tauint2 layer).
Parameters come in as keyword arguments instead of the reference's toml dict lookups.
"""
from __future__ import annotations

import math
from typing import Sequence, Tuple

from . import abi
from .scene import (Scene, box, capsule, cylinder, invert, model, mono, rotate_y, sphere, torus,
                    translate, egg, revolution)


def setup_scat_test(tau: float) -> Scene:
    """setupGeometry.f90:409-435: isotropic sphere r=1, mus=tau, in a 2^3 box."""
    opt1 = mono(tau, 0.0, 0.0, 1.0)
    opt2 = mono(0.0, 0.0, 0.0, 1.0)
    return Scene([sphere(1.0, opt1, 1), box((2.0, 2.0, 2.0), opt2, 2)])


def setup_scat_test2(tau: float, hgg: float) -> Scene:
    """setupGeometry.f90:437-464: 200^3 box, mus=tau, mua=1e-17, g=hgg."""
    opt = mono(tau, 1e-17, hgg, 1.0)
    return Scene([box((200.0, 200.0, 200.0), opt, 2)])


def setup_sphere(mus: float, mua: float, hgg: float, n: float, radius: float,
                 position=(0.0, 0.0, 0.0), bounding=(2.0, 2.0, 2.0)) -> Scene:
    """setupGeometry.f90:10-71 (geom_name='sphere')."""
    t = invert(translate(position))
    return Scene([sphere(radius, mono(mus, mua, hgg, n), 1, transform=t),
                  box(bounding, mono(0.0, 0.0, 0.0, 1.0), 2)])


def setup_box(mus: float, mua: float, hgg: float, n: float, box_dims, bounding,
              position=(0.0, 0.0, 0.0)) -> Scene:
    """setupGeometry.f90:73-147 (geom_name='box' / 'test_box')."""
    t = invert(translate(position))
    return Scene([box(box_dims, mono(mus, mua, hgg, n), 1, transform=t),
                  box(bounding, mono(0.0, 0.0, 0.0, 1.0), 2)])


def setup_tran_and_jacques() -> Scene:
    """setupGeometry.f90:335-363 (geom_name='aptran'): n=1.33 sphere r=0.5 in a 2^3 box
    inside an absorbing 2.01^3 box (mua=1e7)."""
    opt1 = mono(0.0, 1e-17, 0.0, 1.0)
    opt2 = mono(0.0, 10000000.0, 0.0, 1.0)
    opt3 = mono(0.0, 1e-17, 0.0, 1.33)
    t = invert(translate((0.0, 0.0, 0.0)))
    return Scene([sphere(0.5, opt3, 1, transform=t),
                  box((2.0, 2.0, 2.0), opt1, 2),
                  box((2.01, 2.01, 2.01), opt2, 3)])


def setup_sphere_scene(spheres: Sequence[Tuple[float, float, float, float]]) -> Scene:
    """setupGeometry.f90:250-294 (geom_name='sphere_scene').

    The reference draws the sphere list from the compiler's RNG before init_rng runs
    (:285-292), so the list is an input here: (radius, x, y, z) per sphere."""
    opt_box = mono(1e-17, 1e-17, 0.0, 1.0)
    opt_sph = mono(0.0, 0.0, 0.9, 1.37)
    sdfs = []
    for i, (r, x, y, z) in enumerate(spheres):
        sdfs.append(sphere(r, opt_sph, i + 1, transform=invert(translate((x, y, z)))))
    sdfs.append(box((2.0, 2.0, 2.0), opt_box, len(spheres) + 1))
    return Scene(sdfs)


def setup_egg(mus, mua, hgg, n, position=(0.0, 0.0, 0.0), bounding=(2.0, 2.0, 2.0), bottom_r=2.0, top_r=1.5,
              sep=1.4, shell=0.02, yolk_r=1.0) -> Scene:
    """setupGeometry.f90:149-248 (geom_name='egg'): yolk sphere (layer 1), albumen and shell as
    revolved Moss eggs (layers 3 and 2, revolution(egg, 0, center=position)), bounding box
    (layer 4). mus/mua/hgg/n are the three-entry optical property lists (numOptProp = 3)."""
    o = [mono(mus[i], mua[i], hgg[i], n[i]) for i in range(3)]
    f = 1.0 - shell
    shell_sdf = revolution(egg(bottom_r, top_r, sep, o[0], 2), 0.0, center=position)
    albumen = revolution(egg(bottom_r * f, top_r * f, sep * f, o[1], 3), 0.0, center=position)
    yolk = sphere(yolk_r, o[2], 1, transform=invert(translate(position)))
    return Scene([yolk, albumen, shell_sdf, box(bounding, mono(0.0, 0.0, 0.0, 1.0), 4)])


def random_sphere_list(num: int, seed: int = 123456789):
    """A fixed-seed stand-in for setup_sphere_scene's draws: radius ~ U(0.001, 0.25),
    centre ~ U(-1+r, 1-r) per axis (the distributions of :286-289)."""
    import numpy as np
    rng = np.random.Generator(np.random.Philox(seed))
    out = []
    for _ in range(num):
        r = 0.001 + rng.random() * (0.25 - 0.001)
        c = [(-1.0 + r) + rng.random() * ((1.0 - r) - (-1.0 + r)) for _ in range(3)]
        out.append((r, c[0], c[1], c[2]))
    return out


def setup_exp(musb, muab, musc, muac, hgga) -> Scene:
    """setupGeometry.f90:365-407 (geom_name='exp'): glass bottle and contents."""
    opt1 = mono(musb, muab, hgga, 1.5)
    opt2 = mono(musc, muac, hgga, 1.3)
    a, b = (-8.0, 0.0, 0.0), (8.0, 0.0, 0.0)
    return Scene([cylinder(a, b, 1.55, opt2, 1),
                  cylinder(a, b, 1.75, opt1, 2),
                  box((20.0, 20.0, 20.0), mono(0.0, 0.0, 0.0, 1.0), 2)])


def setup_omg_sdf() -> Scene:
    """setupGeometry.f90:466-549 (geom_name='omg'): smooth-union model of a torus and
    nine cylinders."""
    opt1 = mono(10.0, 0.16, 0.0, 2.65)
    opt2 = mono(0.0, 0.0, 0.0, 1.0)
    layer = 1
    parts = [torus(0.2, 0.05, opt1, layer, transform=invert(translate((0.0, 0.0, -0.7))))]
    segs = [((-.25, 0.0, -.25), (-.25, 0.0, .25), invert(rotate_y(90.0))),
            ((-.25, 0.0, -.25), (.25, 0.0, .0), None),
            ((.25, 0.0, .0), (-.25, 0.0, .25), None),
            ((-.25, 0.0, .25), (.25, 0.0, .25), None),
            ((-.25, 0.0, .5), (.25, 0.0, .5), None),
            ((-.25, 0.0, .5), (-.25, 0.0, .75), None),
            ((.25, 0.0, .5), (.25, 0.0, .75), None),
            ((.25, 0.0, .75), (0.0, 0.0, .75), None),
            ((0.0, 0.0, .625), (0.0, 0.0, .75), None)]
    for a, b, t in segs:
        parts.append(cylinder(a, b, 0.05, opt1, layer, transform=t))
    return Scene([model(parts, abi.OP_SMOOTH_UNION, 0.09),
                  box((2.0, 2.0, 2.0), opt2, 2)])


def get_vessels(edges, nodes, radii) -> Scene:
    """setupGeometry.f90:552-652 (geom_name='vessels') from the values its reads leave:
    `edges` (E, 2) 1-based node indices, `nodes` (N, 3) and `radii` (N,). Rows of `nodes` the
    reference never reads (its node loop runs to the edge count, :615) are passed as 0.0, the
    value the C++ front end and the Fortran glue give them (the reference leaves them
    undefined). Rescaling as :629-639 in the same operation order, res = 0.001; one capsule
    per edge with the radius of its first node (vessel optics, layer 1), then the dermis box
    .32 x .18 x .26 (layer 2)."""
    import numpy as np
    edges = np.asarray(edges, dtype=np.int64).reshape(-1, 2)
    nodes = np.array(nodes, dtype=np.float64).reshape(-1, 3)
    radii = np.asarray(radii, dtype=np.float64).reshape(-1)
    res = 0.001
    opt_v = mono(94.0, 231.0, 0.9, 1.37)
    opt_d = mono(357.0, 0.458, 0.9, 1.37)
    mx = np.abs(nodes).max(axis=0)
    nodes = nodes / mx - 0.5
    nodes = nodes * mx * res
    sdfs = []
    for e1, e2 in edges:
        a = tuple(float(v) for v in nodes[e1 - 1])
        b = tuple(float(v) for v in nodes[e2 - 1])
        sdfs.append(capsule(a, b, float(radii[e1 - 1] * res), opt_v, 1))
    sdfs.append(box((.32, .18, .26), opt_d, 2))
    return Scene(sdfs)


def synthetic_vessels(n_capsules: int = 512, seed: int = 2025, extent=(0.32, 0.18, 0.26)):
    """Build-defined stand-in for get_vessels (setupGeometry.f90:552-652), whose data files
    res/{edges,nodes,radii}.dat are not in the reference: a random tree of capsules with
    radii 5-30 um in a .32 x .18 x .26 cm box, vessel/dermis optical properties of
    :572-583. Capsules are separate top-level SDFs in layer 1 like the reference."""
    import numpy as np
    rng = np.random.Generator(np.random.Philox(seed))
    opt_v = mono(94.0, 231.0, 0.9, 1.37)
    opt_d = mono(357.0, 0.458, 0.9, 1.37)
    half = np.array(extent) * 0.5 * 0.9
    nodes = [rng.uniform(-half, half)]
    sdfs = []
    for i in range(n_capsules):
        parent = nodes[int(rng.integers(0, len(nodes)))]
        step = rng.normal(size=3)
        step = step / np.linalg.norm(step) * rng.uniform(0.005, 0.03)
        child = np.clip(parent + step, -half, half)
        nodes.append(child)
        r = float(rng.uniform(5e-4, 3e-3))
        sdfs.append(capsule(tuple(map(float, parent)), tuple(map(float, child)), r, opt_v, 1))
    sdfs.append(box(extent, opt_d, 2))
    return Scene(sdfs)


def skin_layers():
    """Build-defined 'skin' (res/skin.toml names geom_name='skin', which the reference's
    setup_simulation does not know, setup.f90:33-60): epidermis / dermis / subcutis slabs
    as boxes stacked in z inside a 0.1 cm cube (grid half-extent 0.05 as in skin.toml).
    Optical properties (cm^-1) are typical visible-range literature values."""
    ep = mono(400.0, 2.0, 0.8, 1.4)     # 0.01 cm epidermis
    de = mono(200.0, 0.5, 0.85, 1.4)    # 0.05 cm dermis
    sc = mono(120.0, 0.3, 0.8, 1.44)    # remainder subcutis
    z_top = 0.05
    t_ep, t_de = 0.01, 0.05
    z_sc = (-0.05 + (z_top - t_ep - t_de)) / 2
    sdfs = [
        box((0.1, 0.1, t_ep), ep, 1, transform=invert(translate((0.0, 0.0, z_top - t_ep / 2)))),
        box((0.1, 0.1, t_de), de, 2, transform=invert(translate((0.0, 0.0, z_top - t_ep - t_de / 2)))),
        box((0.1, 0.1, (z_top - t_ep - t_de) + 0.05), sc, 3, transform=invert(translate((0.0, 0.0, z_sc)))),
        box((0.1, 0.1, 0.1), mono(0.0, 0.0, 0.0, 1.0), 4),
    ]
    return Scene(sdfs)
