"""The SDF domain modifiers of sdfModifiers.f90 (revolution, extrude, onion, twist, bend,
elongate, displacement) in the CPU restatement, on CPU.

Pinned by the reference's own bend KAT (test/SDF/test_SDF.f90:267-304; its twist, elongate,
extrude, revolution, onion and displacement tests are commented out of the suite and hold no
values, :54-62) and by properties the formulas imply exactly (a revolved 2-D egg is the 3-D
Moss egg of setup_egg; twist and bend of a shape symmetric about the rotation axis change
nothing; onion, extrude and elongate of a sphere against their closed forms). The GPU
parity of the same path is tests/test_gpu_parity.py::test_modifier_scenes / test_egg_scene.
"""
import math

import numpy as np
import pytest

from oracle import pyoracle as O
from rsmcrt_amd import abi, builders, scene
from rsmcrt_amd.scene import Scene, box, egg, mono, sphere

OPT = mono(1.0, 0.1, 0.0, 1.0)
EPS = np.finfo(np.float64).eps


def f32(x):
    """A default-real (single precision) literal of the Fortran tests, widened."""
    return float(np.float32(x))


def val(sdf, p):
    return O.sdf_eval(Scene([sdf]), [p])[0]


def test_bend_reference_kat():
    """test_SDF.f90:267-304: box(vector(1.0,1.0,1.0)) bent with k = 10: inside at the origin,
    outside at (0.6, 0, 0) and at (0.4, -0.4, -0.4), where the unbent box is inside."""
    bbox = box((1.0, 1.0, 1.0), OPT, 1)
    bendy = scene.bend(bbox, 10.0)
    assert val(bendy, (0.0, 0.0, 0.0)) < 0.0
    assert val(bendy, (f32(0.6), 0.0, 0.0)) > 0.0
    assert val(bendy, (f32(0.4), f32(-0.4), f32(-0.4))) > 0.0
    assert val(bbox, (f32(0.4), f32(-0.4), f32(-0.4))) < 0.0


def test_revolution_of_egg_is_the_moss_egg():
    """revolution(egg, 0): q = (|p.xz|, p.y, 0), so the revolved egg at (x, y, 0) equals the
    2-D egg at (|x|, y, 0), and it is symmetric about the y axis (setup_egg's shell)."""
    e = egg(2.0, 1.5, 1.4, OPT, 2)
    r = scene.revolution(e, 0.0)
    rng = np.random.Generator(np.random.Philox(3))
    for _ in range(200):
        x, y = rng.uniform(-3.0, 3.0, size=2)
        assert val(r, (x, y, 0.0)) == val(e, (abs(x), y, 0.0))
        th = rng.uniform(0.0, 2.0 * math.pi)
        rr = math.hypot(x, 0.0)
        assert abs(val(r, (rr * math.cos(th), y, rr * math.sin(th))) - val(r, (rr, y, 0.0))) <= 8 * EPS * 4
    # the reference's egg KAT points (test_SDF.f90:1000-1016) hold for the revolved egg in the xy plane
    e2 = scene.revolution(egg(2.5, 0.75, 1.5, OPT, 1), 0.0)
    assert abs(val(e2, (0.0, 0.0, 0.0)) + 2.5) <= EPS and abs(val(e2, (2.5, 0.0, 0.0))) <= EPS
    assert abs(val(e2, (0.0, 4.0, 0.0))) <= 1e-5 and abs(val(e2, (2.5, 2.5, 0.0)) - 0.630294) <= 1e-5


def test_revolution_center_and_offset():
    """center shifts the point first; o is subtracted from the radial distance."""
    s = sphere(0.5, OPT, 1)
    r = scene.revolution(s, 1.0, center=(0.25, -0.5, 0.125))  # a torus of radii 1 and 0.5 about y
    for p in [(1.25, -0.5, 0.125), (0.25, -0.5, 1.125), (2.0, 0.3, -0.7)]:
        q = (p[0] - 0.25, p[1] + 0.5, p[2] - 0.125)
        want = math.hypot(math.hypot(q[0], q[2]) - 1.0, q[1]) - 0.5
        assert abs(val(r, p) - want) <= 16 * EPS


@pytest.mark.parametrize("k", [0.7, -3.0, 12.5])
def test_twist_and_bend_of_axis_symmetric_shapes(k):
    """Rotations in the xy plane keep |p| and p.z: a sphere at the origin is unchanged by
    twist and bend; a box is unchanged by a twist of pi/2 * z-periods only at z = 0."""
    s = sphere(0.8, OPT, 1)
    rng = np.random.Generator(np.random.Philox(5))
    for p in rng.uniform(-1.5, 1.5, size=(100, 3)):
        assert abs(val(scene.twist(s, k), p) - val(s, p)) <= 16 * EPS
        assert abs(val(scene.bend(s, k), p) - val(s, p)) <= 16 * EPS
        assert val(scene.twist(box((1.0, 2.0, 3.0), OPT, 1), k), (p[0], p[1], 0.0)) == \
            val(box((1.0, 2.0, 3.0), OPT, 1), (p[0], p[1], 0.0))


def test_twist_stores_a_single_precision_k():
    """twist_init takes k as a default real (sdfModifiers.f90:131): 0.1 becomes float32(0.1)."""
    t = Scene([scene.twist(sphere(1.0, OPT, 1), 0.1)])
    assert t.nodes[0].param[0] == f32(0.1) != 0.1


def test_onion_extrude_elongate_closed_forms():
    s = sphere(1.0, OPT, 1)
    rng = np.random.Generator(np.random.Philox(9))
    for p in rng.uniform(-2.0, 2.0, size=(100, 3)):
        d = val(s, p)
        assert val(scene.onion(s, 0.1), p) == abs(d) - 0.1
        # extrude: w = (d, |z| - h)
        wy = abs(p[2]) - 0.5
        want = min(max(d, wy), 0.0) + math.sqrt(max(d, 0.0) ** 2 + max(wy, 0.0) ** 2)
        assert abs(val(scene.extrude(s, 0.5), p) - want) <= 8 * EPS
        # elongate a sphere along x by 0.5: a capsule of radius 1 from x = -0.5 to 0.5 where
        # the elongation is outside; inside, min(max(q), 0) is added (sdfModifiers.f90:346-349)
        q = np.abs(p) - np.array([0.5, 0.0, 0.0])
        w = min(max(q[0], max(q[1], q[2])), 0.0)
        qm = np.maximum(q, 0.0)
        assert abs(val(scene.elongate(s, (0.5, 0.0, 0.0)), p) - (math.sqrt(qm @ qm) - 1.0 + w)) <= 8 * EPS


def test_displacement_sine():
    s = sphere(1.0, OPT, 1)
    dsp = scene.displacement_sine(s, 0.05, (7.0, 5.0, 3.0))
    for p in [(0.3, 0.2, 0.1), (-0.9, 0.4, -0.2), (1.2, -1.1, 0.7)]:
        want = val(s, p) + 0.05 * math.sin(7.0 * p[0]) * math.sin(5.0 * p[1]) * math.sin(3.0 * p[2])
        assert abs(val(dsp, p) - want) <= 64 * EPS


def test_nested_modifiers_and_models():
    """Modifiers wrap models and each other (three composite levels), in the reference's
    evaluate chain: onion(revolution(model(union, sphere, box)))."""
    m = scene.model([sphere(0.3, OPT, 1), box((0.2, 0.6, 0.2), OPT, 1)], abi.OP_UNION)
    t = scene.onion(scene.revolution(m, 0.5), 0.05)
    for p in [(0.5, 0.0, 0.0), (0.0, 0.2, 0.5), (1.0, -0.3, 0.4)]:
        q = (math.sqrt(p[0] * p[0] + 0.0 * 0.0 + p[2] * p[2]) - 0.5, p[1], 0.0)  # (length(pxz), vector_class.f90:405-411)
        assert val(t, p) == abs(min(val(sphere(0.3, OPT, 1), q), val(box((0.2, 0.6, 0.2), OPT, 1), q))) - 0.05


def test_egg_scene_runs_on_the_oracle():
    """The egg_test.toml scene (setup_egg) through the restatement: photons reach every layer
    and no photon faults."""
    sc = builders.setup_egg([1.0] * 3, [0.0] * 3, [0.0] * 3, [1.0] * 3, (0.0, 0.0, 0.0), (5.0, 5.0, 5.0))
    g = scene.grid(32, 32, 32, 2.5, 2.5, 2.5)
    r = O.run(sc, g, scene.point_source(), 200)
    c = r.counters_dict()
    assert c["photons"] == 200 and c["faults"] == 0 and c["deposits"] > 0
