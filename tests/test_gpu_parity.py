"""GPU parity: the HIP path (through the C ABI) against the CPU restatement (oracle/) on the
same seeded inputs.

Integer outputs (counters, nscatt, photon records, unit-weight absorb/emission/detector
bins) must be bit-exact; each photon's final position/direction must be bit-identical
(same Philox stream, same IEEE operations, no FMA contraction on either side). fp64 tallies
built from many atomic adds (jmean, survival-bias absorb, moments) differ only by summation
order: |gpu - cpu| <= 1e-12 * |cpu| + 1e-300 per voxel.
"""
import math

import numpy as np
import pytest

from oracle import pyoracle as O
from rsmcrt_amd import abi, builders, scene
from rsmcrt_amd.engine import Engine

pytestmark = pytest.mark.gpu

RTOL = 1e-12
SEED = 123456789


def compare(gpu, cpu, exact_absorb=True):
    assert gpu.counters_dict() == cpu.counters_dict()
    assert gpu.nscatt[0] == cpu.nscatt[0]
    if gpu.records.size:
        for f in ("pos", "dir", "weight", "cell", "layer", "nscatt", "bounces", "draws", "status"):
            assert np.array_equal(gpu.records[f], cpu.records[f]), f
    np.testing.assert_allclose(gpu.jmean, cpu.jmean, rtol=RTOL, atol=1e-300)
    if exact_absorb:
        assert np.array_equal(gpu.absorb, cpu.absorb)
        assert np.array_equal(gpu.emission, cpu.emission)
    else:
        np.testing.assert_allclose(gpu.absorb, cpu.absorb, rtol=RTOL, atol=1e-300)
    assert np.array_equal(gpu.det_bins, cpu.det_bins)
    np.testing.assert_allclose(gpu.moments, cpu.moments, rtol=RTOL, atol=1e-300)


def both(sc, g, src, n, flags=abi.FLAG_PATHLENGTH, dets=(), first=0, seed=SEED):
    with Engine(sc, g, dets) as eng:
        gpu = eng.run(src, n, seed=seed, flags=flags, first_photon=first, records=True)
    cpu = O.run(sc, g, src, n, seed=seed, flags=flags, dets=dets, first_photon=first, records=True)
    return gpu, cpu


def test_scat_test():
    gpu, cpu = both(builders.setup_scat_test(10.0), scene.grid(64, 64, 64, 1, 1, 1), scene.point_source(), 4000)
    compare(gpu, cpu)
    assert cpu.counter("faults") == 0


def test_scat_test_kernel_mode_and_offset():
    gpu, cpu = both(builders.setup_scat_test(10.0), scene.grid(40, 41, 42, 1, 1, 1), scene.point_source(), 3000,
                    flags=abi.FLAG_PATHLENGTH | abi.FLAG_TEST_KERNEL, first=10 ** 12 + 7)
    compare(gpu, cpu)


def test_single_sphere_hg():
    """M1, the north-star workload: one HG sphere (mus=10, mua=0.1, g=0.9), point source."""
    sc = builders.setup_sphere(10.0, 0.1, 0.9, 1.0, 1.0)
    gpu, cpu = both(sc, scene.grid(128, 128, 128, 1, 1, 1), scene.point_source(), 2000,
                    flags=abi.FLAG_PATHLENGTH | abi.FLAG_RENDER_SOURCE)
    compare(gpu, cpu)
    assert cpu.counter("absorbed") > 0


def test_refracting_sphere_fresnel():
    """aptran: n=1.33 sphere, Fresnel reflect/refract, uniform line source (vector direction)."""
    sc = builders.setup_tran_and_jacques()
    src = scene.uniform_source((-0.25, 0.0, 0.99999), (0.5, 0.0, 0.0), (0.0, 0.0, 0.0), (0.0, 0.0, -1.0))
    gpu, cpu = both(sc, scene.grid(67, 67, 67, 1, 1, 1), src, 4000)
    compare(gpu, cpu)
    assert cpu.counter("fresnel") > 0 and cpu.counter("reflections") > 0


def test_sphere_scene():
    """sphere_scene: 40 non-scattering n=1.37 spheres, uniform source, many SDFs."""
    sc = builders.setup_sphere_scene(builders.random_sphere_list(40))
    src = scene.uniform_source((-1.0, -1.0, 0.9999999), (2.0, 0.0, 0.0), (0.0, 2.0, 0.0), (0.0, 0.0, -1.0))
    gpu, cpu = both(sc, scene.grid(50, 50, 50, 1, 1, 1), src, 2000)
    compare(gpu, cpu)


@pytest.mark.parametrize("variant", ["table", "culled", "global"])
def test_tail_machinery_wall_photons(variant, monkeypatch):
    """Photons launched next to a wall of the bounding box and moving parallel to it march in
    thousands of tiny steps (M2's tail), so most of their steps run in sparse
    waves: the solo march and the cooperative EVAL from the LDS table ("table"), the
    cooperative culled EVAL ("culled": SMCRT_COOP_TAB=0) or the global cooperative EVAL
    ("global": table and culling off). Every variant must equal the oracle bit for bit."""
    if variant != "table":
        monkeypatch.setenv("SMCRT_COOP_TAB", "0")
    if variant == "global":
        monkeypatch.setenv("SMCRT_CULL", "0")
    sc = builders.setup_sphere_scene(builders.random_sphere_list(40))
    src = scene.uniform_source((-1.0, -1.0, 0.9999999), (1e-3, 0.0, 0.0), (0.0, 2.0, 0.0), (0.0, 0.0, -1.0))
    gpu, cpu = both(sc, scene.grid(32, 32, 32, 1, 1, 1), src, 300)
    compare(gpu, cpu)
    assert cpu.counter("sdf_evals") > 300 * 41 * 500  # (long marches: the tail machinery ran)


@pytest.mark.parametrize("case", ["gm2", "gm1", "gm0", "survival", "culled", "off"])
def test_far_field_march(case, monkeypatch):
    """The far-field march (far.h): a lone photon's long march re-evaluates only its nearest
    SDF while a certificate from the last full EVAL bounds every other one. Photons within
    1e-3 of a side wall march parallel to it for ~2/δ steps, most of them in the far-field
    loop. Counters (SDF evaluations, deposits, grid updates), photon records and jmean must
    equal the oracle's exactly as without it ("off": SMCRT_FAR_MARCH=0), on every grid kind
    (GM 2: power-of-two cells, 1: power-of-two extent, 0: neither) and with the unbinned
    (survival-bias) deposit path. "culled": the certificate comes from the culled EVAL
    (SMCRT_COOP_TAB=0) instead of the LDS table."""
    if case == "off":
        monkeypatch.setenv("SMCRT_FAR_MARCH", "0")
    if case == "culled":
        monkeypatch.setenv("SMCRT_COOP_TAB", "0")
    flags = abi.FLAG_PATHLENGTH | (abi.FLAG_SURVIVAL_BIAS if case == "survival" else 0)
    g = {"gm1": scene.grid(50, 50, 50, 1, 1, 1), "gm0": scene.grid(40, 36, 44, 1.25, 1.25, 1.25)}.get(
        case, scene.grid(32, 32, 32, 1, 1, 1))
    sc = builders.setup_sphere_scene(builders.random_sphere_list(40))
    src = scene.uniform_source((-1.0, -1.0, 0.9999999), (1e-3, 0.0, 0.0), (0.0, 2.0, 0.0), (0.0, 0.0, -1.0))
    n = 200
    with Engine(sc, g) as eng:
        eng.kernel_times()
        gpu = eng.run(src, n, seed=SEED, flags=flags, records=True)
        kt = eng.kernel_times()
    cpu = O.run(sc, g, src, n, seed=SEED, flags=flags, records=True)
    compare(gpu, cpu, exact_absorb=case != "survival")
    steps = cpu.counter("grid_updates")
    assert steps > n * 2000  # (long marches)
    if case == "off":
        assert kt["far_steps"] == 0, kt
    else:
        assert kt["far_steps"] > steps // 2, (kt, steps)  # most steps ran in the far-field loop


@pytest.mark.parametrize("variant", ["models", "off"])
def test_far_field_march_with_models(variant, monkeypatch):
    """Round 4: tops that are models of far-eligible primitives (union, smooth union,
    subtraction, intersection, nested) no longer switch the far-field march off (smcrt.hip
    far_ok; their error bound: test_far_bound.py). 30 spheres, 6 models and a medium box take
    the culled EVAL, whose certificate bounds the models as non-near tops; wall photons march
    1e-3 from a side wall. Bit-exact against the oracle and against SMCRT_FAR_MARCH=0."""
    from rsmcrt_amd.scene import Scene, box, capsule, invert, model, mono, sphere, translate
    if variant == "off":
        monkeypatch.setenv("SMCRT_FAR_MARCH", "0")
    sc0 = builders.setup_sphere_scene(builders.random_sphere_list(30))
    sdfs = list(sc0.sdfs[:-1])
    lay = lambda: len(sdfs) + 1  # noqa: E731
    om = mono(4.0, 0.2, 0.6, 1.3)
    t = lambda c: invert(translate(c))  # noqa: E731
    for j in range(6):
        x = -0.6 + 0.24 * j
        kids = [sphere(0.08, om, lay(), transform=t((x, 0.5, 0.2))),
                box((0.06, 0.05, 0.07), om, lay(), transform=t((x + 0.05, 0.52, 0.2))),
                capsule((x, 0.4, 0.0), (x + 0.1, 0.45, 0.1), 0.03, om, lay())]
        op = (abi.OP_UNION, abi.OP_SMOOTH_UNION, abi.OP_SUBTRACTION, abi.OP_INTERSECTION)[j % 4]
        m = model(kids, op, 0.04)
        if j == 5:
            m = model([model(kids[:2], abi.OP_SMOOTH_UNION, 0.03), kids[2]], abi.OP_UNION)
        sdfs.append(m)
    sdfs.append(sc0.sdfs[-1])
    sc = Scene(sdfs)
    g = scene.grid(32, 32, 32, 1, 1, 1)
    src = scene.uniform_source((-1.0, -1.0, 0.9999999), (1e-3, 0.0, 0.0), (0.0, 2.0, 0.0), (0.0, 0.0, -1.0))
    n = 200
    with Engine(sc, g) as eng:
        eng.kernel_times()
        gpu = eng.run(src, n, seed=SEED, records=True)
        kt = eng.kernel_times()
    cpu = O.run(sc, g, src, n, seed=SEED, records=True)
    compare(gpu, cpu)
    assert cpu.counter("grid_updates") > n * 2000  # (long marches)
    if variant == "off":
        assert kt["far_steps"] == 0, kt
    else:
        assert kt["far_steps"] > cpu.counter("grid_updates") // 2, kt


@pytest.mark.parametrize("geom", ["parallel", "oblique"])
@pytest.mark.parametrize("variant", ["table", "culled", "off"])
def test_far_glance_wall_photons(variant, geom, monkeypatch):
    """The boundary probe's glancing loop (inttau2.f90:226-237) with the near top only
    (far.h far_glance). Photons launched within 5e-9 (< eps) of a side wall: moving parallel
    to it ("parallel") the loop never ends in the reference and stops here at the glancing
    guard (MAX_GLANCE_ITERS) with a fault; moving away from it at 1e-3 rad ("oblique") it ends
    after ~1000 iterations. The certificate comes from the LDS table (sphere_scene, 41 tops)
    or the culled EVAL (an 81-top capsule net); "off": SMCRT_FAR_MARCH=0. Counters (faults,
    SDF evaluations), photon records and jmean must equal the oracle's bit for bit."""
    if variant == "off":
        monkeypatch.setenv("SMCRT_FAR_MARCH", "0")
    if variant == "table" or variant == "off":
        sc = builders.setup_sphere_scene(builders.random_sphere_list(40))
        g = scene.grid(32, 32, 32, 1, 1, 1)
        p1, p3 = (-1.0, -1.0, 0.9999999), (0.0, 2.0, 0.0)
    else:
        sc = builders.synthetic_vessels(80)
        g = scene.grid(64, 64, 64, 0.16, 0.09, 0.13)
        p1, p3 = (-0.16, -0.09, 0.1299), (0.0, 0.18, 0.0)
    d = (0.0, 0.0, -1.0) if geom == "parallel" else (math.sin(1e-3), 0.0, -math.cos(1e-3))
    src = scene.uniform_source(p1, (5e-9, 0.0, 0.0), p3, d)
    n = 4
    with Engine(sc, g) as eng:
        eng.kernel_times()
        gpu = eng.run(src, n, seed=SEED, records=True)
        kt = eng.kernel_times()
    cpu = O.run(sc, g, src, n, seed=SEED, records=True)
    compare(gpu, cpu)
    if geom == "parallel":
        assert cpu.counter("faults") == n  # (every photon reached the glancing guard)
    if variant == "off":
        assert kt["far_steps"] == 0, kt
    elif geom == "parallel":
        assert kt["far_steps"] > n * 50000, kt  # most iterations ran in far_glance
    else:
        assert kt["far_steps"] > 0, kt


def test_detectors_validation1():
    sc = builders.setup_box(90.0, 10.0, 0.75, 1.0, (100.0, 100.0, 0.02), (100.0, 100.0, 0.03))
    g = scene.grid(50, 50, 50, 50.0, 50.0, 0.015)
    src = scene.pencil_source((0.0, 0.0, -0.01), (0.0, 0.0, 1.0))
    dets = [scene.circle_dect((0.0, 0.0, -0.01), (0.0, 0.0, -1.0), 1, 20.0, 100),
            scene.circle_dect((0.0, 0.0, 0.01), (0.0, 0.0, 1.0), 1, 20.0, 100)]
    gpu, cpu = both(sc, g, src, 5000, dets=dets)
    compare(gpu, cpu)
    assert cpu.counter("detector_hits") > 0


def test_detectors_all_kinds():
    """res/test_dects.toml detectors (circle, annulus, camera) on scat_test."""
    dets = [scene.circle_dect((-1.0, 0, 0), (-1.0, 0, 0), 4, 0.5, 10),
            scene.annulus_dect((-1.0, 0, 0), (-1.0, 0, 0), 3, 0.5, 1.0, 10),
            scene.camera((-1.0, -1.0, -1.0), (0.0, 2.0, 0.0), (0.0, 0.0, 2.0), 2, 10, 5000.0)]
    gpu, cpu = both(builders.setup_scat_test(10.0), scene.grid(32, 32, 32, 1, 1, 1), scene.point_source(), 3000,
                    dets=dets)
    compare(gpu, cpu)


def test_survival_bias():
    sc = builders.setup_sphere(10.0, 1.0, 0.9, 1.0, 1.0)
    gpu, cpu = both(sc, scene.grid(32, 32, 32, 1, 1, 1), scene.point_source(), 2000,
                    flags=abi.FLAG_PATHLENGTH | abi.FLAG_SURVIVAL_BIAS)
    compare(gpu, cpu, exact_absorb=False)


def test_no_pathlength_mode():
    sc = builders.setup_sphere(10.0, 0.1, 0.9, 1.0, 1.0)
    gpu, cpu = both(sc, scene.grid(32, 32, 32, 1, 1, 1), scene.point_source(), 2000, flags=0)
    compare(gpu, cpu)
    assert cpu.counter("deposits") == 0


def test_csg_model_omg():
    """omg: smooth-union model (torus + 9 cylinders), n=2.65."""
    sc = builders.setup_omg_sdf()
    src = scene.uniform_source((-1.0, -1.0, 0.9999999), (2.0, 0.0, 0.0), (0.0, 2.0, 0.0), (0.0, 0.0, -1.0))
    gpu, cpu = both(sc, scene.grid(32, 32, 32, 1, 1, 1), src, 2000)
    compare(gpu, cpu)


def test_moments_scat_test2():
    g = scene.grid(200, 200, 200, 100.0, 100.0, 100.0)
    src = scene.pencil_source((0.0, 0.0, 0.0), (0.0, 0.0, 1.0))
    gpu, cpu = both(builders.setup_scat_test2(10.0, 0.9), g, src, 20000,
                    flags=abi.FLAG_PATHLENGTH | abi.FLAG_TEST_KERNEL | abi.FLAG_END_EARLY)
    compare(gpu, cpu)


# ----------------------------------------------------- full-size properties (GPU only) --
def test_kat_scat_test_full_size(kats):
    """Reference KAT at 1e6 photons (10x the TOML) on the 128^3 metric grid."""
    n = 1_000_000
    with Engine(builders.setup_scat_test(10.0), scene.grid(128, 128, 128, 1, 1, 1)) as eng:
        r = eng.run(scene.point_source(), n, flags=abi.FLAG_PATHLENGTH | abi.FLAG_TEST_KERNEL)
    assert abs(r.nscatt[0] / n - kats["scat_test_nscatt"]["value"]) <= kats["scat_test_nscatt"]["thr"]
    c = r.counters_dict()
    assert c["photons"] == n and c["escaped"] + c["absorbed"] + c["faults"] == n and c["faults"] == 0


def test_shard_invariance():
    """Splitting a run into photon-index shards (what multi-GPU does) changes nothing:
    integer tallies bit-exact, jmean equal up to summation order."""
    sc = builders.setup_sphere(10.0, 0.1, 0.9, 1.0, 1.0)
    g = scene.grid(64, 64, 64, 1, 1, 1)
    src = scene.point_source()
    n = 200_000
    with Engine(sc, g) as eng:
        whole = eng.run(src, n)
        parts = None
        for k in range(4):
            parts = eng.run(src, n // 4, first_photon=k * (n // 4), result=parts)
    assert whole.counters_dict() == parts.counters_dict()
    assert np.array_equal(whole.absorb, parts.absorb)
    np.testing.assert_allclose(whole.jmean, parts.jmean, rtol=1e-10, atol=1e-300)


def test_point_source_symmetry():
    """An isotropic point source at the centre of a sphere: the 8 octants of jmean agree
    within Monte Carlo noise."""
    n = 2_000_000
    with Engine(builders.setup_scat_test(10.0), scene.grid(64, 64, 64, 1, 1, 1)) as eng:
        r = eng.run(scene.point_source(), n)
    j = r.jmean
    octs = [j[a:a + 32, b:b + 32, c:c + 32].sum() for a in (0, 32) for b in (0, 32) for c in (0, 32)]
    octs = np.array(octs)
    assert np.all(np.abs(octs / octs.mean() - 1.0) < 0.01)
    # Path per photon ~6 cm: a value the survey measured by running the reference's own code
    # (SURVEY §8(d) "[probe]": 6.05 cm/photon at 128^3), not a value the reference holds, so a
    # loose sanity bound only; the reference-held checks are tests/test_reference_targets.py.
    assert abs(j.sum() / n - 6.0) < 0.1


@pytest.mark.parametrize("env", [{}, {"SMCRT_DEPOSIT": "sorted"}, {"SMCRT_FUSED_HIST": "0"},
                                 {"SMCRT_DEPOSIT": "atomic"}],
                         ids=["buckets", "sorted-fused-hist", "sorted-hist-kernel", "atomics"])
def test_deposit_paths(monkeypatch, env):
    """Every jmean deposition path (records filed into per-tile buckets by the transport
    kernel; records sorted by tile with the histogram fused into the transport kernel or
    built by the separate bin_hist kernel; fp64 atomics) gives the oracle's result. The paths
    are chosen when the scene is created."""
    for k, v in env.items():
        monkeypatch.setenv(k, v)
    sc = builders.setup_sphere(10.0, 0.1, 0.9, 1.0, 1.0)
    gpu, cpu = both(sc, scene.grid(96, 96, 96, 1, 1, 1), scene.point_source(), 20000)
    compare(gpu, cpu)
    assert cpu.counter("deposits") > 1_000_000


@pytest.mark.parametrize("mode", ["buckets", "sorted"])
def test_pool_exhaustion_spills_to_atomics(monkeypatch, mode):
    """A record pool far too small for the launch (SMCRT_POOL_CAP) runs out mid-kernel: the
    deposits that no longer fit are added with fp64 atomics, and the tallies still equal
    the oracle's."""
    monkeypatch.setenv("SMCRT_POOL_CAP", str(3 * 16384))
    if mode == "sorted":
        monkeypatch.setenv("SMCRT_DEPOSIT", "sorted")
    sc = builders.setup_sphere(10.0, 0.1, 0.9, 1.0, 1.0)
    gpu, cpu = both(sc, scene.grid(64, 64, 64, 1, 1, 1), scene.point_source(), 20000)
    compare(gpu, cpu)
    assert cpu.counter("deposits") > 20 * 3 * 16384


@pytest.mark.parametrize("cap", [0, 4 * 16384], ids=["pool", "small-pool"])
def test_bucket_contention_pencil_beam(monkeypatch, cap):
    """Block-shared buckets under the worst contention: a pencil beam along +z through a
    weakly scattering sphere, so every lane of every wave of a block crosses the same voxels
    at the same time and files into the same tile word. Claims of the next bucket race with
    deposits of the other waves (deposits past the next bucket take the exact atomic path),
    optionally with a pool that runs out; the tallies still equal the oracle's."""
    if cap:
        monkeypatch.setenv("SMCRT_POOL_CAP", str(cap))
    sc = builders.setup_sphere(0.5, 0.01, 0.9, 1.0, 1.0)
    src = scene.pencil_source((0.0, 0.0, -0.99), (0.0, 0.0, 1.0))
    gpu, cpu = both(sc, scene.grid(64, 64, 64, 1, 1, 1), src, 60000)
    compare(gpu, cpu)
    assert cpu.counter("deposits") > 60000 * 40


def test_multi_launch_pool_reuse():
    """A scene reused for batches of very different size (calibration launch, pool growth,
    sub-batching) accumulates exactly the single-run result."""
    sc = builders.setup_sphere(10.0, 0.1, 0.9, 1.0, 1.0)
    g = scene.grid(64, 64, 64, 1, 1, 1)
    src = scene.point_source()
    with Engine(sc, g) as eng:
        res = eng.run(src, 300, seed=SEED)
        for first, n in ((300, 700_000), (700_300, 50), (700_350, 2_000)):
            eng.run(src, n, seed=SEED, first_photon=first, result=res)
    cpu = O.run(sc, g, src, 702_350, seed=SEED)
    assert res.counters_dict() == cpu.counters_dict()
    np.testing.assert_allclose(res.jmean, cpu.jmean, rtol=RTOL, atol=1e-300)
    assert np.array_equal(res.absorb, cpu.absorb)


def test_vessels_capsule_net():
    """M4 (build-defined): a capsule tree as separate top-level SDFs in a
    dermis box, uniform source over the top face: a deep SDF array (49 SDFs per EVAL),
    bit for bit against the oracle."""
    sc = builders.synthetic_vessels(n_capsules=48)
    g = scene.grid(48, 40, 44, 0.16, 0.09, 0.13)
    src = scene.uniform_source((-0.16, -0.09, 0.1299), (0.32, 0.0, 0.0), (0.0, 0.18, 0.0), (0.0, 0.0, -1.0))
    gpu, cpu = both(sc, g, src, 1500)
    compare(gpu, cpu)
    assert cpu.counter("sdf_evals") > 1500 * 49 * 10


def test_skin_layers_with_detectors():
    """M5 (build-defined): layered boxes with different n (Fresnel at every interface), a
    pencil beam and reflectance detectors on the top surface."""
    sc = builders.skin_layers()
    g = scene.grid(50, 50, 50, 0.05, 0.05, 0.05)
    src = scene.pencil_source((0.0, 0.0, 0.0499), (0.0, 0.0, -1.0))
    dets = [scene.circle_dect((0.0, 0.0, 0.0499), (0.0, 0.0, 1.0), 1, 0.05, 50),
            scene.annulus_dect((0.0, 0.0, 0.0499), (0.0, 0.0, 1.0), 1, 0.005, 0.02, 25)]
    gpu, cpu = both(sc, g, src, 3000, dets=dets)
    compare(gpu, cpu)
    assert cpu.counter("fresnel") > 0


# ---------------------------------------------- general emitter --
def _xsrc_cases():
    rot = (0.3, -0.4, 0.5)
    yield "circular", scene.circular_source((0.1, -0.2, 0.3), (1.0, 2.0, 2.0), 0.5)
    for ft in ("square", "circle", "gaussian"):
        yield f"focus-{ft}", scene.focus_source((0.2, -0.1, 0.4), rot, focal_length=1.5, focus_type=ft, beam_size=0.3)
    for at in ("tophat", "besselAnnulus", "gaussian"):
        yield f"annulus-{at}", scene.annulus_source((0.0, 0.0, 0.9), (0.0, 0.0, -1.0), focal_length=1.2,
                                                    annulus_type=at, rlo=0.3, rhi=0.4, sigma=0.04)
    yield "annulus-outside", scene.annulus_source((-1.5, 0.0, 0.0), (1.0, 0.0, 0.0), focal_length=1.5,
                                                  annulus_type="besselAnnulus", rlo=0.48, rhi=0.52)
    yield "focus-outside", scene.focus_source((0.0, 0.0, 1.6), (0.0, 0.0, -1.0), focal_length=1.6,
                                              focus_type="circle", beam_size=0.4)


@pytest.mark.parametrize("name,src", list(_xsrc_cases()), ids=[c[0] for c in _xsrc_cases()])
def test_general_emitter_sources(name, src):
    """circular / focus / annulus sources (photon.f90:214-308, 361-563, 850-1043) through the
    XSRC kernel instantiation: every photon bit-identical to the CPU restatement."""
    sc = builders.setup_sphere(10.0, 0.1, 0.9, 1.0, 1.0)
    gpu, cpu = both(sc, scene.grid(40, 40, 40, 1, 1, 1), src, 3000,
                    flags=abi.FLAG_PATHLENGTH | abi.FLAG_RENDER_SOURCE)
    compare(gpu, cpu)
    assert cpu.counter("photons") == 3000


def _blood():
    import os
    p = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "test", "optical_props", "blood.dat")
    return np.loadtxt(p, delimiter=",")


@pytest.mark.parametrize("kind", ["point", "uniform", "pencil"])
def test_spectrum_1d_on_basic_sources(kind):
    """A 1-D source spectrum (piecewise1D) moves the basic sources onto the general emitter
    and adds one draw per emission: still bit-identical."""
    if kind == "point":
        s = scene.point_source()
    elif kind == "uniform":
        s = scene.uniform_source((-1.0, -1.0, 0.9999999), (2.0, 0.0, 0.0), (0.0, 2.0, 0.0), (0.0, 0.0, -1.0))
    else:
        s = scene.pencil_source((0.0, 0.0, 0.9999), (0.0, 0.0, -1.0))
    scene.attach_spectrum(s, scene.spectrum_1d(_blood()))
    gpu, cpu = both(builders.setup_scat_test(10.0), scene.grid(32, 32, 32, 1, 1, 1), s, 2000)
    compare(gpu, cpu)


def test_slm_source_2d_spectrum():
    """slm (photon.f90:159-212) sampling a 2-D image (piecewise2D, Morton-ordered CDF)."""
    rng = np.random.default_rng(7)
    img = (rng.random((200, 200)) > 0.7).astype(np.float64)
    s = scene.slm_source((0.0, 0.0, 0.9999), (0.0, 0.0, -1.0), scene.spectrum_2d(img, 2.0 / 200, 2.0 / 200))
    # the emitter maps pixel x to (x - 100) / (nx / (2 xmax)): a 200-wide image needs nx = ny = 200
    gpu, cpu = both(builders.setup_sphere(10.0, 0.1, 0.9, 1.0, 1.0), scene.grid(200, 200, 20, 1, 1, 1), s, 3000,
                    flags=abi.FLAG_PATHLENGTH | abi.FLAG_RENDER_SOURCE)
    compare(gpu, cpu)
    assert cpu.counter("faults") == 0


@pytest.mark.parametrize("kind", ["dslit", "aperture"])
def test_diffraction_sources(kind):
    """dslit / aperture (photon.f90:712-848) with a constant and a 1-D spectrum."""
    g = scene.grid(40, 40, 40, 5.0, 5.0, 5.0)
    sc = builders.setup_box(0.0, 0.0, 0.0, 1.0, (10.0, 10.0, 10.0), (10.0, 10.0, 10.0))
    for sp in (scene.spectrum_constant(500e-7), scene.spectrum_1d(_blood() * [1e-7, 1.0])):
        s = scene.dslit_source() if kind == "dslit" else scene.aperture_source()
        scene.attach_spectrum(s, sp)
        gpu, cpu = both(sc, g, s, 2000)
        compare(gpu, cpu)


def test_fibre_detectors():
    """check_hit_fibre (detectors.f90:331-393) on validateFibreDect.toml's layout: fibres of
    growing aperture above a point source in an empty box; bins bit-exact."""
    sc = builders.setup_box(0.0, 0.0, 0.0, 1.0, (10.0, 10.0, 10.0), (10.0, 10.0, 10.0))
    g = scene.grid(20, 20, 20, 5.0, 5.0, 5.0)
    dets = [scene.fibre_dect((0.0, 0.0, 2.0), (0.0, 0.0, 1.0), 1, 100, focal1=2.0, focal2=20.0, f1_aperture=a,
                             f2_aperture=a, back_offset=20.0, pin_aperture=200.0, core_diameter=1.0)
            for a in (0.5, 1.0, 1.5, 2.0)]
    gpu, cpu = both(sc, g, scene.point_source(), 20000, dets=dets)
    compare(gpu, cpu)
    assert cpu.counter("detector_hits") > 0


# ------------------------------------ escape function --------------
def _escape_scene():
    sc = builders.setup_sphere(10.0, 0.5, 0.8, 1.0, 0.8)
    g = scene.grid(20, 20, 20, 1, 1, 1)
    dets = [scene.circle_dect((0.0, 0.0, 0.99), (0.0, 0.0, 1.0), 1, 0.6, 20),
            scene.annulus_dect((0.0, 0.0, -0.99), (0.0, 0.0, -1.0), 1, 0.2, 0.7, 10),
            scene.camera((-1.0, -1.0, 0.98), (2.0, 0.0, 0.0), (0.0, 2.0, 0.0), 1, 8, 5000.0)]
    return sc, g, dets


def test_run_origins_matches_per_origin_runs():
    """smcrt_run_origins (all launch cells in one batched launch) == one CPU run per origin,
    as the reference calls run_MCRT per cell: per-origin detector totals and counters
    bit-exact, tallies of all origins equal up to summation order."""
    sc, g, dets = _escape_scene()
    origins = [(0.0, 0.0, 0.0), (0.3, -0.2, 0.1), (-0.5, 0.45, 0.2), (0.1, 0.1, -0.6), (0.7, 0.0, 0.0)]
    n = 700
    with Engine(sc, g, dets) as eng:
        tot, res = eng.run_origins(origins, n, seed=SEED, flags=abi.FLAG_PATHLENGTH | abi.FLAG_RENDER_SOURCE)
    cpu = None
    want = np.zeros((len(origins), len(dets)))
    for k, o in enumerate(origins):
        r = O.run(sc, g, scene.point_source(o), n, seed=SEED, flags=abi.FLAG_PATHLENGTH | abi.FLAG_RENDER_SOURCE,
                  dets=dets)
        want[k] = [r.detector(d).sum() for d in range(len(dets))]
        cpu = r if cpu is None else cpu.merge(r)
    assert np.array_equal(tot, want)
    assert want.sum() > 0
    assert res.counters_dict() == cpu.counters_dict()
    assert res.nscatt[0] == cpu.nscatt[0]
    np.testing.assert_allclose(res.jmean, cpu.jmean, rtol=RTOL, atol=1e-300)
    assert np.array_equal(res.absorb, cpu.absorb) and np.array_equal(res.emission, cpu.emission)


def test_classify_matches_oracle_sdfs():
    sc, g, dets = _escape_scene()
    rng = np.random.default_rng(3)
    pts = rng.uniform(-1.2, 1.2, size=(5000, 3))
    with Engine(sc, g, dets) as eng:
        lay, kap = eng.classify(pts)
    ds = np.stack([O.sdf_eval(sc, pts, which=i) for i in range(sc.n_top)], axis=1)
    want = np.zeros(len(pts), dtype=np.int32)
    for p in range(len(pts)):
        best = None
        for i in range(sc.n_top):
            if ds[p, i] < 0.0 and (best is None or ds[p, i] > ds[p, best]):
                best = i
        want[p] = 0 if best is None else best + 1
    assert np.array_equal(lay, want)
    assert set(np.unique(lay)) == {0, 1, 2}


@pytest.mark.parametrize("sym", [("none", (3, 3, 3), (0.9, 0.9, 0.9)),
                                 ("flipped", (3, 2, 4), (0.8, 0.8, 0.8)),
                                 ("360rotational", (3, 4, 3), (0.9, 0.0, 0.9))], ids=lambda s: s[0])
def test_escape_function_end_to_end(sym):
    """smcrt_escape_run (classify, one batched launch, symmetry fill, interpolation) against
    oracle/escape_oracle.py (one CPU run_MCRT per launch cell): escapeSymmetry and escape
    bit-exact (fp32), tallies as in the per-cell runs."""
    from oracle import escape_oracle as EO
    from rsmcrt_amd import escape
    sc, g, dets = _escape_scene()
    kind, n, mx = sym
    cfg = escape.escape_config(kind, n, mx)
    S = EO.Sym(kind, n, mx, (0.0, 0.0, 0.0), (0.0, 0.0, 1.0), 0.0)
    nph = 300
    with Engine(sc, g, dets) as eng:
        es, e, res = eng.escape(cfg, nph, seed=SEED)
    wes, we, cpu = EO.escape_function(sc, g, dets, S, nph, seed=SEED)
    assert np.array_equal(es, wes)
    assert np.array_equal(e, we)
    assert res.counters_dict() == cpu.counters_dict()
    np.testing.assert_allclose(res.jmean, cpu.jmean, rtol=RTOL, atol=1e-300)
    assert es.max() > 0


@pytest.mark.parametrize("apply_trial", [False, True], ids=["reference", "apply-trial"])
def test_inverse_mcrt(apply_trial):
    """smcrt_inverse_run (resident scene, one run per step) against oracle/inverse_oracle.py
    (one CPU run_MCRT per step): gradDescentData bit-exact; the layer is restored."""
    from oracle import inverse_oracle as IO
    sc, g, dets = _escape_scene()
    targets = [0.05, -1.0, 0.3]
    cfg = abi.InverseConfig()
    cfg.layer, cfg.max_steps, cfg.seed = 1, 4, SEED
    cfg.flags = abi.INVERSE_FIND_MUS | abi.INVERSE_FIND_G | (abi.INVERSE_APPLY_TRIAL if apply_trial else 0)
    src = scene.point_source((0.0, 0.0, 0.1))
    with Engine(sc, g, dets) as eng:
        before = eng.get_optprops(0)
        got = eng.inverse(src, cfg, 400, targets, seed=SEED)
        assert eng.get_optprops(0) == before
    want = IO.inverse_mcrt(sc, g, dets, src, 1, {"mus", "g"}, 4, 400, targets, seed=SEED, apply_trial=apply_trial)
    assert np.array_equal(got, want)
    if not apply_trial:
        assert np.all(got[:, 4] == got[0, 4])  # the reference reruns the same scene every step
    else:
        assert len(set(got[:, 4])) > 1


def test_general_emitter_with_detectors():
    """thinBarrier.toml's annulus beam through a 0.5-thick scattering barrier onto a circle
    detector: the general emitter (XSRC) with detector tallies, bit-exact."""
    sc = builders.setup_box(10.0, 0.075, 0.0, 1.0, (0.5, 2.0, 2.0), (3.0, 2.0, 2.0), position=(-0.75, 0.0, 0.0))
    g = scene.grid(61, 41, 41, 1.5, 1.0, 1.0)
    src = scene.annulus_source((-1.5, 0.0, 0.0), (1.0, 0.0, 0.0), focal_length=1.5, annulus_type="besselAnnulus",
                               rlo=0.48, rhi=0.52, sigma=0.05)
    dets = [scene.circle_dect((1.49, 0.0, 0.0), (1.0, 0.0, 0.0), 2, 1.0, 10)]
    gpu, cpu = both(sc, g, src, 3000, dets=dets)
    compare(gpu, cpu)
    assert cpu.counter("detector_hits") > 0


@pytest.mark.parametrize("overlap,slots", [(False, 4), (True, 4), (True, 2)], ids=["async-fold", "overlap", "overlap-2"])
def test_async_fold_pipeline(overlap, slots, monkeypatch):
    """FLAG_ASYNC_FOLD launches on a caller stream (the bench's mode: the fold of launch k runs
    beside later launches' transport kernels in other record slots) + a fence give the same
    tallies as one synchronous run of the same photons. With FLAG_OVERLAP the launches also
    rotate over the scene's internal streams (four here: small record slots; two with
    SMCRT_SLOTS=2), so launch k+1.. start while launch k's slowest photons finish; a plain run
    afterwards is ordered behind them, and the tallies are the same."""
    import torch
    if slots == 2:
        monkeypatch.setenv("SMCRT_SLOTS", "2")
    sc = builders.setup_sphere(10.0, 0.1, 0.9, 1.0, 1.0)
    g = scene.grid(64, 64, 64, 1, 1, 1)
    src = scene.point_source()
    nv = 64 ** 3
    dev = torch.device("cuda", 0)
    jm = torch.zeros(nv, dtype=torch.float64, device=dev)
    ab = torch.zeros(nv, dtype=torch.float64, device=dev)
    ctr = torch.zeros(abi.NCOUNTERS, dtype=torch.int64, device=dev)
    dt = abi.DeviceTallies()
    dt.jmean, dt.absorb, dt.counters = jm.data_ptr(), ab.data_ptr(), ctr.data_ptr()
    stream = torch.cuda.current_stream()
    n, k = 300_000, 5
    fl = abi.FLAG_PATHLENGTH | abi.FLAG_ASYNC_FOLD | (abi.FLAG_OVERLAP if overlap else 0)
    with Engine(sc, g) as eng:
        for i in range(k):
            eng.run_device(src, Engine.config(n, seed=SEED, flags=fl, first_photon=i * n), dt, stream.cuda_stream)
        if overlap:  # a plain launch on the caller's stream waits for the overlapped ones
            eng.run_device(src, Engine.config(n, seed=SEED, flags=abi.FLAG_PATHLENGTH, first_photon=k * n), dt,
                           stream.cuda_stream)
            k += 1
        eng.fence(stream.cuda_stream)
        torch.cuda.synchronize()
        ref = eng.run(src, n * k, seed=SEED)
    np.testing.assert_allclose(jm.cpu().numpy().reshape(64, 64, 64), ref.jmean, rtol=1e-10, atol=1e-300)
    assert np.array_equal(ab.cpu().numpy().reshape(64, 64, 64), ref.absorb)
    c = ctr.cpu().numpy()
    assert int(c[abi.CTR["deposits"]]) == ref.counter("deposits") and int(c[abi.CTR["photons"]]) == n * k


def test_coop_eval_models_and_many_tops():
    """The cooperative tail EVAL (transport.h eval_sdfs_coop, used for scenes with >= 8 tops):
    smooth-union and intersection models among 13 tops, several at once over the same query
    point, Fresnel everywhere (n differs per layer), and a small batch so most EVALs run in
    sparse waves. Must equal the oracle's serial maxloc/minval bit for bit."""
    from rsmcrt_amd.scene import Scene, box, cylinder, invert, model, mono, sphere, translate
    sdfs = []
    for i in range(10):
        x, y, z = (-0.6 + 0.13 * i, 0.25 * ((i % 3) - 1), 0.2 * ((i % 4) - 1.5))
        sdfs.append(sphere(0.08 + 0.01 * (i % 3), mono(3.0, 0.1, 0.8, 1.2 + 0.02 * i), len(sdfs) + 1,
                           transform=invert(translate((x, y, z)))))
    opt_m = mono(5.0, 0.2, 0.5, 1.45)
    sdfs.append(model([sphere(0.2, opt_m, len(sdfs) + 1, transform=invert(translate((0.0, 0.0, 0.5)))),
                       cylinder((0.0, -0.3, 0.5), (0.0, 0.3, 0.5), 0.08, opt_m, len(sdfs) + 1)],
                      abi.OP_SMOOTH_UNION, 0.05))
    sdfs.append(model([sphere(0.25, opt_m, len(sdfs) + 1, transform=invert(translate((0.0, 0.5, -0.5)))),
                       box((0.3, 0.3, 0.3), opt_m, len(sdfs) + 1, transform=invert(translate((0.1, 0.5, -0.5))))],
                      abi.OP_INTERSECTION, 0.0))
    sdfs.append(box((2.0, 2.0, 2.0), mono(0.5, 0.01, 0.0, 1.0), len(sdfs) + 1))
    sc = Scene(sdfs)
    assert sc.n_top == 13
    src = scene.uniform_source((-1.0, -1.0, 0.999), (2.0, 0.0, 0.0), (0.0, 2.0, 0.0), (0.0, 0.0, -1.0))
    gpu, cpu = both(sc, scene.grid(40, 40, 40, 1, 1, 1), src, 1500)
    compare(gpu, cpu)
    assert cpu.counter("fresnel") > 0


def _nested_models(lay, opt_m):
    """Models nested two and three levels deep (eval_model recursing into a child model,
    sdf_base.f90:146-161), with every CSG op at some level."""
    from rsmcrt_amd.scene import box, capsule, cylinder, invert, model, sphere, torus, translate
    t = lambda c: invert(translate(c))  # noqa: E731
    inner = model([sphere(0.1, opt_m, lay(), transform=t((0.3, 0.3, 0.3))),
                   box((0.08, 0.08, 0.08), opt_m, lay(), transform=t((0.35, 0.3, 0.3)))], abi.OP_INTERSECTION)
    two = model([model([capsule((0.2, 0.2, 0.3), (0.4, 0.4, 0.3), 0.03, opt_m, lay()),
                        sphere(0.06, opt_m, lay(), transform=t((0.2, 0.4, 0.3)))], abi.OP_SMOOTH_UNION, 0.04),
                 inner,
                 sphere(0.04, opt_m, lay(), transform=t((0.4, 0.2, 0.3)))], abi.OP_UNION)
    three = model([model([model([sphere(0.12, opt_m, lay(), transform=t((-0.3, -0.3, -0.2))),
                                 sphere(0.09, opt_m, lay(), transform=t((-0.22, -0.3, -0.2)))], abi.OP_SUBTRACTION),
                          torus(0.1, 0.02, opt_m, lay(), transform=t((-0.3, -0.3, -0.1)))], abi.OP_SMOOTH_UNION, 0.03),
                   cylinder((-0.3, -0.45, -0.2), (-0.3, -0.15, -0.2), 0.03, opt_m, lay())], abi.OP_UNION)
    return [two, three, _deep_chain(lay, opt_m)]


def _deep_chain(lay, opt_m, levels=16):
    """A top whose composites nest `levels` deep (geometry.h node_value's explicit stack; the
    reference's eval_model recursion has no depth limit): models (smooth union with a box) and
    modifiers (elongate, revolution) alternate down to a sphere."""
    from rsmcrt_amd.scene import box, elongate, invert, model, revolution, sphere, translate
    t = lambda c: invert(translate(c))  # noqa: E731
    node = sphere(0.05, opt_m, lay(), transform=t((0.3, -0.3, 0.0)))
    for i in range(levels - 1):
        if i % 3 == 0:
            node = model([node, box((0.03, 0.03, 0.03), opt_m, lay(), transform=t((0.33, -0.3, 0.02 * (i % 5))))],
                         abi.OP_SMOOTH_UNION, 0.01)
        elif i % 3 == 1:
            node = elongate(node, (0.002, 0.0, 0.001))
        else:
            node = revolution(node, 0.0, center=(0.0, 0.0, 0.0)) if i == 2 else model([node], abi.OP_UNION)
    return node


@pytest.mark.parametrize("path", ["serial", "coop", "culled"])
def test_nested_models(path):
    """Models inside models (geometry.h PROG_SUB: a child model is one op whose value folds
    its own children, a grandchild model first), two, three and 16 levels deep, in scenes of
    4, 12 and ~56 tops that take the serial, cooperative and culled EVALs: a scene with
    composites below the top level runs the general instantiation (smcrt.hip), and since
    round 4 its COOP variant when it has many tops (cooperative and culled EVALs with the
    composite evaluator), so these check that routing too. Fresnel at every nested surface
    (n differs). Photon records, counters and grids bit-exact against the oracle, whose
    eval_model recursion is the reference's."""
    from rsmcrt_amd.scene import Scene, box, invert, mono, sphere, translate
    sdfs = []
    lay = lambda: len(sdfs) + 1  # noqa: E731
    opt_m = mono(5.0, 0.2, 0.5, 1.45)
    if path == "culled":
        sc0 = _culling_scene()
        sdfs = list(sc0.sdfs[:-1])
    elif path == "coop":
        for i in range(8):
            sdfs.append(sphere(0.05, mono(3.0, 0.1, 0.8, 1.2 + 0.02 * i), lay(),
                               transform=invert(translate((-0.6 + 0.15 * i, 0.5, 0.0)))))
    for m in _nested_models(lay, opt_m):
        sdfs.append(m)
    sdfs.append(box((2.0, 2.0, 2.0), mono(2.0, 0.05, 0.8, 1.0), lay()))
    sc = Scene(sdfs)
    src = scene.uniform_source((-1.0, -1.0, 0.999), (2.0, 0.0, 0.0), (0.0, 2.0, 0.0), (0.0, 0.0, -1.0))
    gpu, cpu = both(sc, scene.grid(32, 32, 32, 1, 1, 1), src, 3000)
    compare(gpu, cpu)
    assert cpu.counter("fresnel") > 0


@pytest.mark.parametrize("kind", ["table", "culled"])
def test_general_emitter_many_tops(kind):
    """A source of the general emitter (circular, photon.f90) in a many-top scene runs
    transport_kernel<.., XSRC, COOP> (round 4; before, such scenes took the serial EVAL): the
    40-sphere scene (cooperative LDS table, far-field march) and the ~56-top culling scene
    (culled EVAL). Counters, photon records and grids bit-exact against the oracle."""
    if kind == "table":
        sc = builders.setup_sphere_scene(builders.random_sphere_list(40))
    else:
        sc = _culling_scene()
    src = scene.circular_source((0.0, 0.0, 0.9999), (0.0, 0.0, -1.0), 0.995)
    gpu, cpu = both(sc, scene.grid(32, 32, 32, 1, 1, 1), src, 3000)
    compare(gpu, cpu)
    assert cpu.counter("photons") == 3000 and cpu.counter("sdf_evals") > 0


def _culling_scene(seed=7):
    """~60 tops for the culled EVAL (cull.h): random capsules, rotated and translated
    spheres, tori and capped cylinders, smooth-union / intersection / subtraction models, a
    cone and a scaled sphere (never culled), inside a medium box (always evaluated)."""
    from rsmcrt_amd.scene import (Scene, box, capsule, cone, cylinder, invert, model, mono, rotate_x, rotate_z,
                                  sphere, torus, translate)
    rng = np.random.default_rng(seed)
    mm = lambda a, b: (np.array(a) @ np.array(b)).tolist()  # noqa: E731
    sdfs = []
    lay = lambda: len(sdfs) + 1  # noqa: E731
    for i in range(30):
        a = rng.uniform(-0.6, 0.6, 3)
        b = a + rng.normal(0, 0.08, 3)
        sdfs.append(capsule(tuple(a), tuple(b), float(rng.uniform(0.01, 0.04)),
                            mono(20.0, 0.5, 0.8, 1.3 + 0.01 * (i % 5)), lay()))
    for i in range(8):
        c = rng.uniform(-0.6, 0.6, 3)
        t = invert(mm(mm(rotate_z(17.0 * i), rotate_x(9.0 * i)), translate(tuple(c))))
        sdfs.append(sphere(float(rng.uniform(0.02, 0.06)), mono(8.0, 0.2, 0.7, 1.4), lay(), transform=t))
    for i in range(4):
        c = rng.uniform(-0.5, 0.5, 3)
        t = invert(mm(rotate_x(30.0 * i), translate(tuple(c))))
        sdfs.append(torus(0.06, 0.015, mono(8.0, 0.2, 0.7, 1.35), lay(), transform=t))
        a = rng.uniform(-0.6, 0.6, 3)
        sdfs.append(cylinder(tuple(a), tuple(a + rng.normal(0, 0.1, 3)), 0.02, mono(8.0, 0.2, 0.7, 1.33), lay()))
    opt_m = mono(5.0, 0.2, 0.5, 1.45)
    sdfs.append(model([sphere(0.07, opt_m, lay(), transform=invert(translate((0.3, 0.3, 0.3)))),
                       capsule((0.3, 0.2, 0.3), (0.3, 0.45, 0.3), 0.03, opt_m, lay())], abi.OP_SMOOTH_UNION, 0.04))
    sdfs.append(model([sphere(0.09, opt_m, lay(), transform=invert(translate((-0.3, 0.3, -0.3)))),
                       box((0.12, 0.12, 0.12), opt_m, lay(), transform=invert(translate((-0.27, 0.3, -0.3))))],
                      abi.OP_INTERSECTION, 0.0))
    sdfs.append(model([sphere(0.05, opt_m, lay(), transform=invert(translate((0.3, -0.3, 0.0)))),
                       sphere(0.08, opt_m, lay(), transform=invert(translate((0.32, -0.3, 0.0))))],
                      abi.OP_SUBTRACTION, 0.0))
    sdfs.append(cone((0.0, -0.5, -0.5), (0.0, -0.4, -0.5), 0.05, 0.02, mono(8.0, 0.2, 0.7, 1.38), lay()))
    sdfs.append(sphere(0.03, mono(8.0, 0.2, 0.7, 1.39), lay(),
                       transform=[[2.0, 0, 0, 0], [0, 2.0, 0, 0], [0, 0, 2.0, 0], [-0.8, 0.8, 0.4, 1.0]]))
    sdfs.append(box((2.0, 2.0, 2.0), mono(3.0, 0.05, 0.8, 1.0), lay()))
    return Scene(sdfs)


@pytest.mark.parametrize("src_kind", ["point", "uniform"])
def test_culled_eval_mixed_scene(src_kind):
    """Exact SDF culling (cull.h, used for scenes with >= 16 tops): a mixed ~60-top scene with
    rigidly transformed primitives, CSG models of every op, and unboundable tops, Fresnel at
    every crossing. Every record, counter and tally equals the oracle's full evaluation."""
    sc = _culling_scene()
    assert sc.n_top >= 50
    src = (scene.point_source() if src_kind == "point" else
           scene.uniform_source((-1.0, -1.0, 0.999), (2.0, 0.0, 0.0), (0.0, 2.0, 0.0), (0.0, 0.0, -1.0)))
    gpu, cpu = both(sc, scene.grid(48, 48, 48, 1, 1, 1), src, 6000)
    compare(gpu, cpu)
    assert cpu.counter("fresnel") > 1000


def test_sync_run_ignores_async_fold_flag():
    """smcrt_run is synchronous: a caller that passes FLAG_ASYNC_FOLD (meant for
    smcrt_run_device) still gets complete tallies, and back-to-back runs do not race the
    previous run's fold (run_sync masks the flag)."""
    sc = builders.setup_sphere(10.0, 0.1, 0.9, 1.0, 1.0)
    g = scene.grid(64, 64, 64, 1, 1, 1)
    src = scene.point_source()
    with Engine(sc, g) as eng:
        a = eng.run(src, 400_000, seed=SEED, flags=abi.FLAG_PATHLENGTH | abi.FLAG_ASYNC_FOLD)
        b = eng.run(src, 400_000, seed=SEED, flags=abi.FLAG_PATHLENGTH | abi.FLAG_ASYNC_FOLD)
        c = eng.run(src, 400_000, seed=SEED)
    for r in (a, b):
        np.testing.assert_allclose(r.jmean, c.jmean, rtol=1e-12, atol=1e-300)
        assert r.counters_dict() == c.counters_dict()


def test_multi_device_run_matches_single():
    """smcrt_multi_run (photon shards over the visible GPUs + one packed RCCL reduce onto the
    first) gives smcrt_run's result: counters, absorb and detector bins bit-exact, jmean to
    the fp64 summation order of the folds (which is not fixed run to run either). On a
    one-GPU box this is the n_devices = 1 path through RCCL."""
    from rsmcrt_amd.engine import MultiEngine
    sc = builders.skin_layers()
    g = scene.grid(64, 64, 64, 0.05, 0.05, 0.05)
    src = scene.pencil_source((0.0, 0.0, 0.0499), (0.0, 0.0, -1.0))
    dets = [scene.circle_dect((0.0, 0.0, 0.0499), (0.0, 0.0, 1.0), 1, 0.05, 50)]
    with MultiEngine(sc, g, dets) as me:
        assert me.n_devices >= 1
        a = me.run(src, 200_000, seed=SEED, first_photon=17)
        me.run(src, 50_000, seed=SEED, first_photon=200_017, result=a)
    with Engine(sc, g, dets) as eng:
        b = eng.run(src, 250_000, seed=SEED, first_photon=17)
    assert a.counters_dict() == b.counters_dict()
    assert np.array_equal(a.absorb, b.absorb)
    assert np.array_equal(a.det_bins, b.det_bins)
    np.testing.assert_allclose(a.jmean, b.jmean, rtol=1e-12, atol=1e-300)
    assert a.nscatt[0] == b.nscatt[0]


def test_reduce_device_tallies_one_rank():
    """smcrt_reduce_device_tallies on a one-rank communicator (the multi-process path bench.py
    takes under torchrun): the packed all-reduce leaves every field as it was, counters
    included (they travel as doubles)."""
    import torch
    from rsmcrt_amd.engine import Comm
    sc = builders.setup_sphere(10.0, 0.1, 0.9, 1.0, 1.0)
    g = scene.grid(32, 32, 32, 1, 1, 1)
    src = scene.point_source()
    dev = torch.device("cuda", 0)
    nv = 32 ** 3
    jm = torch.zeros(nv, dtype=torch.float64, device=dev)
    ab = torch.zeros(nv, dtype=torch.float64, device=dev)
    ns = torch.zeros(1, dtype=torch.float64, device=dev)
    ctr = torch.zeros(abi.NCOUNTERS, dtype=torch.int64, device=dev)
    dt = abi.DeviceTallies()
    dt.jmean, dt.absorb, dt.nscatt, dt.counters = jm.data_ptr(), ab.data_ptr(), ns.data_ptr(), ctr.data_ptr()
    stream = torch.cuda.current_stream()
    comm = Comm(Comm.unique_id(), 1, 0, 0)
    with Engine(sc, g) as eng:
        eng.run_device(src, Engine.config(100_000, seed=SEED), dt, stream.cuda_stream)
        torch.cuda.synchronize()
        before = (jm.clone(), ab.clone(), ns.clone(), ctr.clone())
        for root in (-1, 0):
            eng.reduce_device_tallies(comm, dt, root=root, stream=stream.cuda_stream)
        torch.cuda.synchronize()
    comm.close()
    for x, y in zip((jm, ab, ns, ctr), before):
        assert torch.equal(x, y)
    assert int(ctr[abi.CTR["photons"]]) == 100_000


def test_bucket_claim_delayed_waits_stay_exact(monkeypatch):
    """The bound on the bucket word's 16-bit fill (deposit.h): a debug knob holds every
    bucket claim open for ~27 us before its CAS (SMCRT_DEBUG_CLAIM_DELAY=8, s_sleep 127 x 8),
    so under the pencil-beam contention the block's other waves fill both buckets of the tile
    and their lanes wait for the claim instead of adding without bound. The tallies still
    equal the oracle's, bit for bit in every counter."""
    monkeypatch.setenv("SMCRT_DEBUG_CLAIM_DELAY", "8")
    sc = builders.setup_sphere(0.5, 0.01, 0.9, 1.0, 1.0)
    src = scene.pencil_source((0.0, 0.0, -0.99), (0.0, 0.0, 1.0))
    gpu, cpu = both(sc, scene.grid(64, 64, 64, 1, 1, 1), src, 60000)
    compare(gpu, cpu)


def test_multi_accumulate_dynamic_chunks_one_collect(monkeypatch):
    """The batched multi-GPU path: photons handed to the devices in many small chunks
    (SMCRT_MULTI_CHUNK) over several smcrt_multi_accumulate calls, overlapped launches
    requested by the caller (SMCRT_FLAG_OVERLAP is honoured: the collect fences every launch
    and fold), then ONE smcrt_multi_collect: the result is smcrt_run's over the same photons,
    counters, absorb and detector bins bit-exact."""
    from rsmcrt_amd.engine import MultiEngine
    monkeypatch.setenv("SMCRT_MULTI_CHUNK", "7000")
    sc = builders.skin_layers()
    g = scene.grid(64, 64, 64, 0.05, 0.05, 0.05)
    src = scene.pencil_source((0.0, 0.0, 0.0499), (0.0, 0.0, -1.0))
    dets = [scene.circle_dect((0.0, 0.0, 0.0499), (0.0, 0.0, 1.0), 1, 0.05, 50)]
    fl = abi.FLAG_PATHLENGTH | abi.FLAG_OVERLAP | abi.FLAG_ASYNC_FOLD
    with MultiEngine(sc, g, dets) as me:
        me.accumulate(src, 60_000, seed=SEED, flags=fl, first_photon=5)
        me.accumulate(src, 40_000, seed=SEED, flags=fl, first_photon=60_005)
        assert sum(me.device_photons()) == 100_000
        a = me.collect()
        assert sum(me.device_photons()) == 0
        b2 = me.run(src, 10_000, seed=SEED, flags=fl, first_photon=5)  # (accumulators were zeroed)
    with Engine(sc, g, dets) as eng:
        b = eng.run(src, 100_000, seed=SEED, first_photon=5)
        c = eng.run(src, 10_000, seed=SEED, first_photon=5)
    assert a.n_photons == 100_000
    assert a.counters_dict() == b.counters_dict() and b2.counters_dict() == c.counters_dict()
    assert np.array_equal(a.absorb, b.absorb) and np.array_equal(a.det_bins, b.det_bins)
    np.testing.assert_allclose(a.jmean, b.jmean, rtol=1e-12, atol=1e-300)
    assert a.nscatt[0] == b.nscatt[0]


@pytest.mark.parametrize("case", ["absorbing", "boundary-source", "test-kernel", "fresnel", "detectors",
                                  "bounce-abort", "fresnel-test-kernel"])
def test_lean_kernel_paths(monkeypatch, case):
    """The lean path (ws_kernel, ws.h: scenes of few tops, the voxel walk and the interactions
    decoupled from the photon; Fresnel scenes by default and detector scenes with SMCRT_LEAN=1
    through its XF instantiation) against the oracle, photon by photon, on the paths it adds:
    * absorbing: mua = 2 (albedo 0.83), so many photons are absorbed while their last
      segment is still being walked (ST_ABSORB waits for the cells recordWeight needs);
    * boundary-source: a uniform source on the top face, so segments near the grid faces are
      synchronous (the photon waits for tflag/cells) and escapes through the walk are common;
    * test-kernel: test_kernel semantics (no re-emission, ds<=0 mask, scatter moments);
    * fresnel: the Tran & Jacques sphere (n=1.33 in air, M3's scene): reflect_refract (the ds
      pair, the calcNormal taps, reflection and refraction) as an event of the event waves;
    * detectors: M5's layered skin with Fresnel at every interface and a circle and an annulus
      detector at the top face (record_hits from each segment's start point);
    * bounce-abort: an almost transparent n=1.5 sphere with an off-centre source, so photons
      caught by total internal reflection reach 1000 bounces and return to their tauint2
      entry (inttau2.f90:313-315);
    * fresnel-test-kernel: the Tran & Jacques sphere with test_kernel semantics, whose events
      stay in the photon waves while its Fresnel events go to the event waves.
    Each case runs the lean path with three and with two segment slots per photon
    (SMCRT_WS_SLOTS=2, the instantiation of grids whose LDS cannot hold three) and
    transport_kernel (SMCRT_LEAN=0): same counters and records."""
    from rsmcrt_amd.engine import Engine as E
    flags = abi.FLAG_PATHLENGTH
    g = scene.grid(48, 48, 48, 1, 1, 1)
    dets = []
    if case in ("fresnel", "fresnel-test-kernel"):
        sc, n = builders.setup_tran_and_jacques(), 30000
        if case == "fresnel-test-kernel":
            flags |= abi.FLAG_TEST_KERNEL
        src = scene.uniform_source((-0.25, 0.0, 0.99999), (0.5, 0.0, 0.0), (0.0, 0.0, 0.0), (0.0, 0.0, -1.0))
    elif case == "detectors":
        sc, n, g = builders.skin_layers(), 30000, scene.grid(48, 48, 48, 0.05, 0.05, 0.05)
        src = scene.pencil_source((0.0, 0.0, 0.0499), (0.0, 0.0, -1.0))
        dets = [scene.circle_dect((0.0, 0.0, 0.0499), (0.0, 0.0, 1.0), 1, 0.05, 50),
                scene.annulus_dect((0.0, 0.0, 0.0499), (0.0, 0.0, 1.0), 1, 0.005, 0.02, 25)]
    elif case == "bounce-abort":
        sc, n, g = builders.setup_sphere(1e-4, 1e-5, 0.0, 1.5, 1.0), 100, scene.grid(32, 32, 32, 1, 1, 1)
        src = scene.point_source((0.85, 0.0, 0.0))
    elif case == "absorbing":
        sc, src, n = builders.setup_sphere(10.0, 2.0, 0.9, 1.0, 1.0), scene.point_source(), 30000
    elif case == "boundary-source":
        sc = builders.setup_sphere(5.0, 0.5, 0.8, 1.0, 1.0)
        src = scene.uniform_source((-1.0, -1.0, 0.999), (2.0, 0.0, 0.0), (0.0, 2.0, 0.0), (0.0, 0.0, -1.0))
        n = 30000
    else:
        sc, src, n = builders.setup_scat_test(10.0), scene.point_source(), 20000
        flags |= abi.FLAG_TEST_KERNEL
    runs = {}
    for lean, slots in (("1", "3"), ("1", "2"), ("0", "3")):
        monkeypatch.setenv("SMCRT_LEAN", lean)
        monkeypatch.setenv("SMCRT_WS_SLOTS", slots)
        with E(sc, g, dets) as eng:
            eng.kernel_times()
            runs[lean + slots] = eng.run(src, n, seed=SEED, flags=flags, records=True)
            kt = eng.kernel_times()
        assert (kt["lean_launches"] > 0) == (lean == "1"), (lean, kt)
        if lean == "1":  # the lean path runs only on the bucketed path: bk_reduce ran and was timed
            assert 0.0 < kt["fold_cu_ms"] < 1e3, kt
            assert kt["lean_hazards"] == 0, kt  # (detectors: starts outside their cell are synchronous)
    cpu = O.run(sc, g, src, n, seed=SEED, flags=flags, records=True, dets=dets)
    for r in runs.values():
        compare(r, cpu)
    if case in ("fresnel", "detectors", "fresnel-test-kernel"):
        assert cpu.counter("fresnel") > n and cpu.counter("reflections") > 0
    if case == "detectors":
        assert cpu.counter("detector_hits") > 0
    if case == "bounce-abort":
        assert cpu.counter("bounce_aborts") > 0
    if case == "absorbing":
        assert cpu.counter("absorbed") > n // 2
    if case == "test-kernel":
        for k in ("13", "12"):
            np.testing.assert_allclose(runs[k].moments, cpu.moments, rtol=1e-12)


def test_lean_path_two_slots_by_lds():
    """A 2048 x 64 x 64 grid: its staged faces (17 KiB) and tile words do not fit beside three
    segment slots per photon, so the lean path picks its two-slot instantiation by itself
    (smcrt.hip: ws_slots); same photons as the oracle, bit for bit."""
    from rsmcrt_amd.engine import Engine as E
    sc, g = builders.setup_sphere(10.0, 0.1, 0.9, 1.0, 1.0), scene.grid(2048, 64, 64, 1, 1, 1)
    src, n = scene.point_source(), 3000
    with E(sc, g) as eng:
        eng.kernel_times()
        gpu = eng.run(src, n, seed=SEED, flags=abi.FLAG_PATHLENGTH, records=True)
        kt = eng.kernel_times()
    assert kt["lean_launches"] > 0 and kt["lean_hazards"] == 0, kt
    cpu = O.run(sc, g, src, n, seed=SEED, flags=abi.FLAG_PATHLENGTH, records=True)
    compare(gpu, cpu)


@pytest.mark.parametrize("knob", ["0", "all"])
def test_lean_hazards_counted_as_faults(monkeypatch, knob):
    """A deferred lean-kernel walk (lean.h) must never end in tflag or an error stop; if one
    did, its photon would already have gone on as if the walk stayed inside the grid. Every
    such "hazard" is counted in SMCRT_CTR_FAULTS and returned in kernel_times.lean_hazards
    (INTEGRATION.md §6). The debug knob SMCRT_DEBUG_LEAN_MARGIN provokes them on the
    boundary-source scene: "0" drops the walk's margin from the grid faces, "all" defers every
    segment that starts in the grid, so walks that leave the grid become hazards. Without the
    knob the same run has no hazard and equals the oracle; with it, the faults counter equals
    the oracle's plus the hazards."""
    sc = builders.setup_sphere(5.0, 0.5, 0.8, 1.0, 1.0)
    src = scene.uniform_source((-1.0, -1.0, 0.999), (2.0, 0.0, 0.0), (0.0, 2.0, 0.0), (0.0, 0.0, -1.0))
    g = scene.grid(48, 48, 48, 1, 1, 1)
    n = 30000
    monkeypatch.setenv("SMCRT_LEAN", "1")
    with Engine(sc, g) as eng:
        eng.kernel_times()
        clean = eng.run(src, n, seed=SEED, records=True)
        kt_clean = eng.kernel_times()
    monkeypatch.setenv("SMCRT_DEBUG_LEAN_MARGIN", knob)
    with Engine(sc, g) as eng:
        eng.kernel_times()
        haz = eng.run(src, n, seed=SEED, records=True)
        kt = eng.kernel_times()
    cpu = O.run(sc, g, src, n, seed=SEED, records=True)
    assert kt_clean["lean_launches"] > 0 and kt_clean["lean_hazards"] == 0, kt_clean
    compare(clean, cpu)
    assert kt["lean_launches"] > 0, kt
    if knob == "all":
        assert kt["lean_hazards"] > 0, kt
    assert haz.counter("faults") == cpu.counter("faults") + kt["lean_hazards"], (haz.counter("faults"), kt)


def test_egg_scene_revolution():
    """res/egg_test.toml's scene (setup_egg, setupGeometry.f90:149-248: two Moss eggs revolved
    about y by the revolution modifier, a yolk, a bounding box) at 64^3, through the general
    instantiation's composite evaluator (geometry.h node_value), bit-exact against the oracle.
    Distinct optical properties per layer so that every layer matters."""
    sc = builders.setup_egg([8.0, 3.0, 15.0], [0.2, 0.05, 1.0], [0.8, 0.6, 0.9], [1.0, 1.0, 1.0],
                            (0.0, 0.0, 0.0), (5.0, 5.0, 5.0))
    gpu, cpu = both(sc, scene.grid(64, 64, 64, 2.5, 2.5, 2.5), scene.point_source(), 3000,
                    flags=abi.FLAG_PATHLENGTH | abi.FLAG_RENDER_SOURCE)
    compare(gpu, cpu)
    assert cpu.counter("absorbed") > 0 and cpu.counter("faults") == 0


def test_modifier_scenes():
    """Every modifier of sdfModifiers.f90 in one Fresnel scene (refractive indices differ, so
    calcNormal and reflect_refract evaluate them too): extrude, onion, twist, bend, elongate,
    displacement, and a revolved CSG model, with a pencil and a point source; bit-exact
    against the oracle."""
    from rsmcrt_amd.scene import box as bx, model, mono as mo, sphere as sp, torus as to, translate, invert
    o1, o2, o3 = mo(5.0, 0.5, 0.7, 1.2), mo(2.0, 0.1, 0.3, 1.0), mo(9.0, 0.2, 0.9, 1.4)
    tops = [
        scene.onion(sp(0.25, o1, 1, transform=invert(translate((0.5, 0.5, 0.0)))), 0.05),
        scene.twist(bx((0.3, 0.2, 0.6), o2, 2, transform=invert(translate((-0.5, 0.5, 0.0)))), 2.5),
        scene.bend(bx((0.5, 0.1, 0.2), o3, 3, transform=invert(translate((0.0, -0.5, 0.3)))), 1.5),
        scene.elongate(to(0.12, 0.04, o1, 4, transform=invert(translate((0.5, -0.5, -0.4)))), (0.1, 0.0, 0.05)),
        scene.displacement_sine(sp(0.2, o2, 5, transform=invert(translate((-0.5, -0.5, -0.3)))), 0.02, (9.0, 7.0, 5.0)),
        scene.extrude(sp(0.2, o3, 6, transform=invert(translate((0.0, 0.0, 0.5)))), 0.1),
        scene.revolution(model([sp(0.1, o1, 7), bx((0.1, 0.3, 0.1), o1, 7)], abi.OP_SMOOTH_UNION, 0.05), 0.3,
                         center=(0.0, 0.1, -0.5)),
        bx((2.0, 2.0, 2.0), mo(0.5, 0.01, 0.0, 1.0), 8),
    ]
    sc = scene.Scene(tops)
    g = scene.grid(48, 48, 48, 1, 1, 1)
    for src, n in ((scene.point_source(), 3000), (scene.pencil_source((0.0, 0.0, 0.99), (0.0, 0.0, -1.0)), 3000)):
        gpu, cpu = both(sc, g, src, n)
        compare(gpu, cpu)
        assert cpu.counter("fresnel") > 0


def test_watchdog_lost_event_is_an_error_not_a_hang(monkeypatch):
    """The watchdog: a photon whose event is marked queued but never
    queued (SMCRT_DEBUG_DROP_EVENT: photon lane 0 of block 0, its first event -- the class of
    the round-5 test_kernel Fresnel bug) would wait forever. With every cross-wave wait bounded
    (SMCRT_WATCHDOG_MS) its wave gives up, the block's waves leave their loops, the grid
    drains, and the run returns DEVICE_FAULT naming the photon-wave wait -- in well under the
    test's time limit. The word is cleared, so the same resident scene then runs exactly."""
    import time
    from rsmcrt_amd.engine import SmcrtError
    sc = builders.setup_sphere(10.0, 0.1, 0.9, 1.0, 1.0)
    g = scene.grid(64, 64, 64, 1, 1, 1)
    src = scene.point_source()
    monkeypatch.setenv("SMCRT_LEAN", "1")
    monkeypatch.setenv("SMCRT_WATCHDOG_MS", "300")
    with Engine(sc, g) as eng:
        monkeypatch.setenv("SMCRT_DEBUG_DROP_EVENT", "1")
        t0 = time.time()
        with pytest.raises(SmcrtError, match=r"DEVICE_FAULT.*watchdog.*photon wave.*block 0"):
            eng.run(src, 20000, seed=SEED)
        assert time.time() - t0 < 60
        monkeypatch.delenv("SMCRT_DEBUG_DROP_EVENT")
        eng.kernel_times()
        gpu = eng.run(src, 3000, seed=SEED, records=True)
        assert eng.kernel_times()["lean_launches"] > 0
        eng.check()  # (nothing pending, no fault)
    cpu = O.run(sc, g, src, 3000, seed=SEED, records=True)
    compare(gpu, cpu)


def test_watchdog_bucket_wait(monkeypatch):
    """The bucket wait of deposit.h under the watchdog: every claim held open ~27 us
    (SMCRT_DEBUG_CLAIM_DELAY=8) against a 5 us budget, so the lanes that wait for a claim give
    up; the run returns DEVICE_FAULT naming the bucket wait (transport_kernel: SMCRT_LEAN=0, so
    no photon-wave wait can fire first). Without the tiny budget the same run is exact
    (test_bucket_claim_delayed_waits_stay_exact)."""
    from rsmcrt_amd.engine import SmcrtError
    monkeypatch.setenv("SMCRT_LEAN", "0")
    monkeypatch.setenv("SMCRT_DEBUG_CLAIM_DELAY", "8")
    monkeypatch.setenv("SMCRT_WATCHDOG_MS", "0.005")
    sc = builders.setup_sphere(0.5, 0.01, 0.9, 1.0, 1.0)
    src = scene.pencil_source((0.0, 0.0, -0.99), (0.0, 0.0, 1.0))
    with Engine(sc, scene.grid(64, 64, 64, 1, 1, 1)) as eng:
        with pytest.raises(SmcrtError, match=r"DEVICE_FAULT.*watchdog.*bucket wait"):
            eng.run(src, 60000, seed=SEED)
