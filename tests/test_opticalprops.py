"""Spectral and mono optical properties, pinned by the reference's own
unit tests test/optical_props/test_opticalprops.f90:

  test_mono      :45-79    mono(10, 0.1, 0.9, 1.35) keeps its values; update gives wave = 0
  test_spectral  :81-142   spectral(mus_a, mua_a, hgg_a, n_a, flux) then 10^4 updates: the
                           wavelength in [100, 1000], hgg = 0.9 +- 0.05, mua = 0.1 +- 0.05,
                           n in [1, 2.2], mus in [0, 4]

The sampling is product code (libsmcrt.so smcrt_spectral_sample, rsmcrt_amd.spectral); the
restatement (oracle_spectral_sample) checks it draw for draw, in all three modes. The reference's
own ran2 stream is compiler-specific, so parity here is: the reference's range checks, and the
library equal to the restatement of opticalProperties.f90:127-201 bit for bit. The -m gpu tests
run scenes whose layer takes its properties from a spectral sampler, before and after an update
on the resident scene, against the oracle photon by photon.
"""
import numpy as np
import pytest

from oracle import pyoracle as O
from rsmcrt_amd import abi, builders, scene, spectral

F32 = np.float32


def reference_tables():
    """The arrays of test_spectral (:94-112). Column 2's literals without a kind suffix are
    default (single precision) reals, widened to real(wp) on assignment."""
    wl = np.arange(100.0, 1001.0, 100.0)
    mua = np.stack([wl, np.full(10, F32(0.1), dtype=np.float64)], axis=1)
    flux = np.stack([wl, np.ones(10)], axis=1)
    n = np.stack([wl, np.array([F32(v) for v in (1.0, 1.5, 1.5, 1.0, 1.5, 1.8, 1.9, 2.0, 2.1, 2.2)], dtype=np.float64)], 1)
    mus = np.stack([wl, np.array([0.0, 1.0, 2.0, 3.0, 4.0, 3.0, 2.0, 1.0, 0.5, 0.0])], axis=1)
    hgg = np.stack([np.array([100.0, 450.0, 900.0]), np.full(3, F32(0.9), dtype=np.float64)], axis=1)
    return mus, mua, hgg, n, flux


def test_mono_kat():
    """test_mono (:45-79): mono(10, 0.1, 0.9, 1.35) within 0.05 of its inputs; init_mono's
    kappa and albedo."""
    o = scene.mono(10.0, 0.1, 0.9, 1.35)
    assert abs(o.mus - 10.0) <= 0.05 and abs(o.mua - 0.1) <= 0.05
    assert abs(o.hgg - 0.9) <= 0.05 and abs(o.n - 1.35) <= 0.05
    assert o.kappa == 10.1 and o.albedo == 10.0 / 10.1
    assert scene.mono(1.0, 0.5e-9, 0.0, 1.0).albedo == 1.0  # :115-119


def test_spectral_kat(lib_path):
    """test_spectral (:81-142) through the library: 10^4 updates, every one in the reference's
    bounds."""
    sp = spectral.spectral(*reference_tables(), seed=1234569)
    waves, n, mus = [], [], []
    for _ in range(10000):
        wave = sp.update()
        assert 100.0 <= wave <= 1000.0
        assert abs(sp.hgg - 0.9) <= 0.05
        assert abs(sp.mua - 0.1) <= 0.05
        assert 1.0 <= sp.n <= 2.2
        assert 0.0 <= sp.mus <= 4.0
        assert sp.g2 == sp.hgg * sp.hgg and sp.kappa == sp.mus + sp.mua
        assert sp.albedo == sp.mus / sp.kappa and sp.flags == abi.NODE_ALBEDO_UNGUARDED
        waves.append(wave); n.append(sp.n); mus.append(sp.mus)
    assert sp.draw == 1 + 10000  # one flux draw per update, one for init_spectral
    # the flux is flat: the CDF's trapezoid weights (50, 100, ..., 100, 50 from x = 200) make
    # the wavelength uniform on [100, 1000] apart from the first interval's half weight
    w = np.array(waves)
    assert abs(np.mean((w > 100) & (w <= 200)) - 100 / 850) < 0.02
    assert abs(np.mean(w > 900) - 50 / 850) < 0.015


def test_spectral_library_equals_restatement(lib_path):
    """smcrt_spectral_sample against oracle_spectral_sample, every mode, 2000 samples on the
    reference's tables and on random ragged ones: the properties, the wavelength and the
    stream position bit for bit."""
    rng = np.random.default_rng(7)
    cases = [reference_tables()]
    for _ in range(3):
        tabs = []
        for _t in range(5):
            m = int(rng.integers(2, 40))
            x = np.sort(rng.uniform(300.0, 900.0, m))
            x[0], x[-1] = 300.0, 900.0
            tabs.append(np.stack([x, rng.uniform(0.0, 3.0, m)], axis=1))
        cases.append(tuple(tabs))
    for tabs in cases:
        for mode in (abi.SPECTRAL_INIT, abi.SPECTRAL_UPDATE, abi.SPECTRAL_INIT_AS_WRITTEN):
            sp = spectral.Spectral(*tabs, seed=99, mode=mode)
            d = 0
            for i in range(2000 if mode == abi.SPECTRAL_UPDATE else 200):
                if i:
                    sp._sample(mode)
                ref, d = O.spectral_sample(tabs, mode, 99, d)
                got = {k: getattr(sp, k) for k in ref}
                assert got == ref, (mode, i)
                assert sp.draw == d
            assert d == (5 if mode == abi.SPECTRAL_INIT_AS_WRITTEN else 1) * (2000 if mode == abi.SPECTRAL_UPDATE else 200)


def test_spectral_init_as_written_samples_the_x_axis(lib_path):
    """init_spectral as compiled calls sample(res%mus, wave): `wave` lands in the unused y and
    no value is passed, so each property is drawn from its own table's x axis (a wavelength) --
    kept as a mode, documented, not the default."""
    sp = spectral.spectral(*reference_tables(), seed=3, mode=abi.SPECTRAL_INIT_AS_WRITTEN)
    assert sp.draw == 5
    for v in (sp.mus, sp.mua, sp.hgg, sp.n):
        assert 100.0 <= v <= 1000.0
    sp2 = spectral.spectral(*reference_tables(), seed=3)  # documented intent
    assert sp2.draw == 1 and abs(sp2.hgg - 0.9) <= 0.05 and sp2.flags == 0
    assert sp2.wavelength == sp.wavelength  # the same first (flux) draw


def test_spectral_rejects_bad_tables(lib_path):
    tabs = list(reference_tables())
    tabs[2] = np.array([[500.0, 0.9]])  # n = 1: init_piecewise1D needs array(n >= 2, 2)
    with pytest.raises(ValueError):
        spectral.spectral(*tabs)
    from rsmcrt_amd.engine import SmcrtError
    sp = spectral.spectral(*reference_tables())
    with pytest.raises(SmcrtError):
        sp._sample(7)  # no such mode


def test_node_flags_select_the_albedo_rule():
    """A node built from updateSpectral's properties carries NODE_ALBEDO_UNGUARDED, and its
    Mono derives the albedo without init_mono's guard (:197-199)."""
    o = scene.Mono(1.0, 0.5e-9, 0.0, 1.0, abi.NODE_ALBEDO_UNGUARDED)
    assert o.albedo == 1.0 / (1.0 + 0.5e-9)
    nd = scene.sphere(1.0, o, 1).node()
    assert nd.flags == abi.NODE_ALBEDO_UNGUARDED
    m = scene.model([scene.sphere(1.0, o, 1), scene.sphere(0.5, scene.mono(1, 1, 0, 1), 1)])
    assert scene.Scene([m]).nodes[0].flags == abi.NODE_ALBEDO_UNGUARDED


def _spectral_scene(sp):
    # setup_sphere's geometry (setupGeometry.f90:437-456) with the sphere's layer spectral
    return scene.Scene([scene.sphere(1.0, sp, 1), scene.box((2.0, 2.0, 2.0), scene.mono(0.0, 0.0, 0.0, 1.0), 2)])


def _gpu_tables(n_lo, n_hi):
    wl = np.linspace(400.0, 800.0, 9)
    return (np.stack([wl, np.linspace(5.0, 15.0, 9)], 1), np.stack([wl, np.linspace(0.05, 0.5, 9)], 1),
            np.stack([wl, np.linspace(0.7, 0.95, 9)], 1), np.stack([wl, np.linspace(n_lo, n_hi, 9)], 1),
            np.stack([wl, 1.0 + np.sin(wl / 80.0) ** 2], 1))


@pytest.mark.gpu
@pytest.mark.parametrize("n_range", [(1.0, 1.0), (1.3, 1.5)], ids=["index-matched", "fresnel"])
def test_spectral_layer_runs_bit_exact(n_range):
    """A sphere whose layer is spectral: the run after init_spectral, then updateSpectral on
    the resident scene (Engine.set_spectral) and a second run, each photon by photon against
    the oracle on the same properties."""
    from rsmcrt_amd.engine import Engine
    from test_gpu_parity import compare
    sp = spectral.spectral(*_gpu_tables(*n_range), seed=2024)
    g = scene.grid(64, 64, 64, 1.0, 1.0, 1.0)
    src = scene.point_source()
    with Engine(_spectral_scene(sp), g) as eng:
        for step in range(3):
            if step:
                wave = eng.set_spectral(0, sp)
                assert 400.0 <= wave <= 800.0 and sp.flags == abi.NODE_ALBEDO_UNGUARDED
                layer, mus, mua, hgg, n = eng.get_optprops(0)
                assert (mua, hgg, n) == (sp.mua, sp.hgg, sp.n)
            gpu = eng.run(src, 3000, first_photon=3000 * step, records=True)
            cpu = O.run(_spectral_scene(sp.mono()), g, src, 3000, first_photon=3000 * step, records=True)
            compare(gpu, cpu)
            assert cpu.counter("absorbed") > 0
            if n_range[0] != 1.0:
                assert cpu.counter("fresnel") > 0
