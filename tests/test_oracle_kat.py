"""End-to-end known-answer tests of the CPU restatement against the reference's own
end-to-end tests and validation constants (tests/golden/reference_kats.json)."""
import math

import numpy as np
import pytest

from oracle import pyoracle as O
from rsmcrt_amd import abi, builders, scene


def test_scat_test_nscatt(kats):
    """test_scat.f90:33-38: point source in an isotropic tau=10 sphere, <nscatt> = 57.5+-0.5."""
    k = kats["scat_test_nscatt"]
    n = 100000
    r = O.run(builders.setup_scat_test(10.0), scene.grid(128, 128, 128, 1.0, 1.0, 1.0), scene.point_source(),
              n, flags=abi.FLAG_PATHLENGTH | abi.FLAG_TEST_KERNEL)
    assert r.counter("photons") == n and r.counter("faults") == 0
    assert abs(r.nscatt[0] / n - k["value"]) <= k["thr"]


def test_scat_test2_moments(kats):
    """test_scat.f90:51-84: pencil beam in an infinite g=0.9 medium, scatter-order moments."""
    k = kats["scat_test2_moments"]
    n = 200000
    g = scene.grid(200, 200, 200, 100.0, 100.0, 100.0)
    src = scene.pencil_source((0.0, 0.0, 0.0), (0.0, 0.0, 1.0))
    r = O.run(builders.setup_scat_test2(10.0, 0.9), g, src, n,
              flags=abi.FLAG_PATHLENGTH | abi.FLAG_TEST_KERNEL | abi.FLAG_END_EARLY)
    m = r.moments
    first = 10.0 * m[:12].reshape(4, 3) / n
    second = 100.0 * m[12:].reshape(4, 3) / n
    want1, want2 = np.array(k["first"]), np.array(k["second"])
    for got, want in ((first, want1), (second, want2)):
        assert np.all(np.abs(got[:, :2] - want[:, :2]) <= k["thr_xy"]), got
        assert np.all(np.abs(got[:, 2] - want[:, 2]) <= k["thr_z"]), got
    # the 4th-order first moment is 1+g+g^2+g^3 = 3.439 analytically (the table's 3.349 is a
    # digit transposition that still passes the reference's 0.143 threshold)
    assert abs(first[3, 2] - 3.439) < 0.03


def validation1_setup(nxyz=50):
    sc = builders.setup_box(90.0, 10.0, 0.75, 1.0, (100.0, 100.0, 0.02), (100.0, 100.0, 0.03))
    g = scene.grid(nxyz, nxyz, nxyz, 50.0, 50.0, 0.015)
    src = scene.pencil_source((0.0, 0.0, -0.01), (0.0, 0.0, 1.0))
    dets = [scene.circle_dect((0.0, 0.0, -0.01), (0.0, 0.0, -1.0), 1, 20.0, 100),
            scene.circle_dect((0.0, 0.0, 0.01), (0.0, 0.0, 1.0), 1, 20.0, 100)]
    return sc, g, src, dets


def test_validation1_vdhulst(kats):
    """tools/validateHGG.py:14,26: diffuse R and T of a matched slab (a=0.9, b=2, g=0.75)."""
    k = kats["validation1_RT"]
    sc, g, src, dets = validation1_setup()
    n = 200000
    r = O.run(sc, g, src, n, dets=dets)
    R = r.detector(0).sum() / n
    T = r.detector(1).sum() / n
    for got, want in ((R, k["R"]), (T, k["T"])):
        sigma = math.sqrt(want * (1 - want) / n)
        assert abs(got - want) < 5 * sigma + 1e-3, (got, want)
