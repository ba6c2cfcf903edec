#!/usr/bin/env python3
"""Photons/s of a CSG-heavy scene with nested composites (~56 tops: the culling scene of
tests/test_gpu_parity.py plus models nested 2, 3 and 16 levels deep), so the library picks
the general instantiation; since round 4 its COOP variant (culled and cooperative EVALs).
SMCRT_LIB selects the library. usage: python3 tools/nested_timing.py [photons]"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
from rsmcrt_amd import scene  # noqa: E402
from rsmcrt_amd.engine import Engine  # noqa: E402
from rsmcrt_amd.scene import Scene, box, mono  # noqa: E402
import test_gpu_parity as T  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 1_000_000
sdfs = list(T._culling_scene().sdfs[:-1])
lay = lambda: len(sdfs) + 1  # noqa: E731
for m in T._nested_models(lay, mono(5.0, 0.2, 0.5, 1.45)):
    sdfs.append(m)
sdfs.append(box((2.0, 2.0, 2.0), mono(2.0, 0.05, 0.8, 1.0), lay()))
src = scene.point_source()  # (a source on a wall adds M2's marching wall photons: no far-field march here)
with Engine(Scene(sdfs), scene.grid(64, 64, 64, 1, 1, 1)) as eng:
    eng.run(src, int(os.environ.get("WARM", "100000")))
    t0 = time.perf_counter()
    r = eng.run(src, n, first_photon=1_000_000)
    dt = time.perf_counter() - t0
print(f"nested CSG scene, {len(sdfs)} tops: {n / dt / 1e6:.3f} M photons/s ({n} photons in {dt:.2f} s), "
      f"sdf_evals/photon {r.counter('sdf_evals') / n:.0f}")
