"""The bench.py workloads are well-formed scenes: each builds, its
source emits inside the grid, and a few photons of it run through the oracle without a
fault (CPU; the GPU-vs-CPU comparison of each runs in bench.py's CPU leg)."""
import pytest

import bench
from oracle import pyoracle as O
from rsmcrt_amd import scene


@pytest.mark.parametrize("name", ["m0", "m1", "m2", "m3", "m4", "m5"])
def test_workload_runs_on_the_oracle(name):
    sc, g, src, dets, desc, batch = bench.workload(name, 0)
    assert batch > 0 and desc
    small = scene.grid(16, 16, 16, g.xmax, g.ymax, g.zmax)
    r = O.run(sc, small, src, 40, dets=dets)
    c = r.counters_dict()
    assert c["photons"] == 40 and c["faults"] == 0
    assert c["deposits"] > 0 and c["sdf_evals"] > 0
    if dets:
        assert c["detector_hits"] > 0


def test_workload_grid_override():
    _, g, _, _, _, _ = bench.workload("m1", 32)
    assert (g.nx, g.ny, g.nz) == (32, 32, 32)
    _, g, _, _, _, _ = bench.workload("m4", 0)
    assert (g.nx, g.xmax) == (256, 0.16)
    with pytest.raises(ValueError):
        bench.workload("m9", 0)
