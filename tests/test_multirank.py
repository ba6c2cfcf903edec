"""World-size-2 gloo runs of the sharding + tally reduction used by bench.py (CPU only).

Each rank computes its photon shards with the CPU restatement (the GPU is not needed to
check the decomposition), the tallies are all-reduced with gloo exactly as bench.py does
with RCCL, and the sum must equal one single-rank run over the same photons: counters
bit-exact, fp64 jmean to summation-order rounding.
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from rsmcrt_amd import abi, builders, scene, shard

STEPS, BATCH, GRID = 3, 300, 24


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, out_dir):
    from oracle import pyoracle as O
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    try:
        sc = builders.setup_sphere(10.0, 0.1, 0.9, 1.0, 1.0)
        g = scene.grid(GRID, GRID, GRID, 1.0, 1.0, 1.0)
        res = None
        for s in range(STEPS):
            res = O.run(sc, g, scene.point_source(), BATCH, first_photon=shard.first_photon(s, rank, world, BATCH),
                        result=res)
        jm = torch.from_numpy(res.jmean.reshape(-1).copy())
        ab = torch.from_numpy(res.absorb.reshape(-1).copy())
        ns = torch.from_numpy(res.nscatt.copy())
        ct = torch.from_numpy(res.counters.astype(np.int64))
        shard.reduce_tallies((jm, ab, ns, ct), dist)
        if rank == 0:
            np.savez(os.path.join(out_dir, "sum.npz"), jmean=jm.numpy(), absorb=ab.numpy(), nscatt=ns.numpy(),
                     counters=ct.numpy())
    finally:
        dist.destroy_process_group()


def test_shard_ranges_disjoint_and_complete():
    for world in (1, 2, 4, 8):
        seen = []
        for s in range(3):
            for r in range(world):
                f = shard.first_photon(s, r, world, 10)
                seen.extend(range(f, f + 10))
        assert sorted(seen) == list(range(3 * world * 10))


@pytest.mark.timeout(300)
def test_gloo_world2_matches_single_rank(tmp_path):
    from oracle import pyoracle as O
    world = 2
    mp.spawn(_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True)
    got = np.load(tmp_path / "sum.npz")
    sc = builders.setup_sphere(10.0, 0.1, 0.9, 1.0, 1.0)
    g = scene.grid(GRID, GRID, GRID, 1.0, 1.0, 1.0)
    ref = O.run(sc, g, scene.point_source(), STEPS * world * BATCH)
    assert np.array_equal(got["counters"], ref.counters.astype(np.int64))
    assert got["counters"][abi.CTR["photons"]] == STEPS * world * BATCH
    assert np.array_equal(got["absorb"], ref.absorb.reshape(-1))
    np.testing.assert_allclose(got["jmean"], ref.jmean.reshape(-1), rtol=1e-12, atol=0)
    assert got["nscatt"][0] == ref.nscatt[0]
