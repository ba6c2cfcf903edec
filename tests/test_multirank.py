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


def _packed_worker(rank, world, port, out_dir):
    """The library's packed layout (smcrt_pack_host / smcrt_unpack_host, the buffer
    smcrt_reduce_device_tallies and smcrt_multi_run reduce over RCCL) reduced with ONE gloo
    all-reduce."""
    from oracle import pyoracle as O
    from rsmcrt_amd import engine
    from rsmcrt_amd.tallies import Result
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    try:
        sc = builders.setup_sphere(10.0, 0.1, 0.9, 1.0, 1.0)
        g = scene.grid(GRID, GRID, GRID, 1.0, 1.0, 1.0)
        dets = [scene.circle_dect((0.0, 0.0, 0.9), (0.0, 0.0, 1.0), 1, 1.0, 20)]
        res = Result(g, dets)
        for s in range(STEPS):
            O.run(sc, g, scene.point_source(), BATCH, dets=dets,
                  first_photon=shard.first_photon(s, rank, world, BATCH), result=res)
        fields = abi.PACK_JMEAN | abi.PACK_ABSORB | abi.PACK_DET_BINS
        buf = torch.from_numpy(engine.pack_result(res, fields))
        dist.all_reduce(buf)  # the one collective
        if rank == 0:
            tot = engine.unpack_into(Result(g, dets), buf.numpy(), fields)
            np.savez(os.path.join(out_dir, "packed.npz"), jmean=tot.jmean, absorb=tot.absorb, det=tot.det_bins,
                     nscatt=tot.nscatt, counters=tot.counters, n=buf.numel())
    finally:
        dist.destroy_process_group()


@pytest.mark.timeout(300)
def test_gloo_world2_packed_layout_matches_single_rank(tmp_path, lib_path):
    from oracle import pyoracle as O
    world = 2
    mp.spawn(_packed_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True)
    got = np.load(tmp_path / "packed.npz")
    sc = builders.setup_sphere(10.0, 0.1, 0.9, 1.0, 1.0)
    g = scene.grid(GRID, GRID, GRID, 1.0, 1.0, 1.0)
    dets = [scene.circle_dect((0.0, 0.0, 0.9), (0.0, 0.0, 1.0), 1, 1.0, 20)]
    ref = O.run(sc, g, scene.point_source(), STEPS * world * BATCH, dets=dets)
    # layout: 2 grids + 21 detector bins + nscatt + 24 moments + 16 counters
    assert int(got["n"]) == 2 * GRID ** 3 + 21 + 1 + 24 + abi.NCOUNTERS
    assert np.array_equal(got["counters"], ref.counters)
    assert np.array_equal(got["absorb"], ref.absorb)
    np.testing.assert_allclose(got["jmean"], ref.jmean, rtol=1e-12, atol=0)
    np.testing.assert_allclose(got["det"], ref.det_bins, rtol=1e-12, atol=0)
    assert got["nscatt"][0] == ref.nscatt[0] and ref.counter("detector_hits") > 0


def test_pack_roundtrip_host(lib_path):
    """smcrt_pack_host -> smcrt_unpack_host accumulates every field (no GPU)."""
    from rsmcrt_amd import engine
    from rsmcrt_amd.tallies import Result
    g = scene.grid(5, 4, 3, 1.0, 1.0, 1.0)
    dets = [scene.circle_dect((0.0, 0.0, 0.9), (0.0, 0.0, 1.0), 1, 1.0, 7)]
    r = Result(g, dets)
    rng = np.random.default_rng(1)
    r.jmean[...] = rng.random(r.jmean.shape)
    r.emission[...] = rng.random(r.jmean.shape)
    r.det_bins[...] = rng.random(r.det_bins.shape)
    r.nscatt[0], r.moments[...] = 12.5, rng.random(24)
    r.counters[...] = np.arange(abi.NCOUNTERS, dtype=np.uint64) * np.uint64(10 ** 12)
    fields = abi.PACK_JMEAN | abi.PACK_EMISSION | abi.PACK_DET_BINS
    buf = engine.pack_result(r, fields)
    assert buf.size == 2 * 60 + 8 + 1 + 24 + abi.NCOUNTERS
    out = Result(g, dets)
    engine.unpack_into(out, buf, fields)
    engine.unpack_into(out, buf, fields)
    assert np.array_equal(out.jmean, 2 * r.jmean) and np.array_equal(out.emission, 2 * r.emission)
    assert not out.absorb.any()  # not packed
    assert np.array_equal(out.det_bins, 2 * r.det_bins) and out.nscatt[0] == 25.0
    assert np.array_equal(out.counters, 2 * r.counters)


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


@pytest.mark.gpu
def test_sharded_device_run_one_rank_comm():
    """bench.sharded_device_run (the N > 1 bench line's GPU side of the parity check) on a
    one-rank RCCL communicator: fresh device tallies, the rank's photons, the packed reduce onto
    root 0 -- equal to eng.run of the same photons (counters and nscatt exact, jmean to fp64
    fold order). The communicator reports one rank."""
    import torch
    import bench
    from rsmcrt_amd import abi, builders, scene
    from rsmcrt_amd.engine import Comm, Engine
    torch.cuda.set_device(0)
    sc = builders.setup_sphere(10.0, 0.1, 0.9, 1.0, 1.0)
    g = scene.grid(32, 32, 32, 1.0, 1.0, 1.0)
    src = scene.point_source()
    comm = Comm(Comm.unique_id(), 1, 0, 0)
    try:
        assert comm.n_ranks == 1
        with Engine(sc, g, device=0) as eng:
            stream = torch.cuda.current_stream()
            got = bench.sharded_device_run(eng, comm, src, g, [], abi.FLAG_PATHLENGTH, 123456789, 5000, 20000,
                                           stream, 0)
            want = eng.run(src, 20000, seed=123456789, first_photon=5000)
    finally:
        comm.close()
    assert got.counters_dict() == want.counters_dict()
    assert got.nscatt[0] == want.nscatt[0]
    np.testing.assert_allclose(got.jmean, want.jmean, rtol=1e-12, atol=1e-15)
    assert np.array_equal(got.absorb, want.absorb)
