"""One rank of tests/test_launch.py::test_bench_n_rank_cpu_leg_and_parity: bench.py's N > 1
CPU leg and parity (bench.sharded_cpu_parity, bench.attach_cpu_leg) with gloo in place of
RCCL and the CPU restatement in place of each rank's GPU. Rank 0 times the restatement on
photons [0, n), every rank runs its share of the same photons, the shares are summed onto
rank 0 (a gloo reduce here, the engine's packed RCCL reduce in bench.py) and rank 0 prints the
bench line's CPU-leg fields as one JSON line."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import numpy as np
    import torch
    import torch.distributed as dist

    import bench
    from oracle import pyoracle as O
    from rsmcrt_amd import builders, scene
    from rsmcrt_amd.tallies import Result

    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        sc = builders.setup_sphere(10.0, 0.1, 0.9, 1.0, 1.0)
        g = scene.grid(16, 16, 16, 1.0, 1.0, 1.0)
        src = scene.point_source()

        def bcast(n):
            box = [n]
            dist.broadcast_object_list(box, src=0)
            return box[0]

        def sharded(first, count):  # (the oracle stands in for this rank's GPU)
            r = O.run(sc, g, src, count, first_photon=first) if count else Result(g)
            packed = [torch.from_numpy(np.ascontiguousarray(a).reshape(-1).astype(np.float64))
                      for a in (r.jmean, r.absorb, r.emission, r.det_bins, r.nscatt, r.counters)]
            for t in packed:
                dist.reduce(t, dst=0)
            if rank != 0:
                return None
            out = Result(g)
            for a, t in zip((out.jmean, out.absorb, out.emission, out.det_bins, out.nscatt), packed):
                a[...] = t.numpy().reshape(a.shape)
            out.counters[...] = packed[-1].numpy().astype(np.uint64)
            return out

        base, agree = bench.sharded_cpu_parity(
            rank, world, lambda: bench.cpu_run(sc, g, src, [], 1.0, 2, 123456789, 50), bcast, sharded)
        # the N > 1 line's per-rank breakdown: this rank's shard timed, then the reduce timed
        import time
        t0 = time.perf_counter()
        mine = O.run(sc, g, src, 200 * (rank + 1), first_photon=1000 * rank)
        t1 = time.perf_counter()
        tj = torch.from_numpy(mine.jmean.reshape(-1).copy())
        dist.all_reduce(tj)
        t2 = time.perf_counter()
        row = bench.rank_row(rank, 200 * (rank + 1), t2 - t0, t1 - t0, (t2 - t1) * 1e3)
        rows = [None] * world
        dist.all_gather_object(rows, row)
        if rank == 0:
            out = bench.attach_cpu_leg({"n_gpus": world}, base, agree, world)
            print(json.dumps(bench.attach_rank_breakdown(out, rows)), flush=True)
    finally:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
