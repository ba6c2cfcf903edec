"""One rank of the launcher test (tests/test_launch.py), started by rsmcrt_amd.launch.spawn
exactly as bench.py starts its GPU ranks: reads RANK/WORLD_SIZE/MASTER_* from the
environment, runs its photon shards of bench.py's step layout with the CPU restatement,
sums the tallies with gloo and has rank 0 print one JSON line."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import numpy as np
    import torch
    import torch.distributed as dist

    from oracle import pyoracle as O
    from rsmcrt_amd import builders, scene, shard

    steps, batch, n = (int(a) for a in sys.argv[1:4])
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    assert os.environ["MASTER_ADDR"] == "127.0.0.1" and int(os.environ["LOCAL_RANK"]) == rank
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        sc = builders.setup_sphere(10.0, 0.1, 0.9, 1.0, 1.0)
        g = scene.grid(n, n, n, 1.0, 1.0, 1.0)
        res = None
        for s in range(steps):
            res = O.run(sc, g, scene.point_source(), batch, first_photon=shard.first_photon(s, rank, world, batch),
                        result=res)
        jm = torch.from_numpy(res.jmean.reshape(-1).copy())
        ct = torch.from_numpy(res.counters.astype(np.int64))
        shard.reduce_tallies((jm, ct), dist)
        if rank == 0:
            print(json.dumps({"n_ranks": world, "counters": ct.tolist(), "jmean_sum": float(jm.sum()),
                              "jmean_max": float(jm.max())}), flush=True)
    finally:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
