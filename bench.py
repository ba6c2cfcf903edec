#!/usr/bin/env python3
"""Throughput benchmark of the photon-transport hot path (BASELINE.json metric:
photon packets/s on a 128^3 fluence grid, 1/2/4/8 GPUs).

Workload (the north-star "single-sphere HG scatterer"): geometry
`sphere` of src/setupGeometry.f90:10-71 (r=1, mus=10, mua=0.1, g=0.9, n=1, in a 2^3 box),
isotropic point source at the origin, 128^3 jmean grid with path-length deposition.
A step = one launch of the transport kernel over a batch of photons per GPU (weak scaling:
the per-GPU batch is fixed). Photon indices are disjoint across steps and ranks, so N GPUs
run N independent shards of one Monte Carlo job; the tallies are summed with one RCCL
all-reduce at the end of the timed region.

Prints ONE JSON line on rank 0. Diagnostics go to stderr.
"""
import argparse
import ctypes as C
import json
import math
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def workload(grid_n):
    from rsmcrt_amd import builders, scene
    sc = builders.setup_sphere(10.0, 0.1, 0.9, 1.0, 1.0)
    g = scene.grid(grid_n, grid_n, grid_n, 1.0, 1.0, 1.0)
    return sc, g, scene.point_source()


def cpu_threads():
    """Host cores to use for the CPU leg: this process's CPU share, at most 16 (the GPU
    box's per-GPU share; nproc there shows the whole machine)."""
    try:
        n = len(os.sched_getaffinity(0))
    except AttributeError:
        n = os.cpu_count() or 1
    env = os.environ.get("OMP_NUM_THREADS")
    if env and env.isdigit():
        n = min(n, int(env))
    return max(1, min(16, n))


def cpu_baseline(sc, g, src, seconds, eng, threads):
    """The CPU restatement (oracle/, C, one photon stream per photon like the GPU) timed on
    `threads` host cores for about `seconds` of wall time: threads pull 2000-photon chunks
    of the same workload (ctypes releases the GIL), so the sample is photons [0, n).
    Then the GPU runs exactly those photons and its fluence is compared with the CPU's."""
    import threading
    import numpy as np
    from oracle import pyoracle as O
    from rsmcrt_amd.tallies import Result
    chunk = 2000
    nxt = [0]
    lock = threading.Lock()
    results = [Result(g) for _ in range(threads)]
    t0 = time.perf_counter()

    def worker(i):
        while time.perf_counter() - t0 < seconds:
            with lock:
                first = nxt[0]
                nxt[0] += chunk
            O.run(sc, g, src, chunk, first_photon=first, result=results[i])

    ths = [threading.Thread(target=worker, args=(i,)) for i in range(threads)]
    for t in ths:
        t.start()
    for t in ths:
        t.join()
    dt = time.perf_counter() - t0
    n = nxt[0]
    res = results[0]
    for r in results[1:]:
        res.merge(r)
    assert res.n_photons == n
    gpu = eng.run(src, n)
    fc, fg = res.normalised_fluence(), gpu.normalised_fluence()
    rmse = float(np.sqrt(np.mean((fg - fc) ** 2)))
    rel = float(np.max(np.abs(fg - fc)) / max(1e-300, float(np.max(np.abs(fc)))))
    same_counters = gpu.counters_dict() == res.counters_dict()
    return {"value": n / dt, "unit": "photon packets/s", "cores": threads, "kind": "port",
            "sample": f"photons [0,{n}) of the same workload, oracle/ C restatement (gcc -O2) on {threads} host "
                      f"threads for {dt:.1f} s",
            "seconds": round(dt, 2)}, {"jmean_rmse_vs_cpu_same_photons": rmse,
                                      "jmean_max_rel_diff_vs_cpu": rel,
                                      "counters_bit_exact_vs_cpu": same_counters,
                                      "photons_compared": n}


def pmc_summary(batch, grid):
    """Per-launch PMC values of the transport kernel (HBM bytes, VALU/SALU instructions)
    from the committed rocprofv3 summary of this exact configuration (tools/profile.sh +
    tools/prof_summary.py -> profiles/transport_traffic.json), else {}."""
    p = os.path.join(ROOT, "profiles", "transport_traffic.json")
    try:
        with open(p) as f:
            t = json.load(f)
    except (OSError, ValueError):
        return {}
    if t.get("batch") != batch or t.get("grid") != grid:
        return {}
    return t


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--batch", type=int, default=16_000_000, help="photons per step per GPU")
    ap.add_argument("--grid", type=int, default=128)
    ap.add_argument("--seed", type=int, default=123456789)
    ap.add_argument("--cpu-seconds", type=float, default=15.0)
    ap.add_argument("--cpu-threads", type=int, default=0, help="0 = this process's CPU share, <= 16")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-deposit", action="store_true", help="diagnostic: pathlength deposition off")
    ap.add_argument("--sync-fold", action="store_true", help="diagnostic: each step waits for its own fold")
    ap.add_argument("--source", default="point", choices=["point", "uniform"],
                    help="diagnostic: uniform = parallelogram source over the z=0.99 plane")
    args = ap.parse_args()

    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", rank=rank, world_size=world)
    else:
        torch.cuda.set_device(0)
    dev = torch.device("cuda", torch.cuda.current_device())

    from rsmcrt_amd import abi, shard
    from rsmcrt_amd.engine import Engine

    sc, g, src = workload(args.grid)
    if args.source == "uniform":
        from rsmcrt_amd import scene as _scene
        src = _scene.uniform_source((-1.0, -1.0, 0.99), (2.0, 0.0, 0.0), (0.0, 2.0, 0.0), (0.0, 0.0, -1.0))
    run_flags = 0 if args.no_deposit else abi.FLAG_PATHLENGTH
    if not args.sync_fold:
        # the deposit fold of step k runs beside step k+1's transport kernel; the fence
        # before the reduce makes jmean complete inside the timed region
        run_flags |= abi.FLAG_ASYNC_FOLD
    eng = Engine(sc, g, device=torch.cuda.current_device())
    nv = g.nx * g.ny * g.nz
    jmean = torch.zeros(nv, dtype=torch.float64, device=dev)
    absorb = torch.zeros(nv, dtype=torch.float64, device=dev)
    nscatt = torch.zeros(1, dtype=torch.float64, device=dev)
    counters = torch.zeros(abi.NCOUNTERS, dtype=torch.int64, device=dev)
    dt_ = abi.DeviceTallies()
    dt_.jmean, dt_.absorb = jmean.data_ptr(), absorb.data_ptr()
    dt_.nscatt, dt_.counters = nscatt.data_ptr(), counters.data_ptr()
    stream = torch.cuda.current_stream()
    B = args.batch

    def step(s):
        cfg = Engine.config(B, seed=args.seed, flags=run_flags, first_photon=shard.first_photon(s, rank, world, B))
        eng.run_device(src, cfg, dt_, stream.cuda_stream)

    for s in range(args.warmup):
        step(s)
    eng.fence(stream.cuda_stream)
    torch.cuda.synchronize()
    eng.set_timing(True)
    eng.kernel_times()  # reset
    c0 = counters.clone()
    if world > 1:
        dist.all_reduce(c0)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for s in range(args.warmup, args.warmup + args.steps):
        step(s)
    eng.fence(stream.cuda_stream)
    if world > 1:
        shard.reduce_tallies((jmean, absorb, nscatt, counters), dist)
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    if world > 1:
        dist.barrier()
    elapsed = torch.tensor([t1 - t0], dtype=torch.float64, device=dev)
    if world > 1:
        dist.all_reduce(elapsed, op=dist.ReduceOp.MAX)
    elapsed = float(elapsed.item())
    kt = eng.kernel_times()  # HIP events around each kernel group, on the launch stream
    eng.set_timing(False)
    launches = max(1, kt["launches"])
    kern_ms = kt["transport_ms"] / launches
    dep_ms = kt["deposit_ms"] / launches
    cdelta = (counters - c0).cpu().numpy()  # all ranks, timed steps only
    photons = world * args.steps * B

    out = None
    if rank == 0:
        deposits = float(cdelta[abi.CTR["deposits"]]) / world  # per rank, over the timed steps
        dep_per_launch = deposits / launches
        # algorithmic HBM bytes of the transport kernel: 8 B per jmean deposit (SURVEY.md
        # §8(d): the reference's fp32 read+write per atomic; here one 8-B deposit record)
        alg_bytes = 8.0 * dep_per_launch
        achieved = alg_bytes / (kern_ms * 1e-3) / 1e9
        pmc = pmc_summary(B, args.grid)
        traffic, traffic_src = pmc.get("hbm_bytes_per_launch"), pmc.get("source")
        # The kernel's binding resource is VALU issue: wave-instructions per launch (PMC
        # SQ_INSTS_VALU of the same command) / the live launch time, against the chip's issue
        # peak of one wave64 VALU instruction per 4 cycles per SIMD (1024 SIMDs, 2.4 GHz).
        valu_peak = 1024 * 2.4e9 / 4 / 1e9
        valu = None
        if pmc.get("valu_insts_per_launch"):
            va = pmc["valu_insts_per_launch"] / (kern_ms * 1e-3) / 1e9
            valu = {"bound": "valu", "achieved": va, "peak": valu_peak, "unit": "G wave-instr/s", "frac": va / valu_peak,
                    "valu_insts_per_launch": pmc["valu_insts_per_launch"],
                    "salu_insts_per_launch": pmc.get("salu_insts_per_launch"), "source": traffic_src}
        out = {
            "metric": "photon packets/sec (128^3 jmean grid, path-length deposition)",
            "value": photons / elapsed,
            "unit": "photon packets/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": elapsed * 1e3 / args.steps,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f64",
            "data": "synthetic (Philox photon streams; scene from setupGeometry.f90 'sphere')",
            "config": {"workload": "M1 single-sphere HG scatterer: sphere r=1 mus=10 mua=0.1 g=0.9 n=1 in 2^3 box, "
                                   "point source at origin, 128^3 grid (setupGeometry.f90:10-71)",
                       "grid": [g.nx, g.ny, g.nz], "photons_per_step_per_gpu": B, "photons_timed": photons,
                       "parallelism": f"photon-index shards x{world} + RCCL all-reduce of tallies"},
            "roofline": {"bound": "hbm", "achieved": achieved, "peak": 8000.0, "unit": "GB/s",
                         "frac": achieved / 8000.0, "traffic": traffic,
                         "kernel": "transport_kernel", "avg_launch_ms": kern_ms,
                         "launches_timed": kt["launches"],
                         "algorithmic_bytes_per_launch": alg_bytes,
                         "traffic_source": traffic_src,
                         "deposits_per_photon": deposits / (args.steps * B),
                         "deposit_fold_ms_per_launch": dep_ms,
                         "wave_iterations_per_launch": float(cdelta[abi.CTR["wave_iters"]]) / world / launches,
                         "binding_resource": "fp64 VALU issue + divergence (see DESIGN.md), not HBM"},
            "valu_roofline": valu,
            "cpu_baseline": None,
        }
    if rank == 0 and world == 1 and not args.no_cpu:
        base, agree = cpu_baseline(sc, g, src, args.cpu_seconds, eng, args.cpu_threads or cpu_threads())
        out["cpu_baseline"] = base
        out["parity"] = agree
    if rank == 0:
        print(json.dumps(out), flush=True)
    eng.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
