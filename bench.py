#!/usr/bin/env python3
"""Throughput benchmark of the photon-transport hot path (BASELINE.json metric:
photon packets/s on a 128^3 fluence grid, 1/2/4/8 GPUs).

Default workload (the north-star "single-sphere HG scatterer"): geometry
`sphere` of src/setupGeometry.f90:10-71 (r=1, mus=10, mua=0.1, g=0.9, n=1, in a 2^3 box),
isotropic point source at the origin, 128^3 jmean grid with path-length deposition.
A step = one launch of the transport kernel over a batch of photons per GPU (weak scaling:
the per-GPU batch is fixed). Photon indices are disjoint across steps and ranks, so N GPUs
run N independent shards of one Monte Carlo job; the tallies are summed with one RCCL
all-reduce at the end of the timed region.

`--workload m0|m2|m3|m4|m5` runs the other §8(d) scenes the same way (diagnostic lines, not
the headline); `--workload escape` times the escape-function driver on
res/default.toml against the CPU restatement run one cell at a time as the reference does.

Prints ONE JSON line on rank 0. Diagnostics go to stderr.
"""
import argparse
import json
import os
import sys
import threading
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

WORKLOADS = ("m0", "m1", "m2", "m3", "m4", "m5", "escape")


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def workload(name, grid_n):
    """(scene, grid, source, detectors, description, default batch) of a SURVEY §8(d) workload.
    grid_n = 0 picks the workload's own grid size."""
    from rsmcrt_amd import builders, scene
    if name == "m0":
        n = grid_n or 200
        return (builders.setup_scat_test(10.0), scene.grid(n, n, n, 1.0, 1.0, 1.0), scene.point_source(), [],
                f"M0 scat_test (res/scat_test.toml): sphere r=1 tau=10 g=0 in 2^3 box, point source, {n}^3 grid "
                "(setupGeometry.f90:409-435)", 3_000_000)
    if name == "m1":
        n = grid_n or 128
        return (builders.setup_sphere(10.0, 0.1, 0.9, 1.0, 1.0), scene.grid(n, n, n, 1.0, 1.0, 1.0),
                scene.point_source(), [],
                "M1 single-sphere HG scatterer: sphere r=1 mus=10 mua=0.1 g=0.9 n=1 in 2^3 box, "
                f"point source at origin, {n}^3 grid (setupGeometry.f90:10-71)", 16_000_000)
    if name == "m2":
        n = grid_n or 128
        return (builders.setup_sphere_scene(builders.random_sphere_list(40)), scene.grid(n, n, n, 1.0, 1.0, 1.0),
                scene.uniform_source((-1.0, -1.0, 0.9999999), (2.0, 0.0, 0.0), (0.0, 2.0, 0.0), (0.0, 0.0, -1.0)),
                [], f"M2 sphere_scene (res/sphere.toml): 40 random spheres n=1.37, uniform source z=0.9999999, "
                f"{n}^3 grid (setupGeometry.f90:250-294)", 400_000)
    if name == "m3":
        n = grid_n or 128
        return (builders.setup_tran_and_jacques(), scene.grid(n, n, n, 1.0, 1.0, 1.0),
                scene.uniform_source((-0.25, 0.0, 0.99999), (0.5, 0.0, 0.0), (0.0, 0.0, 0.0), (0.0, 0.0, -1.0)),
                [], f"M3 aptran (res/aptran.toml, vector direction applied): Tran&Jacques sphere n=1.33 with "
                f"Fresnel, line source, {n}^3 grid (setupGeometry.f90:335-363)", 4_000_000)
    if name == "m4":
        n = grid_n or 256
        return (builders.synthetic_vessels(512), scene.grid(n, n, n, 0.16, 0.09, 0.13),
                scene.uniform_source((-0.16, -0.09, 0.1299), (0.32, 0.0, 0.0), (0.0, 0.18, 0.0), (0.0, 0.0, -1.0)),
                [], f"M4 (build-defined) synthetic vessel net: 512 capsules + dermis box, uniform source, {n}^3 grid",
                1_000_000)
    if name == "m5":
        n = grid_n or 128
        dets = [scene.circle_dect((0.0, 0.0, 0.0499), (0.0, 0.0, 1.0), 1, 0.05, 50),
                scene.annulus_dect((0.0, 0.0, 0.0499), (0.0, 0.0, 1.0), 1, 0.005, 0.02, 25)]
        return (builders.skin_layers(), scene.grid(n, n, n, 0.05, 0.05, 0.05),
                scene.pencil_source((0.0, 0.0, 0.0499), (0.0, 0.0, -1.0)), dets,
                f"M5 (build-defined) skin: layered boxes with Fresnel at every interface, pencil beam, circle + "
                f"annulus reflectance detectors, {n}^3 grid", 8_000_000)
    raise ValueError(name)


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


def cpu_baseline(sc, g, src, dets, seconds, eng, threads, seed, chunk):
    """The CPU restatement (oracle/, C, one photon stream per photon like the GPU) timed on
    `threads` host cores for about `seconds` of wall time: threads pull `chunk`-photon chunks
    of the same workload (ctypes releases the GIL), so the sample is photons [0, n).
    Then the GPU runs exactly those photons and its fluence is compared with the CPU's."""
    import numpy as np
    from oracle import pyoracle as O
    from rsmcrt_amd.tallies import Result
    nxt = [0]
    lock = threading.Lock()
    results = [Result(g, dets) for _ in range(threads)]
    t0 = time.perf_counter()

    def worker(i):
        while time.perf_counter() - t0 < seconds:
            with lock:
                first = nxt[0]
                nxt[0] += chunk
            O.run(sc, g, src, chunk, seed=seed, dets=dets, first_photon=first, result=results[i])

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
    gpu = eng.run(src, n, seed=seed)
    fc, fg = res.normalised_fluence(), gpu.normalised_fluence()
    rmse = float(np.sqrt(np.mean((fg - fc) ** 2)))
    rel = float(np.max(np.abs(fg - fc)) / max(1e-300, float(np.max(np.abs(fc)))))
    agree = {"jmean_rmse_vs_cpu_same_photons": rmse, "jmean_max_rel_diff_vs_cpu": rel,
             "counters_bit_exact_vs_cpu": gpu.counters_dict() == res.counters_dict(),
             "photons_compared": n}
    if dets:
        db = float(np.max(np.abs(gpu.det_bins - res.det_bins)) / max(1e-300, float(np.max(np.abs(res.det_bins)))))
        agree["det_bins_max_rel_diff_vs_cpu"] = db
    return {"value": n / dt, "unit": "photon packets/s", "cores": threads, "kind": "port",
            "sample": f"photons [0,{n}) of the same workload, oracle/ C restatement (gcc -O2) on {threads} host "
                      f"threads for {dt:.1f} s",
            "seconds": round(dt, 2)}, agree


def pmc_summary(name, batch, grid):
    """Per-launch PMC values of the transport kernel (HBM bytes, VALU/SALU instructions)
    from the committed rocprofv3 summary of this exact configuration (tools/profile.sh +
    tools/prof_summary.py -> profiles/transport_traffic.json), else {}."""
    p = os.path.join(ROOT, "profiles", "transport_traffic.json")
    try:
        with open(p) as f:
            t = json.load(f)
    except (OSError, ValueError):
        return {}
    if t.get("workload", "m1") != name or t.get("batch") != batch or t.get("grid") != grid:
        return {}
    return t


def escape_bench(args):
    """Escape function on res/default.toml's scene and detectors (a 50x62x64 scattering box,
    11 annulus detectors) with its 360rotational symmetry on a reduced symmetry grid. The GPU
    runs every launch cell in one batched launch (smcrt_escape_run); the CPU restatement runs
    a sample of cells one run_MCRT at a time, as the reference does (kernelsMod.f90:85-1460),
    on host threads (cells are independent), extrapolated to all cells."""
    import numpy as np
    import torch
    from rsmcrt_amd import escape, scene
    from rsmcrt_amd.engine import Engine
    from rsmcrt_amd.job import Job
    torch.cuda.set_device(0)
    j = Job(os.path.join(ROOT, "tests", "golden", "res", "default.toml"), mode="escape")
    d = j.desc
    c = j.escape_config()
    c.n[0], c.n[2] = args.esc_nr, args.esc_nz  # 360rotational: nr x 1 x nz cells (reference: 100 x 200)
    sc = scene.Scene([])
    sc.nodes = [j.nodes[i] for i in range(d.n_nodes)]
    sc.top = list(j.top[:d.n_top])
    dets = j.detectors
    _, pos = escape.cells(c)
    photons = args.batch or 100000  # the file's nphotons
    with Engine(sc, d.grid, dets) as eng:
        eng.escape(c, 200, source=d.source, seed=d.seed)  # warm-up (pool sizing)
        t0 = time.perf_counter()
        es, _, res = eng.escape(c, photons, source=d.source, seed=d.seed)
        t_gpu = time.perf_counter() - t0
        lay, kap = eng.classify(pos)
        live = (lay != 0) & (kap != 0.0)
        run_cells = int(np.sum(live))
        t0 = time.perf_counter()
        eng.run_origins(pos[live], photons, source=d.source, seed=d.seed)
        t_mc = time.perf_counter() - t0
    t0 = time.perf_counter()
    escape.map_to_grid(c, d.grid, es)
    t_map = time.perf_counter() - t0
    gpu_rate = run_cells * photons / t_gpu
    out = {"metric": "escape-function photon packets/sec (all launch cells, incl. host mapping)",
           "value": gpu_rate, "unit": "photon packets/s", "n_gpus": 1, "steps": 1, "warmup": 1,
           "ms_per_step": t_gpu * 1e3, "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
           "dtype": "f64", "data": "res/default.toml scene and detectors (tests/golden/res)",
           "config": {"workload": "escape function, 360rotational, symmetry grid "
                                  f"{args.esc_nr}x1x{args.esc_nz} ({run_cells} cells run), {photons} photons per cell"},
           "batched_launch_seconds": t_mc, "host_map_seconds": t_map,
           "scatters_per_photon": res.counter("scatters") / (run_cells * photons),
           "deposits_per_photon": res.counter("deposits") / (run_cells * photons),
           "escape_sym_max": float(es.max()), "cpu_baseline": None}
    if not args.no_cpu:
        from oracle import pyoracle as O  # the CPU leg only
        threads = args.cpu_threads or cpu_threads()
        sample = [i for i in range(len(pos)) if live[i]][:threads]
        times = []
        lock = threading.Lock()

        def work(k):
            t = time.perf_counter()
            O.run(sc, d.grid, scene.point_source(tuple(pos[k])), photons, seed=d.seed, dets=dets)
            with lock:
                times.append(time.perf_counter() - t)

        ths = [threading.Thread(target=work, args=(k,)) for k in sample]
        for t in ths:
            t.start()
        for t in ths:
            t.join()
        per_cell = float(np.mean(times))
        cpu_total = per_cell * run_cells / threads
        out["cpu_baseline"] = {"value": run_cells * photons / cpu_total, "unit": "photon packets/s",
                               "cores": threads, "kind": "port",
                               "sample": f"{len(sample)} cells x {photons} photons, one oracle run per cell "
                                         f"(one per thread), extrapolated to {run_cells} cells",
                               "seconds_per_cell_per_thread": per_cell, "seconds_extrapolated": cpu_total}
    print(json.dumps(out), flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--workload", default="m1", choices=WORKLOADS)
    ap.add_argument("--batch", type=int, default=0, help="photons per step per GPU (0 = workload default; "
                                                        "escape: photons per cell)")
    ap.add_argument("--grid", type=int, default=0, help="grid cells per axis (0 = workload default)")
    ap.add_argument("--seed", type=int, default=123456789)
    ap.add_argument("--cpu-seconds", type=float, default=15.0)
    ap.add_argument("--cpu-threads", type=int, default=0, help="0 = this process's CPU share, <= 16")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-deposit", action="store_true", help="diagnostic: pathlength deposition off")
    ap.add_argument("--sync-fold", action="store_true", help="diagnostic: each step waits for its own fold")
    ap.add_argument("--source", default="default", choices=["default", "uniform"],
                    help="diagnostic: uniform = parallelogram source over the z=0.99 plane")
    ap.add_argument("--no-dets", action="store_true", help="diagnostic: the workload's scene without its detectors")
    ap.add_argument("--esc-nr", type=int, default=20)
    ap.add_argument("--esc-nz", type=int, default=10)
    args = ap.parse_args()

    if args.workload == "escape":
        escape_bench(args)
        return

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

    sc, g, src, dets, desc, default_batch = workload(args.workload, args.grid)
    if args.no_dets:
        dets = []
    if args.source == "uniform":
        from rsmcrt_amd import scene as _scene
        src = _scene.uniform_source((-1.0, -1.0, 0.99), (2.0, 0.0, 0.0), (0.0, 2.0, 0.0), (0.0, 0.0, -1.0))
    run_flags = 0 if args.no_deposit else abi.FLAG_PATHLENGTH
    if not args.sync_fold:
        # the deposit fold of step k runs beside step k+1's transport kernel; the fence
        # before the reduce makes jmean complete inside the timed region
        run_flags |= abi.FLAG_ASYNC_FOLD
    eng = Engine(sc, g, dets, device=torch.cuda.current_device())
    nv = g.nx * g.ny * g.nz
    jmean = torch.zeros(nv, dtype=torch.float64, device=dev)
    absorb = torch.zeros(nv, dtype=torch.float64, device=dev)
    nscatt = torch.zeros(1, dtype=torch.float64, device=dev)
    counters = torch.zeros(abi.NCOUNTERS, dtype=torch.int64, device=dev)
    from rsmcrt_amd.tallies import Result
    det_bins = torch.zeros(max(1, len(Result(g, dets).det_bins)), dtype=torch.float64, device=dev)
    dt_ = abi.DeviceTallies()
    dt_.jmean, dt_.absorb = jmean.data_ptr(), absorb.data_ptr()
    dt_.nscatt, dt_.counters = nscatt.data_ptr(), counters.data_ptr()
    if dets:
        dt_.det_bins = det_bins.data_ptr()
    stream = torch.cuda.current_stream()
    B = args.batch or default_batch

    def step(s):
        cfg = Engine.config(B, seed=args.seed, flags=run_flags, first_photon=shard.first_photon(s, rank, world, B))
        eng.run_device(src, cfg, dt_, stream.cuda_stream)

    tw = time.perf_counter()
    for s in range(args.warmup):
        step(s)
    eng.fence(stream.cuda_stream)
    torch.cuda.synchronize()
    log(f"[bench] {args.workload}: {args.warmup} warmup steps of {B} photons in {time.perf_counter() - tw:.2f} s")
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
        shard.reduce_tallies((jmean, absorb, nscatt, counters, det_bins), dist)
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    if world > 1:
        dist.barrier()
    elapsed = torch.tensor([t1 - t0], dtype=torch.float64, device=dev)
    if world > 1:
        dist.all_reduce(elapsed, op=dist.ReduceOp.MAX)
    elapsed = float(elapsed.item())
    log(f"[bench] {args.workload}: {args.steps} timed steps in {elapsed:.2f} s")
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
        pmc = pmc_summary(args.workload, B, g.nx)
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
        metric = "photon packets/sec (128^3 jmean grid, path-length deposition)"
        if args.workload != "m1" or g.nx != 128:
            metric = f"photon packets/sec ({args.workload}, {g.nx}x{g.ny}x{g.nz} jmean grid, path-length deposition)"
        out = {
            "metric": metric,
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
            "data": "synthetic (Philox photon streams; scenes from setupGeometry.f90 / SURVEY §8(d))",
            "config": {"workload": desc,
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
                         "sdf_evals_per_photon": float(cdelta[abi.CTR["sdf_evals"]]) / world / (args.steps * B),
                         "binding_resource": "fp64 VALU issue + divergence (see DESIGN.md), not HBM"},
            "valu_roofline": valu,
            "cpu_baseline": None,
        }
    if rank == 0 and world == 1 and not args.no_cpu:
        log(f"[bench] CPU leg: {args.cpu_seconds} s on the oracle restatement")
        chunk = max(50, min(2000, B // 1000))
        base, agree = cpu_baseline(sc, g, src, dets, args.cpu_seconds, eng, args.cpu_threads or cpu_threads(),
                                   args.seed, chunk)
        out["cpu_baseline"] = base
        out["parity"] = agree
    if rank == 0:
        print(json.dumps(out), flush=True)
    eng.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
