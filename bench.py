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
# at least eight (at most 32) hardware queues for the scene's streams, set before torch starts
# the HIP runtime (rsmcrt_amd/__init__.py explains; the boxes export HIP's default of 4). The
# package imports no torch, so this still runs first.
from rsmcrt_amd import _raise_hw_queues  # noqa: E402

_raise_hw_queues()

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
                f"{n}^3 grid (setupGeometry.f90:250-294)", 25_600_000)
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
                8_000_000)
    if name == "m5":
        n = grid_n or 128
        dets = [scene.circle_dect((0.0, 0.0, 0.0499), (0.0, 0.0, 1.0), 1, 0.05, 50),
                scene.annulus_dect((0.0, 0.0, 0.0499), (0.0, 0.0, 1.0), 1, 0.005, 0.02, 25)]
        return (builders.skin_layers(), scene.grid(n, n, n, 0.05, 0.05, 0.05),
                scene.pencil_source((0.0, 0.0, 0.0499), (0.0, 0.0, -1.0)), dets,
                f"M5 (build-defined) skin: layered boxes with Fresnel at every interface, pencil beam, circle + "
                f"annulus reflectance detectors, {n}^3 grid", 6_000_000)
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


def cpu_run(sc, g, src, dets, seconds, threads, seed, chunk):
    """The CPU restatement (oracle/, C, one photon stream per photon like the GPU) timed on
    `threads` host cores for about `seconds` of wall time: threads pull `chunk`-photon chunks
    of the same workload (ctypes releases the GIL), so the sample is photons [0, n). Returns
    the baseline object and the CPU tallies of photons [0, n)."""
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
    base = {"value": n / dt, "unit": "photon packets/s", "cores": threads, "kind": "port",
            "sample": f"photons [0,{n}) of the same workload, oracle/ C restatement (gcc -O2) on {threads} host "
                      f"thread{'s' if threads > 1 else ''} for {dt:.1f} s",
            "seconds": round(dt, 2)}
    return base, res


def compare_with_cpu(gpu, cpu):
    """The GPU's tallies of photons [0, n) against the CPU restatement's of the same photons."""
    import numpy as np
    fc, fg = cpu.normalised_fluence(), gpu.normalised_fluence()
    rmse = float(np.sqrt(np.mean((fg - fc) ** 2)))
    rel = float(np.max(np.abs(fg - fc)) / max(1e-300, float(np.max(np.abs(fc)))))
    agree = {"jmean_rmse_vs_cpu_same_photons": rmse, "jmean_max_rel_diff_vs_cpu": rel,
             "counters_bit_exact_vs_cpu": gpu.counters_dict() == cpu.counters_dict(),
             "photons_compared": cpu.n_photons}
    if cpu.det_bins.size > 1 or cpu.det_bins.any():
        db = float(np.max(np.abs(gpu.det_bins - cpu.det_bins)) / max(1e-300, float(np.max(np.abs(cpu.det_bins)))))
        agree["det_bins_max_rel_diff_vs_cpu"] = db
    return agree


def cpu_baseline(sc, g, src, dets, seconds, eng, threads, seed, chunk):
    """cpu_run, then (with an engine) the GPU runs exactly photons [0, n) and its fluence,
    counters and detector bins are compared with the CPU's."""
    base, res = cpu_run(sc, g, src, dets, seconds, threads, seed, chunk)
    if eng is None:
        return base, None
    return base, compare_with_cpu(eng.run(src, res.n_photons, seed=seed), res)


def sharded_cpu_parity(rank, world, cpu_leg, broadcast, sharded_gpu_run):
    """The CPU leg and the GPU-vs-port parity of an N-rank bench line (after the timed region).
    Rank 0 times the CPU restatement on photons [0, n) (cpu_leg() -> (baseline, CPU Result));
    n reaches every rank (broadcast); every rank runs its share [r n / N, (r+1) n / N) of the
    SAME photons and the shares are summed over the ranks by the engine's packed RCCL reduce
    (sharded_gpu_run(first, count) -> the summed Result on rank 0, None elsewhere); rank 0
    compares the sum with the CPU's tallies. Returns (baseline, parity) on rank 0, else
    (None, None). The reference means to sum its ranks' tallies with mpi_reduce
    (kernelsMod.f90:2351-2357)."""
    base = cpu = None
    n = 0
    if rank == 0:
        base, cpu = cpu_leg()
        n = cpu.n_photons
    n = int(broadcast(n))
    lo, hi = rank * n // world, (rank + 1) * n // world
    gpu = sharded_gpu_run(lo, hi - lo)
    if rank != 0:
        return None, None
    gpu.n_photons = n
    agree = compare_with_cpu(gpu, cpu)
    agree["gpu_side"] = (f"photons [0,{n}) split over {world} ranks, each rank its share, summed with the "
                         f"engine's one packed RCCL reduce (smcrt_reduce_device_tallies) onto rank 0")
    return base, agree


def attach_cpu_leg(out, base, agree, rccl_ranks=None):
    """The CPU leg's fields of the bench line: the baseline, the GPU-vs-port parity and, for
    N > 1 ranks, the rank count of the RCCL communicator that summed the GPU side."""
    out["cpu_baseline"] = base
    out["parity"] = agree
    if rccl_ranks is not None:
        out["rccl_ranks"] = rccl_ranks
    return out


def rank_row(rank, photons, seconds, transport_s, reduce_ms):
    """One rank's line of an N > 1 bench line's `ranks` breakdown: the photons it ran in the
    timed region, its wall seconds (barrier to barrier), its transport seconds (HIP events on
    its launch stream from the start of the timed region to the end of its last fold) and the
    packed RCCL reduce's own time (HIP events around smcrt_reduce_device_tallies)."""
    return {"rank": int(rank), "photons": int(photons), "seconds": float(seconds),
            "transport_s": float(transport_s), "reduce_ms": float(reduce_ms),
            "photons_per_s_transport": float(photons) / transport_s if transport_s > 0 else None}


def attach_rank_breakdown(out, rows):
    """Rank 0's summary of every rank's row (rank_row): the rows in rank order, the slowest
    rank's transport time, the reduce's largest time and the spread of transport times, so a
    non-linear scaling curve can be read from the line (transport imbalance vs collective
    cost). The reference's intended reduce is mpi_reduce to rank 0 (kernelsMod.f90:2351-2357)."""
    rows = sorted(rows, key=lambda r: r["rank"])
    ts = [r["transport_s"] for r in rows]
    out["ranks"] = rows
    out["rank_summary"] = {
        "photons_total": sum(r["photons"] for r in rows),
        "transport_s_max": max(ts), "transport_s_min": min(ts),
        "transport_imbalance": (max(ts) / min(ts) - 1.0) if min(ts) > 0 else None,
        "slowest_rank": rows[ts.index(max(ts))]["rank"],
        "reduce_ms_max": max(r["reduce_ms"] for r in rows),
        "reduce_share_of_step_time": (max(r["reduce_ms"] for r in rows) * 1e-3 / max(r["seconds"] for r in rows)),
    }
    return out


def sharded_device_run(eng, comm, src, g, dets, flags, seed, first, count, stream, rank):
    """One rank's share [first, first + count) of a photon range into fresh device tallies,
    then ONE packed RCCL reduce of every rank's tallies onto rank 0 (smcrt_reduce_device_tallies);
    rank 0 gets the summed tallies as a host Result."""
    import torch
    from rsmcrt_amd import abi
    from rsmcrt_amd.engine import Engine
    from rsmcrt_amd.tallies import Result
    dev = torch.device("cuda", torch.cuda.current_device())
    res = Result(g, dets)
    nv = g.nx * g.ny * g.nz
    t = {k: torch.zeros(nv, dtype=torch.float64, device=dev) for k in ("jmean", "absorb", "emission")}
    t["det_bins"] = torch.zeros(len(res.det_bins), dtype=torch.float64, device=dev)
    t["nscatt"] = torch.zeros(1, dtype=torch.float64, device=dev)
    t["counters"] = torch.zeros(abi.NCOUNTERS, dtype=torch.int64, device=dev)
    dt = abi.DeviceTallies()
    for k, v in t.items():
        if k != "det_bins" or dets:
            setattr(dt, k, v.data_ptr())
    if count > 0:
        eng.run_device(src, Engine.config(count, seed=seed, flags=flags, first_photon=first), dt, stream.cuda_stream)
    eng.fence(stream.cuda_stream)
    eng.reduce_device_tallies(comm, dt, root=0, stream=stream.cuda_stream)
    torch.cuda.synchronize()
    if rank != 0:
        return None
    shape = (g.nz, g.ny, g.nx)
    res.jmean[...] = t["jmean"].cpu().numpy().reshape(shape)
    res.absorb[...] = t["absorb"].cpu().numpy().reshape(shape)
    res.emission[...] = t["emission"].cpu().numpy().reshape(shape)
    if dets:
        res.det_bins[...] = t["det_bins"].cpu().numpy()
    res.nscatt[...] = t["nscatt"].cpu().numpy()
    res.counters[...] = t["counters"].cpu().numpy().astype("uint64")
    return res


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


# fp64 operations (add/sub, mul, div, sqrt; abs/min/max not counted) of one evaluation of each
# SDF primitive as geometry.h writes it (sdfs.f90:494-735), of its transform (translation
# only: 3 adds; general vec_dot_mat: 9 mul + 9 add) and of each CSG fold (sdfModifiers.f90)
SDF_FLOP = {1: 7, 2: 10, 3: 12, 4: 45, 5: 6, 6: 29, 7: 30, 8: 50, 9: 20, 10: 5}
CSG_FLOP = {0: 0, 1: 8, 2: 1, 3: 1}
FP64_PEAK_TFLOPS = 78.6  # MI355X fp64 vector, spec


def flop_per_eval(sc):
    """fp64 FLOP of one evaluation of the whole SDF array (every top, models folded)."""
    tot = 0
    for t in sc.top:
        nd = sc.nodes[t]
        kids = [nd] if nd.kind != 11 else [sc.nodes[nd.first_child + c] for c in range(nd.n_children)]
        for i, c in enumerate(kids):
            tr = list(c.transform)
            ident = tr[0] == 1 and tr[5] == 1 and tr[10] == 1 and not any(tr[k] for k in (1, 2, 4, 6, 8, 9))
            tot += SDF_FLOP.get(c.kind, 0) + (3 if ident else 18)
            if nd.kind == 11 and i > 0:
                tot += CSG_FLOP.get(nd.op, 0)
    return tot


def fp64_roofline(sc, sdf_evals_per_launch, kern_ms):
    """the SDF march's fp64 FLOP/s = SDF evaluations (packet%cnts, device
    counter) x FLOP per evaluation, over the transport kernel's launch time."""
    n_top = max(1, len(sc.top))
    flop = sdf_evals_per_launch / n_top * flop_per_eval(sc)
    ach = flop / (kern_ms * 1e-3) / 1e12
    return {"bound": "fp64-valu", "achieved": ach, "peak": FP64_PEAK_TFLOPS, "unit": "TFLOP/s",
            "frac": ach / FP64_PEAK_TFLOPS, "sdf_flop_per_launch": flop, "flop_per_array_eval": flop_per_eval(sc)}


# Issue cycles per wave64 VALU instruction on one SIMD, measured on MI355X with 3 waves per
# SIMD and 8 independent chains (tools/microbench/valu_rates.hip, profiles/r04_s1/valu_rates.txt:
# v_add_u32 / v_xor_b32 / v_mul_f32 3.2, fp64 add/mul/fma 5.1, v_rcp_f64 16.8, v_mad_u64_u32 7.7;
# round 3 assumed 2 cycles for 32-bit ops, which under-stated the utilisation)
VALU_CYCLES = {"f64_addmulfma": 5.1, "f64_trans": 16.8, "int64": 7.7, "other_32bit": 3.2}
SIMDS, CLOCK_HZ = 1024, 2.4e9


def valu_roofline(pmc, kern_ms):
    """VALU issue utilisation of the transport kernel from the PMC instruction mix of the
    committed profile of this configuration: sum over classes of (instructions x issue
    cycles) / (1024 SIMDs x 2.4 GHz x the live launch time)."""
    tot = pmc.get("valu_insts_per_launch")
    if not tot:
        return None
    cls = pmc.get("valu_classes") or {}
    f64 = sum(cls.get(k, 0.0) for k in ("SQ_INSTS_VALU_ADD_F64", "SQ_INSTS_VALU_MUL_F64", "SQ_INSTS_VALU_FMA_F64"))
    tr = cls.get("SQ_INSTS_VALU_TRANS_F64", 0.0)
    i64 = cls.get("SQ_INSTS_VALU_INT64", 0.0)
    rest = max(0.0, tot - f64 - tr - i64)
    mix = {"f64_addmulfma": f64, "f64_trans": tr, "int64": i64, "other_32bit": rest}
    cycles = sum(mix[k] * VALU_CYCLES[k] for k in mix)
    avail = SIMDS * CLOCK_HZ * kern_ms * 1e-3
    return {"bound": "valu-issue", "achieved": cycles / avail, "peak": 1.0, "unit": "fraction of SIMD issue cycles",
            "frac": cycles / avail, "valu_insts_per_launch": tot, "mix": mix, "issue_cycles": VALU_CYCLES,
            "salu_insts_per_launch": pmc.get("salu_insts_per_launch"), "source": pmc.get("source")}


def reference_pinned(device):
    """Spatial tallies of the HIP path against targets the reference itself holds (labelled
    reference-pinned, separate from the GPU == port parity above; tests/test_reference_targets.py
    holds the acceptance rules): the RI-mismatch absorb-depth fits of
    tools/validateRIMismatch.py:28-46 (res/validation2.toml, validation3.toml, 1e6 photons)
    and the fibre collection efficiency of tools/validateFibreDect.py:25 (1e6 photons)."""
    import numpy as np
    from rsmcrt_amd import scene as S
    from rsmcrt_amd.engine import Engine
    from rsmcrt_amd.job import Job
    from tests import refval
    with open(os.path.join(ROOT, "tests", "golden", "reference_kats.json")) as f:
        kats = json.load(f)
    out = {}

    def job_scene(j):
        sc = S.Scene([])
        sc.nodes = [j.nodes[i] for i in range(j.desc.n_nodes)]
        sc.top = list(j.top[:j.desc.n_top])
        return sc

    for which in ("validation2", "validation3"):
        j = Job(os.path.join(ROOT, "tests", "golden", "res", f"{which}.toml"))
        d = j.desc
        g = S.grid(5, 5, d.grid.nz, d.grid.xmax, d.grid.ymax, d.grid.zmax)
        with Engine(job_scene(j), g, device=device) as eng:
            r = eng.run(d.source, d.n_photons, seed=d.seed)
        sums = r.absorb.sum(axis=(1, 2))
        dz = 2 * g.zmax / g.nz
        depths, fit = refval.ri_fit(kats, which)
        sim = refval.to_reference_units(sums, d.n_photons, dz)
        sig = refval.to_reference_units(np.sqrt(np.maximum(sums, 1.0)), d.n_photons, dz)
        ok, rep = refval.compare_profile(sim, fit, depths, sig, refval.model_term(which))
        out[f"{which}_absorb_depth_vs_fit"] = {"photons": d.n_photons, "rel_rms": rep["rel_rms"],
                                               "integral_ratio": rep["integral_ratio"], "bins": rep["bins"],
                                               "model_term": refval.model_term(which),
                                               "model_term_note": refval.MODEL_TERM_NOTE,
                                               "bins_outside_4sigma_plus_model": len(rep["failed"]), "pass": ok}
    j = Job(os.path.join(ROOT, "tests", "golden", "res", "validateFibreDect.toml"))
    d = j.desc
    g = S.grid(20, 20, 20, d.grid.xmax, d.grid.ymax, d.grid.zmax)
    with Engine(job_scene(j), g, j.detectors, device=device) as eng:
        r = eng.run(d.source, d.n_photons, seed=d.seed)
    a, p = refval.fibre_expected(kats)
    eff = np.array([r.detector(i).sum() / d.n_photons for i in range(10)])
    ok, z = refval.fibre_check(eff, p, d.n_photons)
    out["fibre_collection_efficiency"] = {"photons": d.n_photons, "max_abs_z": float(np.max(np.abs(z))),
                                          "max_rel_err": float(np.max(np.abs(eff - p) / p)), "pass": ok}
    out["source"] = "tools/validateRIMismatch.py:28-46, tools/validateFibreDect.py:25 (reference_kats.json)"
    return out


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
        # warm-up at the timed size: the record pool is sized (and allocated) outside the
        # timed call, as every other workload's warm-up steps do
        eng.escape(c, photons, source=d.source, seed=d.seed)
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
    ap.add_argument("--gpus", type=int, default=None,
                    help="GPUs (one rank each). Without a launcher, bench.py starts the ranks itself "
                         "(rsmcrt_amd/launch.py); under torch.distributed.run it must equal WORLD_SIZE")
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--workload", default="m1", choices=WORKLOADS)
    ap.add_argument("--batch", type=int, default=0, help="photons per step per GPU (0 = workload default; "
                                                        "escape: photons per cell)")
    ap.add_argument("--grid", type=int, default=0, help="grid cells per axis (0 = workload default)")
    ap.add_argument("--seed", type=int, default=123456789)
    ap.add_argument("--cpu-seconds", type=float, default=12.0)
    ap.add_argument("--cpu1-seconds", type=float, default=8.0, help="the 1-core CPU leg (0 = skip)")
    ap.add_argument("--cpu-threads", type=int, default=0, help="0 = this process's CPU share, <= 16")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-ref", action="store_true", help="skip the reference-pinned spatial checks")
    ap.add_argument("--no-deposit", action="store_true", help="diagnostic: pathlength deposition off")
    ap.add_argument("--sync-fold", action="store_true", help="diagnostic: each step waits for its own fold")
    ap.add_argument("--overlap", type=int, default=1, choices=(0, 1),
                    help="1: steps rotate over the scene's internal streams (SMCRT_FLAG_OVERLAP: up to four, two "
                         "with record pools above 24 GiB), so a "
                         "step's slowest photons finish beside the next step")
    ap.add_argument("--source", default="default", choices=["default", "uniform"],
                    help="diagnostic: uniform = parallelogram source over the z=0.99 plane")
    ap.add_argument("--no-dets", action="store_true", help="diagnostic: the workload's scene without its detectors")
    ap.add_argument("--esc-nr", type=int, default=20)
    ap.add_argument("--esc-nz", type=int, default=10)
    args = ap.parse_args()

    from rsmcrt_amd import launch
    if not launch.under_launcher():
        gpus = 1 if args.gpus is None else args.gpus
        if gpus != 1:
            # no launcher: start one rank per GPU here, before anything touches the GPU
            if args.workload == "escape":
                log("[bench] the escape workload runs on one GPU; drop --gpus")
                sys.exit(2)
            try:
                rc = launch.spawn(gpus, [sys.executable, os.path.abspath(__file__), *sys.argv[1:]])
            except launch.LaunchError as e:
                log(f"[bench] {e}")
                sys.exit(2)
            sys.exit(rc)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if args.gpus is not None and args.gpus != world:
        log(f"[bench] --gpus {args.gpus} but the launcher started WORLD_SIZE={world} ranks")
        sys.exit(2)

    if args.workload == "escape":
        if world != 1:
            log("[bench] the escape workload runs on one GPU")
            sys.exit(2)
        escape_bench(args)
        return

    import torch
    import torch.distributed as dist

    ngpu = torch.cuda.device_count()
    if local >= ngpu:
        log(f"[bench] rank {rank} wants GPU {local} but only {ngpu} GPUs are visible")
        sys.exit(2)
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", rank=rank, world_size=world)
        assert dist.get_world_size() == world
    else:
        torch.cuda.set_device(0)
    dev = torch.device("cuda", torch.cuda.current_device())

    from rsmcrt_amd import abi, shard
    from rsmcrt_amd.engine import Comm, Engine

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
    if args.overlap:
        run_flags |= abi.FLAG_OVERLAP
    eng = Engine(sc, g, dets, device=torch.cuda.current_device())
    comm = None
    if world > 1:
        # the engine's own RCCL communicator (smcrt_comm_init_rank): rank 0's id reaches the
        # other ranks through the torch process group, then libsmcrt reduces its tallies
        uid = [Comm.unique_id() if rank == 0 else None]
        dist.broadcast_object_list(uid, src=0)
        comm = Comm(uid[0], world, rank, torch.cuda.current_device())
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
        dist.all_reduce(c0)  # (the timed reduce sums `counters` over ranks: subtract the sum)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    # HIP events on `stream` (torch's current stream, where the steps, the fence and the
    # reduce are enqueued): start, end of the last fold, end of the reduce
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
    t0 = time.perf_counter()
    ev[0].record(stream)
    for s in range(args.warmup, args.warmup + args.steps):
        step(s)
    eng.fence(stream.cuda_stream)
    ev[1].record(stream)
    if comm is not None:  # ONE packed RCCL all-reduce of every tally, inside libsmcrt
        eng.reduce_device_tallies(comm, dt_, root=-1, stream=stream.cuda_stream)
    ev[2].record(stream)
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    if world > 1:
        dist.barrier()
    mine = torch.tensor([t1 - t0], dtype=torch.float64, device=dev)
    per_rank = [mine.clone() for _ in range(world)]
    if world > 1:
        dist.all_gather(per_rank, mine)
    per_rank_s = [float(x.item()) for x in per_rank]
    elapsed = max(per_rank_s)  # the max over ranks
    eng.check()  # (after the timed region) the watchdog of every timed launch: a fault fails the line
    rows = None
    if world > 1:  # every rank's photons, transport time and reduce time (rank_row)
        mine_row = rank_row(rank, args.steps * B, t1 - t0, ev[0].elapsed_time(ev[1]) * 1e-3, ev[1].elapsed_time(ev[2]))
        rows = [None] * world
        dist.all_gather_object(rows, mine_row)
    log(f"[bench] {args.workload}: {args.steps} timed steps in {elapsed:.2f} s")
    kt = eng.kernel_times()  # HIP events around each kernel group, on the launch stream
    eng.set_timing(False)
    ms_per_step = elapsed * 1e3 / args.steps
    launches = kt["launches"]
    kern_ms = kt["transport_ms"] / launches if launches > 0 else 0.0
    dep_ms = kt["deposit_ms"] / launches if launches > 0 else 0.0
    timing_src = "HIP events around each transport launch (smcrt_scene_kernel_times)"
    if not kern_ms > 0.0:  # no launch was timed: fall back to the wall time per step (flagged)
        launches = max(1, launches)
        kern_ms = ms_per_step * args.steps / launches
        timing_src = "FALLBACK: wall time per step (the event timing returned no launches)"
    cdelta = (counters - c0).cpu().numpy()  # all ranks, timed steps only
    photons = world * args.steps * B

    out = None
    if rank == 0:
        per_rank = 1.0 / world  # (counters were summed over the ranks)
        deposits = float(cdelta[abi.CTR["deposits"]]) * per_rank  # per rank, over the timed steps
        dep_per_launch = deposits / launches
        # algorithmic HBM bytes of the transport kernel: 8 B per jmean deposit (SURVEY.md
        # §8(d): the reference's fp32 read+write per atomic; here one 8-B deposit record)
        alg_bytes = 8.0 * dep_per_launch
        achieved = alg_bytes / (kern_ms * 1e-3) / 1e9
        pmc = pmc_summary(args.workload, B, g.nx)
        traffic, traffic_src = pmc.get("step_hbm_bytes_per_launch"), pmc.get("source")
        metric = "photon packets/sec (128^3 jmean grid, path-length deposition)"
        if args.workload != "m1" or g.nx != 128:
            metric = f"photon packets/sec ({args.workload}, {g.nx}x{g.ny}x{g.nz} jmean grid, path-length deposition)"
        sdf_evals = float(cdelta[abi.CTR["sdf_evals"]]) * per_rank
        out = {
            "metric": metric,
            "value": photons / elapsed,
            "unit": "photon packets/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": ms_per_step,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f64",
            "data": "synthetic (Philox photon streams; scenes from setupGeometry.f90 / SURVEY §8(d))",
            "rank_seconds": per_rank_s,
            "config": {"workload": desc,
                       "grid": [g.nx, g.ny, g.nz], "photons_per_step_per_gpu": B, "photons_timed": photons,
                       "parallelism": f"photon-index shards x{world}" + (
                           " + one packed RCCL all-reduce of the tallies in libsmcrt" if world > 1 else "")},
            # SURVEY §8(d)'s HBM view of the deposition: 8 B per jmean deposit (the reference's
            # fp32 read+write per atomic) / the transport kernel's launch time. `traffic` is the
            # PMC HBM bytes of the whole step (transport + deposit folds) per launch.
            "roofline": {"bound": "hbm", "achieved": achieved, "peak": 8000.0, "unit": "GB/s",
                         "frac": achieved / 8000.0, "traffic": traffic,
                         # the kernel the timed launches ran: the lean path's ws_kernel or
                         # transport_kernel (smcrt_kernel_times.lean_launches)
                         "kernel": "ws_kernel" if kt.get("lean_launches", 0) > 0 else "transport_kernel",
                         "avg_launch_ms": kern_ms, "timing": timing_src,
                         "launches_timed": launches,
                         "algorithmic_bytes_per_launch": alg_bytes,
                         "traffic_source": traffic_src,
                         "traffic_by_kernel": pmc.get("hbm_bytes_per_launch_by_kernel"),
                         "traffic_over_algorithmic": (traffic / alg_bytes) if traffic and alg_bytes else None,
                         "deposits_per_photon": deposits / (args.steps * B),
                         # the HIP-event interval from a launch's end to its fold's end: the fold
                         # kernels (bk_scan, bk_place, bk_reduce) wait for CU slots behind the next
                         # persistent launch, so this is mostly queueing, not fold work
                         "fold_interval_ms_per_launch": dep_ms,
                         # the fold's own work: bk_reduce's workgroup run times (in-kernel wall
                         # clock) summed and divided by the CU count, i.e. the whole-chip time the
                         # fold takes from the transport kernel per launch
                         "fold_cu_ms_per_launch": kt.get("fold_cu_ms", 0.0) / launches,
                         "wave_iterations_per_launch": float(cdelta[abi.CTR["wave_iters"]]) * per_rank / launches,
                         "sdf_evals_per_photon": sdf_evals / (args.steps * B),
                         # march steps the far-field march took: counted above as
                         # the reference's deposits and SDF evaluations, done without a record or a
                         # full EVAL
                         "far_march_steps_per_launch": kt.get("far_steps", 0) / launches,
                         "note": "the transport kernel is bound by fp64 VALU issue and divergence, not by "
                                 "HBM: see valu_roofline / fp64_roofline and DESIGN.md §4.2"},
            "fp64_roofline": fp64_roofline(sc, sdf_evals / launches, kern_ms),
            "valu_roofline": valu_roofline(pmc, kern_ms),
            "cpu_baseline": None,
        }
        if rows is not None:
            attach_rank_breakdown(out, rows)
    if not args.no_cpu:
        threads = args.cpu_threads or cpu_threads()
        chunk = max(50, min(2000, B // 1000))
        if rank == 0:
            log(f"[bench] CPU leg: {args.cpu_seconds} s on {threads} threads + {args.cpu1_seconds} s on 1 core")
        if world == 1:
            base, agree = cpu_baseline(sc, g, src, dets, args.cpu_seconds, eng, threads, args.seed, chunk)
        else:  # the same photons on every rank's GPU, summed by the engine's RCCL reduce
            def bcast(n):
                box = [n]
                dist.broadcast_object_list(box, src=0)
                return box[0]

            def sharded(first, count):  # (path-length deposition as the CPU leg, whatever the timed flags)
                return sharded_device_run(eng, comm, src, g, dets, abi.FLAG_PATHLENGTH, args.seed, first, count,
                                          stream, rank)

            base, agree = sharded_cpu_parity(
                rank, world, lambda: cpu_run(sc, g, src, dets, args.cpu_seconds, threads, args.seed, chunk),
                bcast, sharded)
        if rank == 0:
            attach_cpu_leg(out, base, agree, comm.n_ranks if world > 1 else None)
            if args.cpu1_seconds > 0:
                one, _ = cpu_baseline(sc, g, src, dets, args.cpu1_seconds, None, 1, args.seed, max(50, chunk // 8))
                out["cpu_baseline_1core"] = one
                out["gpu_over_cpu_1core"] = out["value"] / one["value"]
            out["gpu_over_cpu"] = out["value"] / base["value"]
    if rank == 0 and not args.no_ref:
        log("[bench] reference-pinned spatial checks (validation2/3 absorb depth, fibre efficiency)")
        out.setdefault("parity", {})["reference_pinned"] = reference_pinned(torch.cuda.current_device())
    if rank == 0:
        print(json.dumps(out), flush=True)
    eng.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
