"""Escape-function throughput: res/default.toml's scene and detectors
(a 50x62x64 scattering box, 11 annulus detectors) with its 360rotational symmetry on a
reduced symmetry grid. The GPU runs every launch cell in one batched launch
(smcrt_escape_run); the CPU restatement runs a sample of cells one run_MCRT at a time, as
the reference does, on --threads host threads (cells are independent), extrapolated to all
cells. Prints one JSON line.

usage: python tools/bench_escape.py [--nr 20] [--nz 10] [--photons 10000] [--cpu-cells 4]"""
import argparse
import json
import os
import sys
import threading
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402

from rsmcrt_amd import abi, escape, scene  # noqa: E402
from rsmcrt_amd.engine import Engine  # noqa: E402
from rsmcrt_amd.job import Job  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--nr", type=int, default=20)
ap.add_argument("--nz", type=int, default=10)
ap.add_argument("--photons", type=int, default=10000)
ap.add_argument("--cpu-cells", type=int, default=4)
ap.add_argument("--threads", type=int, default=4)
a = ap.parse_args()

j = Job(os.path.join(ROOT, "tests", "golden", "res", "default.toml"), mode="escape")
d = j.desc
c = j.escape_config()
c.n[0], c.n[2] = a.nr, a.nz  # 360rotational: nr x 1 x nz launch cells (reference: 100 x 200)
sc = scene.Scene([])
sc.nodes = [j.nodes[i] for i in range(d.n_nodes)]
sc.top = list(j.top[:d.n_top])
dets = j.detectors
idx, pos = escape.cells(c)
with Engine(sc, d.grid, dets) as eng:
    eng.escape(c, 200, source=d.source, seed=d.seed)  # warm-up (pool sizing)
    t0 = time.perf_counter()
    es, e, res = eng.escape(c, a.photons, source=d.source, seed=d.seed)
    t_gpu = time.perf_counter() - t0
    lay, kap = eng.classify(pos)
    run_cells = int(np.sum((lay != 0) & (kap != 0.0)))
    org = pos[(lay != 0) & (kap != 0.0)]
    t0 = time.perf_counter()
    tot, _ = eng.run_origins(org, a.photons, source=d.source, seed=d.seed)
    t_mc = time.perf_counter() - t0
t0 = time.perf_counter()
escape.map_to_grid(c, d.grid, es)
t_map = time.perf_counter() - t0

from oracle import pyoracle as O  # noqa: E402  (the CPU leg only)
sample = [i for i in range(len(pos)) if lay[i] != 0 and kap[i] != 0.0][:a.cpu_cells]
times = []
lock = threading.Lock()


def work(k):
    t = time.perf_counter()
    O.run(sc, d.grid, scene.point_source(tuple(pos[k])), a.photons, seed=d.seed, dets=dets)
    with lock:
        times.append(time.perf_counter() - t)


ths = [threading.Thread(target=work, args=(k,)) for k in sample]
for t in ths:
    t.start()
for t in ths:
    t.join()
per_cell = float(np.mean(times))
cpu_total = per_cell * run_cells / a.threads
print(json.dumps({
    "workload": "res/default.toml escape function, 360rotational, symmetry grid "
                f"{a.nr}x1x{a.nz} ({run_cells} cells run), {a.photons} photons per cell",
    "gpu_seconds": t_gpu, "gpu_photons_per_s": run_cells * a.photons / t_gpu,
    "batched_launch_seconds": t_mc, "host_map_seconds": t_map,
    "mc_speedup": per_cell * run_cells / a.threads / t_mc,
    "cpu_seconds_per_cell_per_thread": per_cell, "cpu_threads": a.threads,
    "cpu_seconds_extrapolated": cpu_total, "speedup": cpu_total / t_gpu,
    "scatters_per_photon": res.counter("scatters") / (run_cells * a.photons),
    "deposits_per_photon": res.counter("deposits") / (run_cells * a.photons),
    "escape_sym_max": float(es.max())}))
