"""Measure the model term of the RI-mismatch profile checks (tests/refval.py): how far the
reference's diffusion-theory fit (tools/validateRIMismatch.py:28-46) lies from the transport
result itself, per 0.02-cm bin of the plotted range, with Monte Carlo noise made small.

Runs the CPU restatement (oracle/, test infrastructure) on res/validation2.toml and
res/validation3.toml for SEEDS independent seeds x PHOTONS photons (z binning of the file,
5 x 5 columns: the tool averages over x, y), averages the profiles, and writes per target
  * rel_resid[b]  = (mean_sim - fit) / fit per tested bin,
  * rel_sigma[b]  = the seed-to-seed standard error of that mean, relative to the fit,
  * model_term    = max over bins of (|rel_resid| + 3 rel_sigma), rounded up to 0.5 %:
                    the fit's own inaccuracy, which tests/refval.py adds to 4 sigma_MC;
to tests/golden/ri_model_residual.json. usage: python tests/golden/make_ri_model_residual.py
"""
import json
import os
import sys
import threading
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

SEEDS = int(os.environ.get("SEEDS", "8"))
PHOTONS = int(os.environ.get("PHOTONS", "1000000"))
THREADS = int(os.environ.get("THREADS", "8"))


def main():
    from oracle import pyoracle as O
    from rsmcrt_amd import scene
    from rsmcrt_amd.job import Job
    from rsmcrt_amd.tallies import Result
    from tests import refval
    kats = json.load(open(os.path.join(ROOT, "tests", "golden", "reference_kats.json")))
    out = {"_source": __doc__.strip().splitlines()[0], "seeds": SEEDS, "photons_per_seed": PHOTONS,
           "rebin": 5, "floor": 0.01}
    for which in ("validation2", "validation3"):
        j = Job(os.path.join(ROOT, "tests", "golden", "res", f"{which}.toml"))
        d = j.desc
        sc = scene.Scene([])
        sc.nodes = [j.nodes[i] for i in range(d.n_nodes)]
        sc.top = list(j.top[:d.n_top])
        g = scene.grid(5, 5, d.grid.nz, d.grid.xmax, d.grid.ymax, d.grid.zmax)
        dz = 2 * g.zmax / g.nz
        depths, fit = refval.ri_fit(kats, which)
        m = refval.plotted_range(depths)
        idx = np.where(m)[0]
        nb = len(idx) // 5
        idx = idx[len(idx) - nb * 5:].reshape(nb, 5)
        f = fit[idx].mean(axis=1)
        keep = f >= 0.01 * f.max()
        profs = []
        t0 = time.time()
        for s in range(SEEDS):
            per = PHOTONS // THREADS
            res = [Result(g, []) for _ in range(THREADS)]
            ths = [threading.Thread(target=lambda i=i: O.run(sc, g, d.source, per, seed=d.seed + 1000 * s,
                                                            first_photon=i * per, result=res[i]))
                   for i in range(THREADS)]
            for t in ths:
                t.start()
            for t in ths:
                t.join()
            r = res[0]
            for o in res[1:]:
                r.merge(o)
            sim = refval.to_reference_units(refval.slice_sums(r.absorb), per * THREADS, dz)
            profs.append(sim[idx].mean(axis=1))
            print(f"{which} seed {s}: {time.time() - t0:.0f} s", file=sys.stderr, flush=True)
        p = np.array(profs)
        mean = p.mean(axis=0)
        se = p.std(axis=0, ddof=1) / np.sqrt(SEEDS)
        rr = ((mean - f) / f)[keep]
        rs = (se / f)[keep]
        term = float(np.ceil(np.max(np.abs(rr) + 3.0 * rs) / 0.005) * 0.005)
        out[which] = {"depth": [float(x) for x in depths[idx].mean(axis=1)[keep]],
                      "rel_resid": [float(x) for x in rr], "rel_sigma": [float(x) for x in rs],
                      "max_abs_rel_resid": float(np.max(np.abs(rr))), "model_term": term}
        print(which, "max |resid|/fit", float(np.max(np.abs(rr))), "model term", term, file=sys.stderr)
    with open(os.path.join(ROOT, "tests", "golden", "ri_model_residual.json"), "w") as fh:
        json.dump(out, fh, indent=1)


if __name__ == "__main__":
    main()
