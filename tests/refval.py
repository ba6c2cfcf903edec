"""Spatial tally targets the reference itself holds, restated for the tests.

* RI-mismatch absorb-depth profile, /root/reference/tools/validateRIMismatch.py:14-46: read
  absorb.nrrd of res/validation2.toml / validation3.toml, average every z slice over its x, y
  voxels, and compare with the tool's fit
      norm * (c1 exp((depth - 1.95) k1 / delta) - c2 exp((depth - 1.95) k2 / delta))
  on depth = linspace(-2, 2, nz), over the plotted range depths[-14] .. 1.6 (:26).
  The fit's `norm` belongs to the file's run: 1e6 photons and 250 x 250 x 1000 voxels of
  0.4 x 0.4 x 0.004 cm. A run with N photons, nx*ny voxels per slice and slices of dz is
  brought to those units by (sum over the slice) / 62500 * (0.004 / dz) * (1e6 / N).
* Fibre collection efficiency, tools/validateFibreDect.py:8-25: detector j of
  res/validateFibreDect.toml (front-lens aperture 0.5 j, focal length 2) collects
  sum(count)/nPackets = 0.5 (1 - cos(atan(a / 2))) of a point source at its front focal
  point; every ray through the lens reaches the fibre core, so the count is binomial.

The constants are data (tests/golden/reference_kats.json); the statistics are this file's.
"""
from __future__ import annotations

import numpy as np

REF_N, REF_XY, REF_DZ = 1_000_000, 250 * 250, 4.0 / 1000


def ri_fit(kats, which: str, nz: int = 1000):
    k = kats["ri_mismatch_absorb_depth"][which]
    depths = np.linspace(-2.0, 2.0, nz)
    fit = k["norm"] * (k["c1"] * np.exp((depths - 1.95) * k["k1"] / k["delta"])
                       - k["c2"] * np.exp((depths - 1.95) * k["k2"] / k["delta"]))
    return depths, fit


def plotted_range(depths):
    """validateRIMismatch.py:26: set_xlim([depths[-14], 1.6])."""
    return (depths >= 1.6) & (depths <= depths[-14])


def slice_sums(absorb_zyx):
    """Sum of each z slice of an (nz, ny, nx) absorb grid (the tool's mean over x, y times
    the voxels it averages)."""
    return np.asarray(absorb_zyx, dtype=np.float64).sum(axis=(1, 2))


def to_reference_units(sums, n_photons, dz):
    """Slice sums of a run -> the tool's mean-over-x,y units of the file's 1e6-photon run."""
    return sums / REF_XY * (REF_DZ / dz) * (REF_N / n_photons)


# An independent ceiling on the model term: the blanket 5 % of round 2, chosen before any
# calibration on the restatement. The measured per-target terms must stay below it.
MODEL_CEILING = 0.05
# The per-target term is calibrated on the CPU restatement itself, so a systematic bias of the
# restatement would be built into it: agreement within it is "parity unpinned", evidence only
# that the GPU equals the restatement and that neither drifted past the ceiling.
MODEL_TERM_NOTE = ("parity unpinned: the model term is calibrated on the CPU restatement "
                   "(tests/golden/ri_model_residual.json), capped by an independent 5 % ceiling")


def model_term(which: str) -> float:
    """The fit's own inaccuracy for target `which`, measured (not chosen): the largest
    |mean transport profile - fit| / fit over the tested bins, plus 3 standard errors, from 8
    seeds x 1e6 photons of the CPU restatement (tests/golden/make_ri_model_residual.py ->
    tests/golden/ri_model_residual.json): validation2 3.5 %, validation3 2.0 %. Never more
    than MODEL_CEILING (an AssertionError if the calibration ever claims more)."""
    import json
    import os
    p = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "ri_model_residual.json")
    with open(p) as f:
        m = float(json.load(f)[which]["model_term"])
    assert 0.0 <= m <= MODEL_CEILING, (which, m)
    return m


def compare_profile(sim, fit, depths, sigma, rel_model, k_sigma=4.0, rebin=5, floor=0.01):
    """Compare a simulated depth profile with the reference fit over the plotted range.

    The range is cut into bins of `rebin` slices (0.02 cm at the file's resolution). A bin
    passes if |sim - fit| <= k_sigma * sigma_MC + rel_model * fit, where sigma_MC is the
    Monte Carlo standard error of the bin (seed-to-seed, or Poisson counts) and rel_model the
    fit's own accuracy as a diffusion-theory fit of the transport result, measured per target
    (model_term). Bins whose fit is below `floor` x the profile's peak are not tested (noise
    only). Returns (ok, report)."""
    m = plotted_range(depths)
    idx = np.where(m)[0]
    nb = len(idx) // rebin
    idx = idx[len(idx) - nb * rebin:].reshape(nb, rebin)
    s = sim[idx].mean(axis=1)
    f = fit[idx].mean(axis=1)
    e = np.sqrt((sigma[idx] ** 2).sum(axis=1)) / rebin
    d = depths[idx].mean(axis=1)
    keep = f >= floor * f.max()
    bad = keep & (np.abs(s - f) > k_sigma * e + rel_model * f)
    rel_rms = float(np.sqrt(np.mean((sim[m] - fit[m]) ** 2)) / np.sqrt(np.mean(fit[m] ** 2)))
    integral = float(sim[m].sum() / fit[m].sum())
    rep = {"bins": int(keep.sum()), "failed": [(float(a), float(b), float(c), float(x)) for a, b, c, x, y in
                                               zip(d, s, f, e, bad) if y],
           "rel_rms": rel_rms, "integral_ratio": integral}
    return not bad.any(), rep


def fibre_expected(kats):
    k = kats["fibre_collection_efficiency"]
    a = np.array(k["apertures"])
    return a, 0.5 * (1.0 - np.cos(np.arctan(a / k["focal_length"])))


def fibre_check(eff, p, n, k_sigma=4.0):
    """Binomial acceptance: |eff - p| <= k_sigma sqrt(p (1 - p) / n) for every detector."""
    sig = np.sqrt(p * (1.0 - p) / n)
    z = (np.asarray(eff) - p) / sig
    return bool(np.all(np.abs(z) <= k_sigma)), z
