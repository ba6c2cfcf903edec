// inverse.cpp — the inverse-MCRT driver (kernelsMod.f90:1462-1787, the -DinverseMCRT build)
// on a resident scene. Host code only; part of libsmcrt.so.
//
// The reference reruns run_MCRT once per step, re-uploading nothing because its scene is
// host memory; here the scene stays on the GPU and a step changes one TopProps entry
// (smcrt_scene_set_optprops) before its run. The guesses come from a host Philox4x32-10
// stream keyed by cfg->seed: the reference draws them from its global ran2 between runs,
// a stream no other implementation can reproduce.
#include <cmath>
#include <cstring>
#include <vector>

#include "../../include/smcrt.h"
#include "hosterr.h"
#include "hostrng.h"
#include "scene_internal.h"

using smcrt::set_error;

// The guess stream: draw d is the (d & 1) half of block (d >> 1, 1, 0, 0xFFFFFFFF) under
// the run's key (hostrng.h), a counter no photon stream uses.

extern "C" {

int smcrt_inverse_run(smcrt_scene* scene, const smcrt_source* src, const smcrt_inverse_config* cfg,
                      const smcrt_run_config* run, const double* targets, double* steps, smcrt_tallies* io) {
  if (!scene || !src || !cfg || !run || !steps) return set_error(SMCRT_ERR_INVALID_ARG, "NULL argument");
  if (cfg->max_steps < 1) return set_error(SMCRT_ERR_INVALID_ARG, "maxNumSteps must be >= 1");
  if (run->n_photons == 0) return set_error(SMCRT_ERR_INVALID_ARG, "n_photons must be > 0");
  const bool fmus = cfg->flags & SMCRT_INVERSE_FIND_MUS, fmua = cfg->flags & SMCRT_INVERSE_FIND_MUA,
             fg = cfg->flags & SMCRT_INVERSE_FIND_G, fn = cfg->flags & SMCRT_INVERSE_FIND_N;
  if (!fmus && !fmua && !fg && !fn)  // :1556-1559
    return set_error(SMCRT_ERR_INVALID_ARG, "Please select at least one of mus, mua, hgg, n to find with inverse MCRT");
  smcrt_grid g;
  int32_t n_top = 0, nd = 0;
  int st = smcrt_scene_info(scene, &g, &n_top, &nd);
  if (st) return st;
  if (nd > 0 && !targets) return set_error(SMCRT_ERR_INVALID_ARG, "targets is NULL");
  // the first SDF of the selected layer and its properties, :1562-1578
  int32_t idx = -1;
  double mus = 0, mua = 0, hgg = 0, n = 0;
  for (int32_t i = 0; i < n_top && idx < 0; ++i) {
    int32_t layer = 0;
    if ((st = smcrt_scene_get_optprops(scene, i, &layer, &mus, &mua, &hgg, &n))) return st;
    if (layer == cfg->layer) idx = i;
  }
  if (idx < 0)  // :1581-1584
    return set_error(SMCRT_ERR_INVALID_ARG, "Selected layer not found in SDF array please choose a layer inside the SDF array");
  double orig[4];  // the node's stored values and flags, restored at the end
  int32_t orig_flags = 0;
  if ((st = smcrt::scene_node_optprops(scene, idx, orig))) return st;
  if ((st = smcrt::scene_node_flags(scene, idx, &orig_flags))) return st;

  // AdaLIPO bounds, :1588-1602
  const double musl = 0.0, musu = 100.0, mual = 0.0, muau = 100.0, gl = -1.0, gu = 1.0, nl = 1.0, nu = 20.0;
  smcrt::HostStream R{(uint32_t)cfg->seed, (uint32_t)(cfg->seed >> 32), smcrt::STREAM_INVERSE};
  const int64_t M = cfg->max_steps;
  const bool apply = cfg->flags & SMCRT_INVERSE_APPLY_TRIAL;
  std::vector<double> bins;
  int64_t nb = 0;
  if ((st = smcrt_scene_det_bins(scene, &nb))) return st;
  int changed = 0;
  // A step is a deterministic function of the layer's properties (every run restarts the
  // same photon streams, :1850): a step whose properties repeat an earlier step's bits has
  // that step's error. In the reference's own mode every step after the first reruns one
  // scene (:1630-1631), so this turns maxNumSteps runs into two.
  struct Memo {
    double p[4];
    double err;
  };
  std::vector<Memo> memo;
  double cur[4] = {orig[0], orig[1], orig[2], orig[3]};  // the properties the scene holds
  for (int64_t i = 1; i <= M && !st; ++i) {
    if (i >= 2) (void)R.next();  // ran = ran2(): always <= 1, the explore branch (:1620-1622)
    double* row = steps;
    row[(0) * M + (i - 1)] = fmus ? R.next() * (musu - musl) + musl : mus;
    row[(1) * M + (i - 1)] = fmua ? R.next() * (muau - mual) + mual : mua;
    row[(2) * M + (i - 1)] = fg ? R.next() * (gu - gl) + gl : hgg;
    row[(3) * M + (i - 1)] = fn ? R.next() * (nu - nl) + nl : n;
    double want[4] = {cur[0], cur[1], cur[2], cur[3]};
    if (apply) {
      want[0] = row[i - 1]; want[1] = row[M + i - 1]; want[2] = row[2 * M + i - 1]; want[3] = row[3 * M + i - 1];
    } else if (i >= 2) {
      // trialOptProp = mono(mus, mua, hgg, n) from the original getters (:1630-1631)
      want[0] = mus; want[1] = mua; want[2] = hgg; want[3] = n;
    }
    bool hit = false;
    // (with caller tallies every step runs, so `io` accumulates maxNumSteps runs as the
    // reference's jmean does over its run_MCRT calls)
    if (!io)
      for (const Memo& m : memo)
        if (std::memcmp(m.p, want, sizeof want) == 0) {
          row[4 * M + (i - 1)] = m.err;
          hit = true;
          break;
        }
    if (hit) continue;
    if (std::memcmp(want, cur, sizeof cur) != 0) {
      st = smcrt_scene_set_optprops(scene, idx, want[0], want[1], want[2], want[3]);
      if (st) break;
      std::memcpy(cur, want, sizeof cur);
      changed = 1;
    }
    bins.assign((size_t)std::max<int64_t>(nb, 1), 0.0);
    smcrt_tallies t;
    if (io) t = *io;
    else std::memset(&t, 0, sizeof t);
    t.det_bins = bins.data();
    t.records = nullptr;
    st = smcrt_run(scene, src, run, &t);
    if (st) break;
    // inverse_evaluate, :1753-1787
    double err = 0.0;
    int counter = 0;
    int64_t off = 0;
    for (int32_t d = 0; d < nd; ++d) {
      int64_t sz = 0;
      if ((st = smcrt::scene_det_size(scene, d, &sz))) break;
      if (targets[d] != -1) {
        double total = 0.0;
        for (int64_t b = 0; b < sz; ++b) total = total + bins[(size_t)(off + b)];
        total = total / (double)run->n_photons;
        err = err + std::fabs((total - targets[d]));
        counter = counter + 1;
      }
      off += sz;
    }
    if (st) break;
    row[4 * M + (i - 1)] = -err / counter;
    Memo m;
    std::memcpy(m.p, cur, sizeof cur);
    m.err = row[4 * M + (i - 1)];
    memo.push_back(m);
  }
  if (changed) {  // restore the layer
    const int rst = smcrt::scene_set_node_props(scene, idx, orig[0], orig[1], orig[2], orig[3], orig_flags);
    if (!st) st = rst;
  }
  return st;
}

}  // extern "C"
