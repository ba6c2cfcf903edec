// far.h — the far-field march: a lone photon's long sphere-tracing run (tauint2's march
// loop, inttau2.f90:155-191) with only the nearest top-level SDF evaluated per step.
//
// Why. M2 (sphere_scene) starts photons on the whole top face of its box, going straight
// down. One whose x or y lies within δ of a side wall is sphere-traced with d = δ (the box's
// distance) for about 2/δ steps; over a 12.8 M-photon launch P(steps > s) ≈ 4/s, so the
// smallest δ is ~1e-7 and one photon marches up to the 10^7-step guard. The solo march
// (smcrt.hip) pays a cooperative EVAL of every top, a DDA crossing and a record per step
// for it, ≈2 µs, so that one photon sets the launch's length (≈20 s).
//
// What stays exact. A march step consumes only minval(abs(ds)) and minval(ds) (:177-191).
// After a full EVAL at p0 whose nearest top is k and whose other tops all have |ds_j| >= m2,
// each other top's true distance changes by at most the distance travelled (1-Lipschitz
// SDFs: spheres, boxes, capsules, segments and tori under translation-only transforms,
// checked by the host), and a computed value is within fm_err of the true one. So while
//     |ds_k(p)| + travel_ub < m2 - 2 fm_err
// every other computed |ds_j(p)| is larger than |ds_k(p)| and keeps its sign: minval(abs(ds))
// is exactly |ds_k(p)|, and minval(ds) > 0 iff ds_k(p) > 0 and no other top was negative at
// p0. travel_ub bounds |p - p0|: the sum of d |dir| (1 + 2^-48), plus fm_step per step for
// the rounding of p + d*dir and of the sum itself.
// A step's deposit segment (update_grids from p over d, :401-441) ends inside p's voxel iff
// each exact quotient (face - old)/dir exceeds d. The loop tests the quotient formed with the
// direction's reciprocal against d (1 + 2^-40), which implies it, and stops otherwise. Such a
// segment deposits real(d, sp)*weight into that voxel; the loop sums those in fp64 and adds
// the sum with one fp64 atomic when it stops (jmean then differs from per-step adds at
// rounding level, as the fold's order of adds already makes it).
// Everything else (the bound fails, the march would end, a voxel face, the optical depth,
// the march guard) stops the loop BEFORE that step, leaving the photon in the state the main
// loop's program points would have left it in: ST_M1 with an EVAL pending (redone in full),
// or ST_M0 with d = minabs = |ds_k(p)| (exact by the bound), so P4 takes the step.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "transport.h"

namespace smcrt {

// Start a certificate only for marches at least this long (the wave-wide minimum costs a
// few hundred cycles per full EVAL)
#ifndef SMCRT_FAR_MIN_LOOP
#define SMCRT_FAR_MIN_LOOP 8
#endif

// The far-field loop for near top k of kind KIND (SPHERE or BOX), run by the photon's lane
// alone. ct: the cooperative EVAL's LDS table; m2 / neg_other: the certificate of the full
// EVAL at p0; trav0: the distance from p0 to L.pos (the step P4 took after that EVAL).
// On entry L is at ST_M1 with an EVAL pending and no segment. Returns the steps taken; acc
// receives their deposits' sum for voxel *vox, nsdf the EVALs consumed.
template <int GM, int KIND>
__device__ __forceinline__ uint32_t far_march(const KParams& K, Lane& L, const double* ct, int k, double m2,
                                              bool neg_other, double trav0, double kap,
                                              const double* __restrict__ xf, const double* __restrict__ yf,
                                              const double* __restrict__ zf, double& acc, uint32_t& vox,
                                              uint32_t& nsdf) {
  const double eps = 1e-8;  // inttau2.f90:56
  double tl[12], pl[8];
#pragma unroll
  for (int r = 0; r < 12; ++r) tl[r] = ct[r * 64 + k];
#pragma unroll
  for (int r = 0; r < 8; ++r) pl[r] = ct[(12 + r) * 64 + k];
  const V3 dir = L.dir;
  const bool zx = dir.x == 0.0, zy = dir.y == 0.0, zz = dir.z == 0.0;
  // (the reciprocal-based test needs operands where the division does no scaling)
  if (!(zx || fabs(dir.x) >= 0x1.0p-500) || !(zy || fabs(dir.y) >= 0x1.0p-500) ||
      !(zz || fabs(dir.z) >= 0x1.0p-500))
    return 0;
  // the voxel of L.pos, as update_grids would find it (start_segment)
  const V3 o0 = v3(L.pos.x + K.xmax, L.pos.y + K.ymax, L.pos.z + K.zmax);
  const int32_t ci = cell_of<GM>(o0.x, K.nx, K.xmax, K.inv2x, K.fex),
                cj = cell_of<GM>(o0.y, K.ny, K.ymax, K.inv2y, K.fey),
                ck = cell_of<GM>(o0.z, K.nz, K.zmax, K.inv2z, K.fez);
  if (ci == -1 || cj == -1 || ck == -1) return 0;
  vox = lin(K, ci, cj, ck);
  // the walls wall_dist would measure from inside that voxel (dda_step_r)
  const double fx = face<GM>(xf, dir.x > 0.0 ? ci : ci - 1, K.fex);
  const double fy = face<GM>(yf, dir.y > 0.0 ? cj : cj - 1, K.fey);
  const double fz = face<GM>(zf, dir.z > 0.0 ? ck : ck - 1, K.fez);
  const double rx = zx ? 0.0 : ieee_rcp_f64(dir.x), ry = zy ? 0.0 : ieee_rcp_f64(dir.y),
               rz = zz ? 0.0 : ieee_rcp_f64(dir.z);
  const double dn = sqrt(dir.x * dir.x + dir.y * dir.y + dir.z * dir.z) * (1.0 + 0x1.0p-48);
  const double lim = m2 - 2.0 * K.fm_err;
  double trav = trav0 * dn + K.fm_step;
  const double w = L.weight;
  uint32_t n = 0;
  for (;;) {
    // ST_M1's EVAL (:177-191), the near top only
    const double v = sdf_prim_s<1>(KIND, tl, pl, L.pos, true);
    const double a = fabs(v);
    if (!(a + trav < lim)) break;           // the certificate no longer covers p (or NaN)
    if (v > 0.0 && !neg_other) break;       // outside every SDF: tflag, the march ends
    if (!(a >= eps)) break;                 // the march loop ends (:155)
    ++nsdf;                                 // P3 consumed the EVAL: d = minabs = a
    // P4 (:155-176): the step is taken here only if it is an interior one
    bool go = L.loopc + 1u <= (uint32_t)MAX_MARCH_ITERS;
    const double t = a * kap;
    go = go && L.taurun + t < L.tau;
    const V3 old = v3(L.pos.x + K.xmax, L.pos.y + K.ymax, L.pos.z + K.zmax);
    go = go && cell_of<GM>(old.x, K.nx, K.xmax, K.inv2x, K.fex) == ci &&
         cell_of<GM>(old.y, K.ny, K.ymax, K.inv2y, K.fey) == cj && cell_of<GM>(old.z, K.nz, K.zmax, K.inv2z, K.fez) == ck;
    const double lo = a * (1.0 + 0x1.0p-40);
    go = go && a < 100000.0 && (zx || (fx - old.x) * rx > lo) && (zy || (fy - old.y) * ry > lo) &&
         (zz || (fz - old.z) * rz > lo);
    if (!go) {  // P4 takes this step in the main loop
      L.minabs = a;
      L.d = a;
      L.st = ST_M0;
      L.pend = false;
      break;
    }
    L.taurun = L.taurun + t;
    L.pos = L.pos + smul(a, dir);
    ++L.loopc;
    acc = acc + (double)(float)a * w;  // jmean(cell) += real(dcell, sp) * weight (:427)
    ++n;
    trav = trav + (a * dn + K.fm_step);
  }
  return n;
}

// Wave minimum of v (every lane active), by the cooperative EVAL's DPP row scans.
__device__ __forceinline__ double wave_min_f64(double v) {
  double b;
  b = dpp_f64<0x111, 0xf>(__builtin_inf(), v); v = b < v ? b : v;
  b = dpp_f64<0x112, 0xf>(__builtin_inf(), v); v = b < v ? b : v;
  b = dpp_f64<0x114, 0xf>(__builtin_inf(), v); v = b < v ? b : v;
  b = dpp_f64<0x118, 0xf>(__builtin_inf(), v); v = b < v ? b : v;
  b = dpp_f64<0x142, 0xa>(__builtin_inf(), v); v = b < v ? b : v;
  b = dpp_f64<0x143, 0xc>(__builtin_inf(), v); v = b < v ? b : v;
  return readlane_f64(v, 63);
}

}  // namespace smcrt
