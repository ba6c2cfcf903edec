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
//
// Strides. M2's long photons move along one axis (the source's direction (0,0,-1)) next to a
// face of the bounding box, so the near top is that box and its distance comes from another
// axis: d is the same number at every step, and each step is p_m <- RN(p_m + s) with s =
// RN(d*dir_m) constant, taurun <- RN(taurun + t) with t = RN(d*kappa) constant. While p_m
// stays inside one binade [2^e + u, 2^(e+1) - u] (u its ulp), every such sum rounds by the
// same amount unless s sits exactly halfway between multiples of u: p_m after k steps is
// p_m + k*D exactly, D = RN(p_m + s) - p_m (and likewise taurun). box_stride takes K steps at
// once when every per-step condition above holds for all of them: each one is monotone along
// the run (the sums are monotone, RN is monotone, |x| is convex), so it is checked exactly
// at the run's first and last step, on the very values those steps compute. The deposits
// are K times real(d, sp)*weight (one product into the fp64 sum). A photon near the 10^7
// step guard then costs a few hundred strides (binades, voxels, certificates) instead of
// 10^7 steps.
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

__device__ __forceinline__ double axis_of(V3 v, int m) { return m == 0 ? v.x : (m == 1 ? v.y : v.z); }

// The binade run of x <- RN(x + s) from x0 (see Strides): D and the range [xmin, xmax] every
// value of the run must stay in. false: x0 is zero or not normal, or s is a rounding tie.
__device__ __forceinline__ bool binade_run(double x0, double s, double& D, double& xmin, double& xmax) {
  const double m = fabs(x0);
  if (!(m >= 0x1.0p-1000) || !(m <= 0x1.0p+1000)) return false;
  const int e = ilogb(m);
  const double lo = ldexp(1.0, e), u = ldexp(1.0, e - 52);
  D = (x0 + s) - x0;  // (exact when x0 + s stays in the binade; otherwise the range check fails)
  if (fabs(s - D) == 0.5 * u) return false;
  const double a0 = lo + u, a1 = 2.0 * lo - u;
  if (x0 > 0.0) { xmin = a0; xmax = a1; } else { xmin = -a1; xmax = -a0; }
  return true;
}
// steps k >= 0 for which x0 + k*D stays in [xmin, xmax] (a large number when D == 0)
__device__ __forceinline__ double run_len(double x0, double D, double xmin, double xmax) {
  if (D > 0.0) return floor((xmax - x0) / D);
  if (D < 0.0) return floor((xmin - x0) / D);
  return 0x1.0p+40;
}

// One stride of K >= 2 march steps along axis m from L.pos (BOX near top, see Strides); the
// EVAL at L.pos gave v (a = |v|) and passed the loop's first three checks. Returns K (0: no
// stride) after applying the steps to pos, taurun and loopc.
template <int GM>
__device__ __forceinline__ uint32_t box_stride(const KParams& K, Lane& L, int m, const double* tl, const double* pl,
                                               double v, double a, double kap, double trav, double inc, double lim,
                                               int32_t cm, double fm, double rm) {
  // the box's distance comes from a fixed axis: q_m (the moving one) stays below it
  const V3 p = v3(L.pos.x + tl[3], L.pos.y + tl[7], L.pos.z + tl[11]);
  const V3 q = vabs(p) - v3(pl[0], pl[1], pl[2]);
  const double qm = axis_of(q, m);
  const double qj = m == 0 ? dmax(q.y, q.z) : (m == 1 ? dmax(q.x, q.z) : dmax(q.x, q.y));
  if (!(qj < 0.0) || !(v == qj) || !(qm < qj)) return 0;
  const double dm = axis_of(L.dir, m), Tm = axis_of(v3(tl[3], tl[7], tl[11]), m), bm = pl[m];
  const double nmax = m == 0 ? K.xmax : (m == 1 ? K.ymax : K.zmax);
  const int32_t nn = m == 0 ? K.nx : (m == 1 ? K.ny : K.nz);
  const double inv = m == 0 ? K.inv2x : (m == 1 ? K.inv2y : K.inv2z);
  const int32_t fe = m == 0 ? K.fex : (m == 1 ? K.fey : K.fez);
  const double x0 = axis_of(L.pos, m);
  const double s = a * dm;  // (smul(a, dir)'s component)
  double D, xmin, xmax;
  if (!binade_run(x0, s, D, xmin, xmax)) return 0;
  const double t = a * kap;
  const double T0 = L.taurun;
  double DT = 0.0, tmin = -0x1.0p+1000, tmax = 0x1.0p+1000;
  if (t != 0.0) {
    if (!binade_run(T0, t, DT, tmin, tmax)) return 0;
    if (!(DT >= 0.0)) return 0;
  }
  const double lo = a * (1.0 + 0x1.0p-40);
  const double inc_hi = inc * (1.0 + 0x1.0p-40);
  // a first guess from every constraint, then the exact check at both ends
  double kf = run_len(x0, D, xmin, xmax);
  kf = fmin(kf, run_len(T0, DT, tmin, tmax));
  kf = fmin(kf, (double)((uint32_t)MAX_MARCH_ITERS - L.loopc));
  if (DT > 0.0) kf = fmin(kf, floor((L.tau - t - T0) / DT));
  kf = fmin(kf, floor((lim - a - trav) / inc_hi));
  if (D != 0.0) {
    const double q0 = (fm - (x0 + nmax)) * rm;
    kf = fmin(kf, floor((q0 - a * (1.0 + 0x1.0p-39)) / fabs(D * rm)) + 1.0);
    const double xa = fabs(x0 + Tm);
    const bool away = (x0 + Tm > 0.0) == (D > 0.0);
    kf = fmin(kf, floor((qj + bm + (away ? -xa : xa)) / fabs(D)));
  }
  kf = fmin(kf - 1.0, 0x1.0p+30);
  if (!(kf >= 2.0)) return 0;
  uint32_t k = (uint32_t)kf;
  for (int tries = 0; tries < 4 && k >= 2; ++tries, k >>= 1) {
    const double kd = (double)k;
    const double xk = x0 + kd * D, xl = x0 + (kd - 1.0) * D;  // (exact: multiples of u in the binade)
    const double Tk = T0 + kd * DT, Tl = T0 + (kd - 1.0) * DT;
    bool ok = xk >= xmin && xk <= xmax && (t == 0.0 || (Tk >= tmin && Tk <= tmax));
    ok = ok && L.loopc + k <= (uint32_t)MAX_MARCH_ITERS && Tl + t < L.tau;
    ok = ok && a + (trav + kd * inc_hi) < lim;
    // the first and the last step's update_grids stay in the voxel
    const double o0 = x0 + nmax, ol = xl + nmax;
    ok = ok && cell_of<GM>(o0, nn, nmax, inv, fe) == cm && cell_of<GM>(ol, nn, nmax, inv, fe) == cm;
    ok = ok && a < 100000.0 && (fm - o0) * rm > lo && (fm - ol) * rm > lo;
    // and their EVALs still read the fixed axis
    ok = ok && fabs(x0 + Tm) - bm < qj && fabs(xl + Tm) - bm < qj;
    if (!ok) continue;
    if (m == 0) L.pos.x = xk;
    else if (m == 1) L.pos.y = xk;
    else L.pos.z = xk;
    L.taurun = Tk;
    L.loopc += k;
    return k;
  }
  return 0;
}

// The near top's transform and parameters: column k of the cooperative EVAL's LDS table
// (stride 64) or a node's own arrays (stride 1).
struct NearTop {
  const double* t;  // t[r * stride], r < 12
  const double* p;  // p[r * stride], r < 8
  int stride;
};
__device__ __forceinline__ void near_load(const NearTop& nt, double* tl, double* pl) {
#pragma unroll
  for (int r = 0; r < 12; ++r) tl[r] = nt.t[r * nt.stride];
#pragma unroll
  for (int r = 0; r < 8; ++r) pl[r] = nt.p[r * nt.stride];
}

// The far-field loop for near top nt of kind KIND (SPHERE or BOX), run by the photon's lane
// alone. m2 / neg_other: the certificate of the full EVAL at p0; trav0: the distance from p0
// to L.pos (the step P4 took after that EVAL).
// On entry L is at ST_M1 with an EVAL pending and no segment. Returns the steps taken; acc
// receives their deposits' sum for voxel *vox, nsdf the EVALs consumed.
template <int GM, int KIND>
__device__ __forceinline__ uint32_t far_march(const KParams& K, Lane& L, const NearTop& nt, double m2,
                                              bool neg_other, double trav0, double kap,
                                              const double* __restrict__ xf, const double* __restrict__ yf,
                                              const double* __restrict__ zf, double& acc, uint32_t& vox,
                                              uint32_t& nsdf) {
  const double eps = 1e-8;  // inttau2.f90:56
  double tl[12], pl[8];
  near_load(nt, tl, pl);
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
  // strides: a box near top and one moving axis whose fixed coordinates are not zeros
  // (p + (+-0) may change a zero's sign)
  int sm = -1;
  if constexpr (KIND == SMCRT_SDF_BOX) {
    if ((int)!zx + (int)!zy + (int)!zz == 1) sm = !zx ? 0 : (!zy ? 1 : 2);
    if ((sm != 0 && L.pos.x == 0.0) || (sm != 1 && L.pos.y == 0.0) || (sm != 2 && L.pos.z == 0.0)) sm = -1;
  }
  uint32_t cool = 0;  // steps before the next stride attempt after a failed one
  uint32_t n = 0;
  for (;;) {
    // ST_M1's EVAL (:177-191), the near top only
    const double v = sdf_prim_s<1>(KIND, tl, pl, L.pos, true);
    const double a = fabs(v);
    if (!(a + trav < lim)) break;           // the certificate no longer covers p (or NaN)
    if (v > 0.0 && !neg_other) break;       // outside every SDF: tflag, the march ends
    if (!(a >= eps)) break;                 // the march loop ends (:155)
    if constexpr (KIND == SMCRT_SDF_BOX) {
      if (sm >= 0 && cool == 0) {
        const int32_t cm = sm == 0 ? ci : (sm == 1 ? cj : ck);
        const double fm = sm == 0 ? fx : (sm == 1 ? fy : fz), rm = sm == 0 ? rx : (sm == 1 ? ry : rz);
        const double inc = a * dn + K.fm_step;
        const uint32_t ks = box_stride<GM>(K, L, sm, tl, pl, v, a, kap, trav, inc, lim, cm, fm, rm);
        if (ks) {
          nsdf += ks;
          n += ks;
          acc = acc + (double)ks * ((double)(float)a * w);
          trav = trav + (double)ks * (inc * (1.0 + 0x1.0p-40));
          continue;
        }
        cool = 32;
      }
      if (cool) --cool;
    }
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


// The boundary probe's glancing loop (inttau2.f90:226-237) with only the near top evaluated
// per iteration. The loop goes on while new_layer == old_layer and minval(abs(dsNew)) < eps,
// each iteration moving smallStepPos = pos + d_sdf*dir with d_sdf = d_sdf + eps (pos and dir
// fixed). Under the certificate of the full EVAL at p0 = the current smallStepPos (header:
// every other computed |ds_j| stays above |ds_k| while |ds_k(p)| + travel < m2 - 2 fm_err),
// minval(abs(dsNew)) = |ds_k| exactly, and while ds_k < 0 maxloc(dsNew, mask dsNew < 0) is k
// (every other negative value is below -|ds_k|). So an iteration with ds_k < 0, top k ==
// old_layer and |ds_k| < eps is one the full EVAL would continue too, with the same values.
// The travel from p0 needs no sum: every smallStepPos is formed afresh from pos, so it is
// (d_sdf - d0)|dir| plus the rounding of the two positions (2 fm_step).
// On entry L is at ST_G0 with the EVAL at L.ssp pending (that EVAL produced the certificate),
// top_k is the near top's 1-based index. The loop stops BEFORE an iteration it cannot decide,
// and before the glancing guard's last iteration, with L at ST_G0, d and ssp of that iteration
// and its EVAL pending, as the main loop's P3 would have left it. Returns the iterations taken
// (each one a full EVAL of the reference, counted in packet%cnts).
template <int KIND>
__device__ __forceinline__ uint32_t far_glance(const KParams& K, Lane& L, const NearTop& nt, int32_t top_k, double m2) {
  const double eps = 1e-8;  // inttau2.f90:56
  if (top_k != L.old_layer) return 0;
  double tl[12], pl[8];
  near_load(nt, tl, pl);
  const V3 dir = L.dir;
  const double dn = sqrt(dir.x * dir.x + dir.y * dir.y + dir.z * dir.z) * (1.0 + 0x1.0p-48);
  const double lim = m2 - 2.0 * K.fm_err;
  const double d0 = L.d;
  uint32_t n = 0;
  for (;;) {
    const double v = sdf_prim_s<1>(KIND, tl, pl, L.ssp, true);
    const double trav = (L.d - d0) * (1.0 + 0x1.0p-48) * dn + 2.0 * K.fm_step;
    if (!(fabs(v) + trav < lim)) break;                  // the certificate no longer covers ssp (or NaN)
    if (!(v < 0.0) || !(-v < eps)) break;                // the loop may end here: the full EVAL decides
    if (L.loopc + 1u > (uint32_t)MAX_GLANCE_ITERS) break; // the guard's iteration (a fault): main loop
    ++L.loopc;                                           // P3, ST_G0 (:232-237)
    L.d = L.d + eps;
    L.ssp = L.pos + smul(L.d, L.dir);
    ++n;
  }
  return n;
}

}  // namespace smcrt
