/*
 * ORACLE — TEST INFRASTRUCTURE ONLY. Never linked into, loaded by, or called from the
 * product (rsmcrt_amd). Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline
 * leg may load it, and only as the checker / the CPU baseline.
 *
 * A scalar, double-precision CPU restatement of signedMCRT's per-photon hot path
 * (/root/reference, snapshot 2025-02-27), written from the Fortran sources:
 *   run_MCRT              src/kernelsMod.f90:1790-1898   (photon loop)
 *   noBiasPropagation     src/kernelsMod.f90:1901-1976
 *   survivalBiasPropagation src/kernelsMod.f90:1979-2067
 *   test_kernel (moments) src/kernelsMod.f90:2069-2182
 *   tauint2               src/inttau2.f90:15-364
 *   update_grids & DDA    src/inttau2.f90:367-614
 *   SDF primitives        src/sdfs/sdfs.f90:494-735, src/sdfs/sdf_base.f90:146-190
 *   CSG operators         src/sdfs/sdfModifiers.f90:428-491
 *   Fresnel               src/surfaces.f90:14-127
 *   emitters              src/photon.f90:311-359 (point), 566-649 (uniform), 652-710 (pencil)
 *   scatter               src/photon.f90:1045-1103
 *   detectors             src/detectors/detector_base.f90:137-235, detectors.f90:147-469,
 *                         src/geometryMod.f90:217-270
 *
 * Parity pinning: the Fortran reference cannot be built here without stand-ins for its
 * un-vendored dependencies (toml-f, fortran_utilities, stdlib — fpm.toml:8-16), so this
 * restatement is pinned by the reference's own known-answer tests instead
 * (test/end_to_end/test_scat.f90, tools/validateHGG.py, test/SDF/test_SDF.f90,
 * test/fresnel/test_fresnel.f90, test/detector/test_detector.f90): see tests/.
 *
 * Documented deviations from the reference (same in the HIP path):
 *  - RNG: ran2() (compiler intrinsic random_number, random_mod.f90:83-90) is replaced by
 *    Philox4x32-10 keyed by (seed, photon index): draw d of photon p is the (d&1) half
 *    of block d>>1, as a 53-bit double in [0,1).
 *  - log/sin/cos: a fixed fdlibm-style implementation (det_log, det_sincos) is used so
 *    the CPU and GPU produce bit-identical trajectories. Accuracy <= 1 ulp.
 *  - jmean/absorb/emission are summed in fp64 (the reference sums fp32); each deposit is
 *    still real(dcell,sp)*weight (inttau2.f90:427,434).
 *  - `error stop` paths terminate only the photon and are counted as faults. A photon
 *    emitted outside every SDF (layer 0; the reference would index array(0)) is a fault.
 *  - Loops the reference leaves unbounded are capped (SMCRT_MAX_* below) identically on
 *    both sides.
 *  - nphotons is int64 (the reference's int32 overflows at 2^31, sim_state.f90:12).
 * Build with -ffp-contract=off: no fused multiply-add anywhere (the GPU side too).
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "../include/smcrt.h"

#define ORACLE_API __attribute__((visibility("default")))

/* caps shared with the HIP path (rsmcrt_amd/csrc/transport.h) */
#define SMCRT_MAX_EMIT_TRIES 100000
#define SMCRT_MAX_HOP_ITERS 1000000
#define SMCRT_MAX_MARCH_ITERS 10000000
#define SMCRT_MAX_GLANCE_ITERS 100000
#define SMCRT_MAX_DDA_ITERS 10000000
#define SMCRT_MAX_RENORM_ITERS 64
#define SMCRT_MAX_INTERACTIONS 100000000

/* ====================================================================== RNG ===== */
static inline uint32_t mulhilo32(uint32_t a, uint32_t b, uint32_t* hi) {
  uint64_t p = (uint64_t)a * (uint64_t)b;
  *hi = (uint32_t)(p >> 32);
  return (uint32_t)p;
}

/* Philox4x32-10 (Salmon et al., SC'11; Random123 philox.h). */
ORACLE_API void oracle_philox4x32_10(const uint32_t ctr_in[4], const uint32_t key_in[2], uint32_t out[4]) {
  uint32_t c0 = ctr_in[0], c1 = ctr_in[1], c2 = ctr_in[2], c3 = ctr_in[3];
  uint32_t k0 = key_in[0], k1 = key_in[1];
  for (int r = 0; r < 10; ++r) {
    if (r > 0) { k0 += 0x9E3779B9u; k1 += 0xBB67AE85u; }
    uint32_t hi0, hi1;
    uint32_t lo0 = mulhilo32(0xD2511F53u, c0, &hi0);
    uint32_t lo1 = mulhilo32(0xCD9E8D57u, c2, &hi1);
    uint32_t n0 = hi1 ^ c1 ^ k0, n1 = lo1, n2 = hi0 ^ c3 ^ k1, n3 = lo0;
    c0 = n0; c1 = n1; c2 = n2; c3 = n3;
  }
  out[0] = c0; out[1] = c1; out[2] = c2; out[3] = c3;
}

typedef struct {
  uint64_t pid, seed;
  uint32_t draws;
} rng_t;

/* ran2() replacement: draw `draws` of photon `pid` */
static double ran2(rng_t* r) {
  uint32_t d = r->draws++;
  uint32_t ctr[4] = {d >> 1, 0u, (uint32_t)r->pid, (uint32_t)(r->pid >> 32)};
  uint32_t key[2] = {(uint32_t)r->seed, (uint32_t)(r->seed >> 32)};
  uint32_t o[4];
  oracle_philox4x32_10(ctr, key, o);
  uint64_t u = (d & 1u) ? (((uint64_t)o[3] << 32) | o[2]) : (((uint64_t)o[1] << 32) | o[0]);
  return (double)(u >> 11) * 0x1.0p-53;
}

ORACLE_API double oracle_uniform(uint64_t seed, uint64_t pid, uint32_t draw) {
  rng_t r = {pid, seed, draw};
  return ran2(&r);
}

/* ================================================== deterministic elementary math ==== */
static inline uint64_t d2u(double x) { uint64_t u; memcpy(&u, &x, 8); return u; }
static inline double u2d(uint64_t u) { double x; memcpy(&x, &u, 8); return x; }

/* natural log, fdlibm e_log.c algorithm (Sun Microsystems, 1993) */
ORACLE_API double oracle_log(double x) {
  const double ln2_hi = 6.93147180369123816490e-01, ln2_lo = 1.90821492927058770002e-10,
               two54 = 1.80143985094819840000e+16, Lg1 = 6.666666666666735130e-01,
               Lg2 = 3.999999999940941908e-01, Lg3 = 2.857142874366239149e-01,
               Lg4 = 2.222219843214978396e-01, Lg5 = 1.818357216161805012e-01,
               Lg6 = 1.531383769920937332e-01, Lg7 = 1.479819860511658591e-01;
  uint64_t ux = d2u(x);
  int32_t hx = (int32_t)(ux >> 32);
  uint32_t lx = (uint32_t)ux;
  int32_t k = 0;
  if (hx < 0x00100000) {
    if (((hx & 0x7fffffff) | lx) == 0) return -INFINITY;
    if (hx < 0) return NAN;
    k -= 54;
    x *= two54;
    ux = d2u(x);
    hx = (int32_t)(ux >> 32);
  }
  if (hx >= 0x7ff00000) return x + x;
  k += (hx >> 20) - 1023;
  hx &= 0x000fffff;
  int32_t i = (hx + 0x95f64) & 0x100000;
  ux = d2u(x);
  x = u2d(((uint64_t)(uint32_t)(hx | (i ^ 0x3ff00000)) << 32) | (ux & 0xffffffffu));
  k += (i >> 20);
  double f = x - 1.0;
  double dk, R;
  if ((0x000fffff & (2 + hx)) < 3) {
    if (f == 0.0) {
      if (k == 0) return 0.0;
      dk = (double)k;
      return dk * ln2_hi + dk * ln2_lo;
    }
    R = f * f * (0.5 - 0.33333333333333333 * f);
    if (k == 0) return f - R;
    dk = (double)k;
    return dk * ln2_hi - ((R - dk * ln2_lo) - f);
  }
  double s = f / (2.0 + f);
  dk = (double)k;
  double z = s * s;
  i = hx - 0x6147a;
  double w = z * z;
  int32_t j = 0x6b851 - hx;
  double t1 = w * (Lg2 + w * (Lg4 + w * Lg6));
  double t2 = z * (Lg1 + w * (Lg3 + w * (Lg5 + w * Lg7)));
  i |= j;
  R = t2 + t1;
  if (i > 0) {
    double hfsq = 0.5 * f * f;
    if (k == 0) return f - (hfsq - s * (hfsq + R));
    return dk * ln2_hi - ((hfsq - (s * (hfsq + R) + dk * ln2_lo)) - f);
  }
  if (k == 0) return f - s * (f - R);
  return dk * ln2_hi - ((s * (f - R) - dk * ln2_lo) - f);
}

/* fdlibm k_sin.c / k_cos.c kernels on |y| <= pi/4 */
static double ksin(double x) {
  const double S1 = -1.66666666666666324348e-01, S2 = 8.33333333332248946124e-03,
               S3 = -1.98412698298579493134e-04, S4 = 2.75573137070700676789e-06,
               S5 = -2.50507602534068634195e-08, S6 = 1.58969099521155010221e-10;
  double z = x * x;
  double v = z * x;
  double r = S2 + z * (S3 + z * (S4 + z * (S5 + z * S6)));
  return x + v * (S1 + z * r);
}
static double kcos(double x) {
  const double C1 = 4.16666666666666019037e-02, C2 = -1.38888888888741095749e-03,
               C3 = 2.48015872894767294178e-05, C4 = -2.75573143513906633035e-07,
               C5 = 2.08757232129817482790e-09, C6 = -1.13596475577881948265e-11;
  uint32_t ix = (uint32_t)(d2u(x) >> 32) & 0x7fffffffu;
  if (ix < 0x3e400000u) return 1.0;
  double z = x * x;
  double r = z * (C1 + z * (C2 + z * (C3 + z * (C4 + z * (C5 + z * C6)))));
  if (ix < 0x3FD33333u) return 1.0 - (0.5 * z - z * r);
  double qx;
  if (ix > 0x3fe90000u) qx = 0.28125;
  else qx = u2d((uint64_t)(ix - 0x00200000u) << 32);
  double hz = 0.5 * z - qx;
  double a = 1.0 - qx;
  return a - (hz - z * r);
}

/* sin and cos of x in [0, 4pi]: medium Cody-Waite reduction (fdlibm e_rem_pio2.c) */
ORACLE_API void oracle_sincos(double x, double* s, double* c) {
  const double invpio2 = 6.36619772367581382433e-01, pio2_1 = 1.57079632673412561417e+00,
               pio2_1t = 6.07710050650619224932e-11;
  int32_t n = (int32_t)(x * invpio2 + 0.5);
  double fn = (double)n;
  double r = x - fn * pio2_1;
  double w = fn * pio2_1t;
  double y = r - w;
  double sy = ksin(y), cy = kcos(y);
  switch (n & 3) {
    case 0: *s = sy; *c = cy; break;
    case 1: *s = cy; *c = -sy; break;
    case 2: *s = -sy; *c = -cy; break;
    default: *s = -cy; *c = sy; break;
  }
}

/* ====================================================================== vec3 ===== */
typedef struct { double x, y, z; } vec3;
static inline vec3 v3(double x, double y, double z) { vec3 r = {x, y, z}; return r; }
static inline vec3 vadd(vec3 a, vec3 b) { return v3(a.x + b.x, a.y + b.y, a.z + b.z); }
static inline vec3 vsub(vec3 a, vec3 b) { return v3(a.x - b.x, a.y - b.y, a.z - b.z); }
static inline vec3 vmul(vec3 a, double s) { return v3(a.x * s, a.y * s, a.z * s); }     /* vec_mult_scal */
static inline vec3 smul(double s, vec3 a) { return v3(s * a.x, s * a.y, s * a.z); }     /* scal_mult_vec */
static inline vec3 vmulv(vec3 a, vec3 b) { return v3(a.x * b.x, a.y * b.y, a.z * b.z); } /* vec_mult_vec */
static inline double vdot(vec3 a, vec3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; } /* vector_class.f90:279-290 */
static inline double vlen(vec3 a) { return sqrt(a.x * a.x + a.y * a.y + a.z * a.z); }   /* vector_class.f90:405-411 */
static inline vec3 vabs(vec3 a) { return v3(fabs(a.x), fabs(a.y), fabs(a.z)); }
static inline double fmaxd(double a, double b) { return a > b ? a : b; }
static inline double fmind(double a, double b) { return a < b ? a : b; }
static inline vec3 vmaxs(vec3 a, double s) { return v3(fmaxd(a.x, s), fmaxd(a.y, s), fmaxd(a.z, s)); }
static inline double clampd(double v, double lo, double hi) { return fmind(fmaxd(v, lo), hi); }

/* vec_dot_mat, vector_class.f90:292-304: p = (x,y,z,1) . t, t column-major */
static inline vec3 vdotmat(vec3 a, const double* t) {
  return v3(t[0] * a.x + t[1] * a.y + t[2] * a.z + t[3],
            t[4] * a.x + t[5] * a.y + t[6] * a.z + t[7],
            t[8] * a.x + t[9] * a.y + t[10] * a.z + t[11]);
}

/* ===================================================================== scene ===== */
typedef struct {
  const smcrt_sdf_node* nodes;
  int32_t n_nodes;
  const int32_t* top;
  int32_t n_top;
  double* kappa; double* albedo; double* mua; double* hgg; double* g2; double* nidx; /* per top-level */
  smcrt_grid grid;
  double* xface; double* yface; double* zface;
  const smcrt_detector* dets;
  int32_t n_dets;
  int64_t* det_off;
} scene_t;

static double sdf_eval_node(const scene_t* S, int32_t idx, vec3 pos, int depth);

static double csg(int32_t op, double d1, double d2, double k) {
  switch (op) {
    case SMCRT_OP_UNION: return fmind(d1, d2);                           /* sdfModifiers.f90:428-440 */
    case SMCRT_OP_SMOOTH_UNION: {                                        /* :442-456 */
      double h = fmaxd(k - fabs(d1 - d2), 0.0) / k;
      return fmind(d1, d2) - h * h * h * k * (1.0 / 6.0);
    }
    case SMCRT_OP_SUBTRACTION: return fmaxd(-d1, d2);                    /* :458-473 */
    default: return fmaxd(d1, d2);                                       /* :475-491 */
  }
}

static double sdf_eval_node(const scene_t* S, int32_t idx, vec3 pos, int depth) {
  const smcrt_sdf_node* nd = &S->nodes[idx];
  const double* P = nd->param;
  if (nd->kind == SMCRT_SDF_MODEL) {                                     /* eval_model sdf_base.f90:146-161 */
    if (depth > 8 || nd->n_children < 1) return NAN;
    double res = sdf_eval_node(S, nd->first_child, pos, depth + 1);
    for (int32_t i = 1; i < nd->n_children; ++i)
      res = csg(nd->op, res, sdf_eval_node(S, nd->first_child + i, pos, depth + 1), nd->k);
    return res;
  }
  vec3 p = vdotmat(pos, nd->transform);
  switch (nd->kind) {
    case SMCRT_SDF_SPHERE:                                               /* sdfs.f90:494-508 */
      return sqrt(p.x * p.x + p.y * p.y + p.z * p.z) - P[0];
    case SMCRT_SDF_BOX: {                                                /* sdfs.f90:510-525 */
      vec3 q = vsub(vabs(p), v3(P[0], P[1], P[2]));
      return vlen(vmaxs(q, 0.0)) + fmind(fmaxd(q.x, fmaxd(q.y, q.z)), 0.0);
    }
    case SMCRT_SDF_TORUS: {                                              /* sdfs.f90:527-542 */
      vec3 q = v3(vlen(v3(p.x, 0.0, p.z)) - P[0], p.y, 0.0);
      return vlen(q) - P[1];
    }
    case SMCRT_SDF_CYLINDER: {                                           /* sdfs.f90:544-581 */
      vec3 a = v3(P[0], P[1], P[2]), b = v3(P[3], P[4], P[5]);
      vec3 ba = vsub(b, a), pa = vsub(p, a);
      double baba = vdot(ba, ba), paba = vdot(pa, ba);
      double x = vlen(vsub(vmul(pa, baba), vmul(ba, paba))) - P[6] * baba;
      double y = fabs(paba - baba * 0.5) - baba * 0.5;
      double x2 = x * x, y2 = (y * y) * baba, d;
      if (fmaxd(x, y) < 0.0) d = -fmind(x2, y2);
      else if (x > 0.0 && y > 0.0) d = x2 + y2;
      else if (x > 0.0) d = x2;
      else if (y > 0.0) d = y2;
      else d = 0.0;
      return copysign(sqrt(fabs(d)) / baba, d);
    }
    case SMCRT_SDF_TRIPRISM: {                                           /* sdfs.f90:583-597 */
      vec3 q = vabs(p);
      return fmaxd(q.z - P[1], fmaxd(q.x * 0.866025 + p.y * 0.5, -p.y) - P[0] * 0.5);
    }
    case SMCRT_SDF_SEGMENT: {                                            /* sdfs.f90:599-626 */
      vec3 a = v3(P[0], P[1], P[2]), b = v3(P[3], P[4], P[5]);
      vec3 pa = vsub(p, a), ba = vsub(b, a);
      double h = clampd(vdot(pa, ba) / vdot(ba, ba), 0.0, 1.0);
      return vlen(vsub(pa, vmul(ba, h))) - 0.1;
    }
    case SMCRT_SDF_CAPSULE: {                                            /* sdfs.f90:628-648 */
      vec3 a = v3(P[0], P[1], P[2]), b = v3(P[3], P[4], P[5]);
      vec3 pa = vsub(p, a), ba = vsub(b, a);
      double h = clampd(vdot(pa, ba) / vdot(ba, ba), 0.0, 1.0);
      return vlen(vsub(pa, vmul(ba, h))) - P[6];
    }
    case SMCRT_SDF_CONE: {                                               /* sdfs.f90:650-686 */
      vec3 a = v3(P[0], P[1], P[2]), b = v3(P[3], P[4], P[5]);
      double ra = P[6], rb = P[7];
      double rba = rb - ra;
      double baba = vdot(vsub(b, a), vsub(b, a));
      double papa = vdot(vsub(p, a), vsub(p, a));
      double paba = vdot(vsub(p, a), vsub(b, a)) / baba;
      double x = sqrt(papa - baba * (paba * paba));
      double cax = (paba < 0.5) ? fmaxd(0.0, x - ra) : fmaxd(0.0, x - rb);
      double cay = fabs(paba - 0.5) - 0.5;
      double k = rba * rba + baba;
      double f = clampd((rba * (x - ra) + paba * baba) / k, 0.0, 1.0);
      double cbx = x - ra - f * rba;
      double cby = paba - f;
      double s = (cbx < 0.0 && cay < 0.0) ? -1.0 : 1.0;
      return s * sqrt(fmind(cax * cax + baba * (cay * cay), cbx * cbx + baba * (cby * cby)));
    }
    case SMCRT_SDF_EGG: {                                                /* sdfs.f90:688-718 */
      double r1 = P[0], r2 = P[1], hh = P[2];
      vec3 pin = v3(fabs(p.x), p.y, p.z);
      double r = r1 - r2;
      double h_in = hh + r;
      double l = (h_in * h_in - r * r) / (2.0 * r);
      if (pin.y <= 0.0) return vlen(pin) - r1;
      if ((pin.y - h_in) * l > pin.x * h_in)
        return vlen(vsub(pin, v3(0.0, h_in, 0.0))) - ((r1 + l) - vlen(v3(h_in, l, 0.0)));
      return vlen(vadd(pin, v3(l, 0.0, 0.0))) - (r1 + l);
    }
    case SMCRT_SDF_PLANE:                                                /* sdfs.f90:720-735 */
      return vdot(p, v3(P[0], P[1], P[2]));
    default:
      return NAN;
  }
}

static inline double sdf_top(const scene_t* S, int32_t i /*0-based*/, vec3 pos) {
  return sdf_eval_node(S, S->top[i], pos, 0);
}

/* ds(i) for all i, plus the reductions tauint2 uses */
typedef struct { double minabs, minv; int32_t maxloc; } dsinfo;

static dsinfo eval_all(const scene_t* S, vec3 pos, double* ds, uint64_t* cnt, int mask_le) {
  dsinfo r;
  r.minabs = INFINITY; r.minv = INFINITY; r.maxloc = 0;
  double best = -INFINITY;
  for (int32_t i = 0; i < S->n_top; ++i) {
    double d = sdf_top(S, i, pos);
    if (ds) ds[i] = d;
    double a = fabs(d);
    if (a < r.minabs) r.minabs = a;            /* minval(abs(ds)) */
    if (d < r.minv) r.minv = d;                /* minval(ds) */
    int neg = mask_le ? (d <= 0.0) : (d < 0.0);
    if (neg && (r.maxloc == 0 || d > best)) {  /* maxloc(ds, mask=ds<0): first max */
      best = d; r.maxloc = i + 1;
    }
  }
  *cnt += (uint64_t)S->n_top;
  return r;
}

/* ====================================================================== packet ===== */
typedef struct {
  vec3 pos, n;
  int32_t xcell, ycell, zcell;
  int tflag;
  int32_t layer;
  uint32_t bounces;
  double weight;
  uint32_t nscatt;
} packet_t;

typedef struct {
  const scene_t* S;
  uint32_t flags;
  double* jmean; double* absorb; double* emission; double* det; double* moments;
  uint64_t ctr[SMCRT_NCOUNTERS];
  double nscatt;
  int fault;
} ctx_t;

/* update_voxels, inttau2.f90:587-614 (pos in corner coordinates) */
static inline int32_t cell_of(double p, int32_t n, double max) {
  double f = floor(((double)n * p) / (2.0 * max));
  if (!(f >= 0.0 && f < (double)n)) return -1;  /* also catches NaN */
  return (int32_t)f + 1;
}
static inline void update_voxels(const scene_t* S, vec3 p, int32_t* ci, int32_t* cj, int32_t* ck) {
  *ci = cell_of(p.x, S->grid.nx, S->grid.xmax);
  *cj = cell_of(p.y, S->grid.ny, S->grid.ymax);
  *ck = cell_of(p.z, S->grid.nz, S->grid.zmax);
}

/* get_voxel_cart, grid.f90:51-78 (pos in centred coordinates) */
static inline int32_t vox_of(double p, int32_t n, double max) {
  double f = floor(((double)n * (p + max)) / (2.0 * max));
  if (!(f >= 0.0 && f < (double)n)) return -1;
  return (int32_t)f + 1;
}

static inline int64_t lin(const scene_t* S, int32_t i, int32_t j, int32_t k) {
  return (int64_t)(i - 1) + (int64_t)S->grid.nx * ((int64_t)(j - 1) + (int64_t)S->grid.ny * (int64_t)(k - 1));
}

/* deposit of inttau2.f90:427/434: jmean(cell) += real(dcell,sp)*weight */
static inline void deposit(ctx_t* C, int32_t i, int32_t j, int32_t k, double dcell, double weight) {
  C->ctr[SMCRT_CTR_DEPOSITS]++;
  if (C->jmean) C->jmean[lin(C->S, i, j, k)] += (double)(float)dcell * weight;
}

/* update_grids + wall_dist + update_pos, inttau2.f90:367-584. `pos` is the segment start
 * (centred); d_sdf the length; the packet's cells/tflag are updated. */
static void update_grids(ctx_t* C, vec3 pos, vec3 dir, double d_sdf, packet_t* pk) {
  const scene_t* S = C->S;
  const double xmax = S->grid.xmax, ymax = S->grid.ymax, zmax = S->grid.zmax;
  C->ctr[SMCRT_CTR_GRID_UPDATES]++;
  vec3 old = v3(pos.x + xmax, pos.y + ymax, pos.z + zmax);
  int32_t ci, cj, ck;
  update_voxels(S, old, &ci, &cj, &ck);
  pk->xcell = ci; pk->ycell = cj; pk->zcell = ck;
  if (!(C->flags & SMCRT_FLAG_PATHLENGTH)) {                         /* :446-463 */
    old.x = old.x + dir.x * d_sdf;
    old.y = old.y + dir.y * d_sdf;
    old.z = old.z + dir.z * d_sdf;
    update_voxels(S, old, &ci, &cj, &ck);
    if (ci == -1 || cj == -1 || ck == -1) pk->tflag = 1;
    pk->xcell = ci; pk->ycell = cj; pk->zcell = ck;
    return;
  }
  const double delta = 1e-8;                                         /* local delta, :393 */
  double d = 0.0;
  if (ci == -1 || cj == -1 || ck == -1) { pk->tflag = 1; return; }   /* :411-415 */
  for (int64_t it = 0;; ++it) {
    if (it >= SMCRT_MAX_DDA_ITERS) { C->fault = 1; pk->tflag = 1; break; }
    /* wall_dist, :467-521 */
    double dx = -999.0, dy = -999.0, dz = -999.0;
    if (dir.x > 0.0) dx = (S->xface[ci] - old.x) / dir.x;
    else if (dir.x < 0.0) dx = (S->xface[ci - 1] - old.x) / dir.x;
    else if (dir.x == 0.0) dx = 100000.0;
    if (dir.y > 0.0) dy = (S->yface[cj] - old.y) / dir.y;
    else if (dir.y < 0.0) dy = (S->yface[cj - 1] - old.y) / dir.y;
    else if (dir.y == 0.0) dy = 100000.0;
    if (dir.z > 0.0) dz = (S->zface[ck] - old.z) / dir.z;
    else if (dir.z < 0.0) dz = (S->zface[ck - 1] - old.z) / dir.z;
    else if (dir.z == 0.0) dz = 100000.0;
    double dcell = fmind(fmind(dx, dy), dz);
    if (dcell < 0.0) { C->fault = 1; pk->tflag = 1; break; }        /* error stop :510-516 */
    int lx = (dcell == dx), ly = (dcell == dy), lz = (dcell == dz);
    if (d + dcell > d_sdf) {                                         /* :421-429 */
      dcell = d_sdf - d;
      d = d_sdf;
      deposit(C, ci, cj, ck, dcell, pk->weight);
      old.x = old.x + dir.x * dcell;                                 /* update_pos(.false.) */
      old.y = old.y + dir.y * dcell;
      old.z = old.z + dir.z * dcell;
      break;
    }
    d = d + dcell;                                                   /* :430-436 */
    deposit(C, ci, cj, ck, dcell, pk->weight);
    /* update_pos(.true.), :538-582 */
    if (lx) {
      if (dir.x > 0.0) old.x = S->xface[ci] + delta;
      else if (dir.x < 0.0) old.x = S->xface[ci - 1] - delta;
      old.y = old.y + dir.y * dcell;
      old.z = old.z + dir.z * dcell;
    } else if (ly) {
      if (dir.y > 0.0) old.y = S->yface[cj] + delta;
      else if (dir.y < 0.0) old.y = S->yface[cj - 1] - delta;
      old.x = old.x + dir.x * dcell;
      old.z = old.z + dir.z * dcell;
    } else if (lz) {
      if (dir.z > 0.0) old.z = S->zface[ck] + delta;
      else if (dir.z < 0.0) old.z = S->zface[ck - 1] - delta;
      old.x = old.x + dir.x * dcell;
      old.y = old.y + dir.y * dcell;
    } else {                                                         /* error stop :570-573 */
      C->fault = 1; pk->tflag = 1; break;
    }
    update_voxels(S, old, &ci, &cj, &ck);
    if (ci == -1 || cj == -1 || ck == -1) { pk->tflag = 1; break; }  /* :437-440 */
  }
  pk->xcell = ci; pk->ycell = cj; pk->zcell = ck;
}

/* ============================================================== detectors ===== */
/* intersectPlane / intersectCircle, geometryMod.f90:217-270 */
static int intersect_circle(vec3 n, vec3 p0, double radius, vec3 l0, vec3 l, double* t, double* d2) {
  *t = 0.0;
  double denom = vdot(n, l);
  if (denom > 1e-6) {
    vec3 p0l0 = vsub(p0, l0);
    double tt = vdot(p0l0, n);
    tt = tt / denom;
    *t = tt;
    if (tt > -1e-6) {
      vec3 p = vadd(l0, vmul(l, tt));
      vec3 v = vsub(p, p0);
      *d2 = sqrt(vdot(v, v));
      if (*d2 <= radius) return 1;
    }
  }
  return 0;
}

/* Fortran NINT (half away from zero) and INT (toward zero) with a bounds guard */
static inline int64_t f_nint(double x) {
  if (!(fabs(x) < 4.0e18)) return x > 0 ? (int64_t)4e18 : -(int64_t)4e18;
  return (int64_t)round(x);
}
static inline int64_t f_int(double x) {
  if (!(fabs(x) < 4.0e18)) return x > 0 ? (int64_t)4e18 : -(int64_t)4e18;
  return (int64_t)x;
}

/* for each detector: record_hit(hit_t(startPos, dir, pointSep, layer, weight)) */
static void record_hits(ctx_t* C, vec3 start, vec3 dir, double pointSep, int32_t layer, double weight) {
  const scene_t* S = C->S;
  double value1D = (double)layer;                                    /* hit_t%value1D <- layer */
  for (int32_t di = 0; di < S->n_dets; ++di) {
    const smcrt_detector* D = &S->dets[di];
    vec3 dpos = v3(D->pos[0], D->pos[1], D->pos[2]);
    vec3 ddir = v3(D->dir[0], D->dir[1], D->dir[2]);
    double* data = C->det ? C->det + S->det_off[di] : NULL;
    double t;
    if (D->kind == SMCRT_DET_CIRCLE) {                               /* detectors.f90:147-164 */
      int hit = intersect_circle(ddir, dpos, D->radius, start, dir, &t, &value1D);
      if (hit && (t <= 0.0 || t > pointSep)) hit = 0;
      if (hit) {
        int64_t idx = f_nint(value1D / D->bin_wid) + 1;              /* detector_base.f90:151 */
        if (idx > D->nbins) idx = D->nbins;
        if (idx >= 1) { if (data) data[idx - 1] += weight; C->ctr[SMCRT_CTR_DETECTOR_HITS]++; }
      }
    } else if (D->kind == SMCRT_DET_ANNULUS) {                       /* detectors.f90:212-244 */
      int h1 = intersect_circle(ddir, dpos, D->r1, start, dir, &t, &value1D);
      int h2 = intersect_circle(ddir, dpos, D->r2, start, dir, &t, &value1D);
      int hit = 0;
      if (!h1 && h2) hit = !(t <= 0.0 || t > pointSep);
      value1D = value1D - D->r1;
      if (hit) {
        int64_t idx = f_nint(value1D / D->bin_wid) + 1;
        if (idx > D->nbins) idx = D->nbins;
        if (idx >= 1) { if (data) data[idx - 1] += weight; C->ctr[SMCRT_CTR_DETECTOR_HITS]++; }
      }
    } else if (D->kind == SMCRT_DET_CAMERA) {                        /* detectors.f90:447-469 */
      vec3 n = ddir, e1 = v3(D->e1[0], D->e1[1], D->e1[2]), e2 = v3(D->e2[0], D->e2[1], D->e2[2]);
      double tt = vdot(vsub(dpos, start), n) / vdot(dir, n);
      if (tt >= 0.0) {
        vec3 v = vsub(vadd(start, smul(tt, dir)), dpos);
        double proj1 = vdot(v, e1) / D->width;
        double proj2 = vdot(v, e2) / D->height;
        if ((proj1 < D->width && proj1 > 0.0) && (proj2 < D->height && proj2 > 0.0)) {
          /* record_hit_2D_sub, detector_base.f90:206-235 */
          double x = start.z + D->pos[0];
          double y = start.y + D->pos[1];
          int64_t idx = f_int(x / D->bin_wid) + 1;
          int64_t idy = f_int(y / D->bin_wid_y) + 1;
          if (idx > D->nbins) idx = D->nbins;
          if (idy > D->nbins) idy = D->nbins;
          if (idx < 1) idx = D->nbins;
          if (idy < 1) idy = D->nbins;
          if (data) data[(idx - 1) + (int64_t)D->nbins * (idy - 1)] += 1.0;
          C->ctr[SMCRT_CTR_DETECTOR_HITS]++;
        }
      }
    }
    /* SMCRT_DET_FIBRE: not supported by this restatement (rejected at scene build) */
  }
}

/* ================================================================ surfaces ===== */
/* fresnel, surfaces.f90:86-127 */
ORACLE_API double oracle_fresnel(const double I[3], const double N[3], double n1, double n2) {
  double costt = fabs(I[0] * N[0] + I[1] * N[1] + I[2] * N[2]);
  if (costt > 1.0) costt = 1.0;
  double sintt = sqrt(1.0 - costt * costt);
  double sint2 = n1 / n2 * sintt;
  if (sint2 > 1.0) return 1.0;
  if (costt == 1.0) return 0.0;
  sint2 = (n1 / n2) * sintt;
  double cost2 = sqrt(1.0 - sint2 * sint2);
  double a = (n1 * costt - n2 * cost2) / (n1 * costt + n2 * cost2);
  double b = (n1 * cost2 - n2 * costt) / (n1 * cost2 + n2 * costt);
  double f1 = fabs(a) * fabs(a), f2 = fabs(b) * fabs(b);
  return 0.5 * (f1 + f2);
}

/* reflect / refract, surfaces.f90:42-84 */
static vec3 reflect(vec3 I, vec3 N) {
  double s = 2.0 * vdot(N, I);
  return vsub(I, smul(s, N));
}
static vec3 refract(vec3 I, vec3 N, double eta) {
  vec3 Nt = N;
  double c1 = vdot(Nt, I);
  if (c1 < 0.0) c1 = -c1;
  else Nt = smul(-1.0, N);
  double c2 = sqrt(1.0 - (eta * eta) * (1.0 - c1 * c1));
  return vadd(smul(eta, I), smul(eta * c1 - c2, Nt));
}

ORACLE_API void oracle_reflect_refract(double I[3], const double N[3], double n1, double n2, double xi, int* rflag) {
  double R = oracle_fresnel(I, N, n1, n2);
  vec3 i = v3(I[0], I[1], I[2]), nn = v3(N[0], N[1], N[2]), o;
  if (xi <= R) { o = reflect(i, nn); *rflag = 1; }
  else { o = refract(i, nn, n1 / n2); *rflag = 0; }
  I[0] = o.x; I[1] = o.y; I[2] = o.z;
}

/* calcNormal, sdf_base.f90:166-190 (tetrahedral difference of one top-level SDF) */
static vec3 calc_normal(const scene_t* S, vec3 p, int32_t top0) {
  const double h = 1e-6;
  vec3 xyy = v3(1.0, -1.0, -1.0), yyx = v3(-1.0, -1.0, 1.0), yxy = v3(-1.0, 1.0, -1.0), xxx = v3(1.0, 1.0, 1.0);
  double e1 = sdf_top(S, top0, vadd(p, vmul(xyy, h)));
  double e2 = sdf_top(S, top0, vadd(p, vmul(yyx, h)));
  double e3 = sdf_top(S, top0, vadd(p, vmul(yxy, h)));
  double e4 = sdf_top(S, top0, vadd(p, vmul(xxx, h)));
  vec3 n = vadd(vadd(vadd(vmul(xyy, e1), vmul(yyx, e2)), vmul(yxy, e3)), vmul(xxx, e4));
  double len = vlen(n);
  return v3(n.x / len, n.y / len, n.z / len);
}

/* ================================================================== tauint2 ===== */
static double pointsep(vec3 a, vec3 b) {
  double dx = a.x - b.x, dy = a.y - b.y, dz = a.z - b.z;
  return sqrt(dx * dx + dy * dy + dz * dz);
}

static void tauint2(ctx_t* C, packet_t* pk, rng_t* rng, double* ds, double* dsNew) {
  const scene_t* S = C->S;
  vec3 pos = pk->pos, oldpos = pos, startPos = pos, dir = pk->n;
  const double eps = 1e-8;                                           /* :56 */
  uint64_t* cnt = &C->ctr[SMCRT_CTR_SDF_EVALS];
  C->ctr[SMCRT_CTR_TAUINT]++;
  double tau = -oracle_log(ran2(rng));                               /* :58 */
  double taurun = 0.0, d_sdf, t_sdf;
  dsinfo I;
  const int ndet = S->n_dets;
  int64_t hop = 0;
  while (taurun <= tau) {                                            /* :61 */
    if (++hop > SMCRT_MAX_HOP_ITERS) { C->fault = 1; pk->tflag = 1; break; }
    I = eval_all(S, pos, ds, cnt, 0);                                /* :63-69 */
    d_sdf = I.minabs;
    if (d_sdf < eps) {                                               /* :73-146 */
      d_sdf = I.minabs + 2.0 * eps;
      vec3 ssp = vadd(pos, smul(d_sdf, dir));
      dsinfo J = eval_all(S, ssp, ds, cnt, 0);
      int32_t L = pk->layer;
      double kap = S->kappa[L - 1];
      if (J.maxloc == pk->layer) {                                   /* forward */
        oldpos = pos;
        t_sdf = d_sdf * kap;
        if (taurun + t_sdf < tau) {
          pos = vadd(pos, smul(d_sdf, dir));
          taurun = taurun + t_sdf;
          update_grids(C, oldpos, dir, d_sdf, pk);
        } else {
          d_sdf = (tau - taurun) / kap;
          taurun = taurun + t_sdf;
          update_grids(C, oldpos, dir, d_sdf, pk);
        }
      } else {                                                       /* backward */
        oldpos = pos;
        t_sdf = d_sdf * kap;
        if (taurun + t_sdf < tau) {
          pos = vsub(pos, smul(d_sdf, dir));
          taurun = taurun + t_sdf;
          update_grids(C, oldpos, dir, d_sdf, pk);
        } else {
          d_sdf = (tau - taurun) / kap;
          pos = vsub(pos, smul(d_sdf, dir));
          update_grids(C, oldpos, dir, d_sdf, pk);
        }
      }
      if (ndet) record_hits(C, startPos, dir, pointsep(pos, startPos), pk->layer, pk->weight);
      startPos = pos;
      I = eval_all(S, pos, ds, cnt, 0);
      d_sdf = I.minabs;
      if (I.minv > 0.0) pk->tflag = 1;
    }
    if (taurun >= tau || pk->tflag) break;                           /* :149-152 */
    int64_t march = 0;
    while (d_sdf >= eps) {                                           /* :155-192 */
      if (++march > SMCRT_MAX_MARCH_ITERS) { C->fault = 1; pk->tflag = 1; break; }
      double kap = S->kappa[pk->layer - 1];
      t_sdf = d_sdf * kap;
      if (taurun + t_sdf < tau) {
        taurun = taurun + t_sdf;
        oldpos = pos;
        update_grids(C, oldpos, dir, d_sdf, pk);
        pos = vadd(pos, smul(d_sdf, dir));
      } else {
        d_sdf = (tau - taurun) / kap;
        taurun = tau;
        oldpos = pos;
        pos = vadd(pos, smul(d_sdf, dir));
        update_grids(C, oldpos, dir, d_sdf, pk);
        break;
      }
      I = eval_all(S, pos, ds, cnt, 0);
      d_sdf = I.minabs;
      if (I.minv > 0.0) { pk->tflag = 1; break; }
    }
    if (ndet) record_hits(C, startPos, dir, pointsep(pos, startPos), pk->layer, pk->weight);
    startPos = pos;
    if (taurun >= tau || pk->tflag) break;                           /* :204-207 */
    /* boundary crossing, :213-235 */
    d_sdf = I.minabs + 2.0 * eps;
    vec3 ssp = vadd(pos, smul(d_sdf, dir));
    dsinfo Nw = eval_all(S, ssp, dsNew, cnt, 0);
    int32_t new_layer = Nw.maxloc;
    double glancing = Nw.minabs;
    int32_t old_layer = pk->layer;
    int64_t gl = 0;
    while (new_layer == old_layer && glancing < eps) {
      if (++gl > SMCRT_MAX_GLANCE_ITERS) { C->fault = 1; pk->tflag = 1; break; }
      d_sdf = d_sdf + eps;
      ssp = vadd(pos, smul(d_sdf, dir));
      Nw = eval_all(S, ssp, dsNew, cnt, 0);
      new_layer = Nw.maxloc;
      glancing = Nw.minabs;
    }
    if (pk->tflag) break;
    if (new_layer == 0) { pk->tflag = 1; break; }                    /* :237-241 */
    double n1 = S->nidx[pk->layer - 1], n2 = S->nidx[new_layer - 1];
    if (n1 != n2) {                                                  /* :248-317 */
      int32_t L = -1;
      if (dsNew[new_layer - 1] < 0.0 && ds[new_layer - 1] >= 0.0) L = new_layer;
      else if (dsNew[old_layer - 1] >= 0.0 && ds[old_layer - 1] < 0.0) L = old_layer;
      else if (dsNew[new_layer - 1] < 0.0 && dsNew[old_layer - 1] < 0.0) L = new_layer;
      else if (ds[old_layer - 1] >= 0.0 && dsNew[old_layer - 1] >= 0.0) L = old_layer;
      else { C->fault = 1; pk->tflag = 1; break; }                   /* error stop :264-277 */
      vec3 N = calc_normal(S, pos, L - 1);
      C->ctr[SMCRT_CTR_FRESNEL]++;
      double Ivec[3] = {dir.x, dir.y, dir.z}, Nv[3] = {N.x, N.y, N.z};
      int rflag;
      oracle_reflect_refract(Ivec, Nv, n1, n2, ran2(rng), &rflag);
      dir = v3(Ivec[0], Ivec[1], Ivec[2]);
      if (!rflag) {                                                  /* transmitted */
        pk->layer = new_layer;
        oldpos = pos;
        update_grids(C, oldpos, dir, d_sdf, pk);
        t_sdf = d_sdf * S->kappa[pk->layer - 1];
        taurun = taurun + t_sdf;
        pos = ssp;
        if (ndet) record_hits(C, startPos, dir, pointsep(pos, startPos), pk->layer, pk->weight);
        startPos = pos;
      } else {                                                       /* reflected */
        C->ctr[SMCRT_CTR_REFLECTIONS]++;
        oldpos = pos;
        startPos = pos;
        pk->bounces += 1;
        if (pk->bounces > 1000) {                                    /* :313-315, no write-back */
          C->ctr[SMCRT_CTR_BOUNCE_ABORTS]++;
          return;
        }
      }
    } else {                                                         /* :318-336 */
      pk->layer = new_layer;
      oldpos = pos;
      update_grids(C, oldpos, dir, d_sdf, pk);
      t_sdf = d_sdf * S->kappa[pk->layer - 1];
      taurun = taurun + t_sdf;
      pos = ssp;
      if (ndet) record_hits(C, startPos, dir, pointsep(pos, startPos), pk->layer, pk->weight);
      startPos = pos;
    }
    if (pk->tflag) break;                                            /* :338 */
  }
  pk->pos = pos;                                                     /* :341-362 */
  pk->n = dir;
  if (fabs(pk->pos.x) > S->grid.xmax) pk->tflag = 1;
  if (fabs(pk->pos.y) > S->grid.ymax) pk->tflag = 1;
  if (fabs(pk->pos.z) > S->grid.zmax) pk->tflag = 1;
}

/* ================================================================== scatter ===== */
static void scatter(ctx_t* C, packet_t* pk, double hgg, rng_t* rng) {  /* photon.f90:1045-1103 */
  double cost, temp;
  if (hgg == 0.0) {
    cost = 2.0 * ran2(rng) - 1.0;
  } else {
    temp = (1.0 - hgg * hgg) / (1.0 - hgg + 2.0 * hgg * ran2(rng));
    cost = (1.0 + hgg * hgg - temp * temp) / (2.0 * hgg);
  }
  double sint = sqrt(1.0 - cost * cost);
  double phi = 6.283185307179586 * ran2(rng);                        /* TWOPI*ran2() */
  double sinp, cosp;
  oracle_sincos(phi, &sinp, &cosp);
  double nxp = pk->n.x, nyp = pk->n.y, nzp = pk->n.z, uxx, uyy, uzz;
  if (nzp > 1.0 - 1e-12) {
    uxx = sint * cosp; uyy = sint * sinp; uzz = cost;
  } else if (nzp < -1.0 + 1e-12) {
    uxx = sint * cosp; uyy = sint * sinp; uzz = -cost;
  } else {
    temp = sqrt(1.0 - nzp * nzp);
    uxx = sint * ((nxp * nzp * cosp - nyp * sinp) / temp) + nxp * cost;
    uyy = sint * ((nyp * nzp * cosp + nxp * sinp) / temp) + nyp * cost;
    uzz = -1.0 * sint * cosp * temp + nzp * cost;
  }
  temp = sqrt(uxx * uxx + uyy * uyy + uzz * uzz);
  int it = 0;
  while (fabs(temp - 1.0) > 1e-12) {
    if (++it > SMCRT_MAX_RENORM_ITERS) { C->fault = 1; pk->tflag = 1; break; }
    uxx = uxx / temp; uyy = uyy / temp; uzz = uzz / temp;
    temp = sqrt(uxx * uxx + uyy * uyy + uzz * uzz);
  }
  pk->n = v3(uxx, uyy, uzz);
}

/* ==================================================================== emit ===== */
static void emit(ctx_t* C, const smcrt_source* src, packet_t* pk, rng_t* rng) {
  const scene_t* S = C->S;
  const double xmax = S->grid.xmax, ymax = S->grid.ymax, zmax = S->grid.zmax;
  if (src->kind == SMCRT_SRC_POINT) {                                /* photon.f90:311-359 */
    pk->pos = v3(src->pos[0], src->pos[1], src->pos[2]);
    double phi = ran2(rng) * 6.283185307179586;
    double sinp, cosp;
    oracle_sincos(phi, &sinp, &cosp);
    double cost = 2.0 * ran2(rng) - 1.0;
    double sint = sqrt(1.0 - cost * cost);
    pk->n = v3(sint * cosp, sint * sinp, cost);
    pk->layer = 1;
  } else {
    if (src->kind == SMCRT_SRC_UNIFORM) {                            /* photon.f90:566-649 */
      double rx = ran2(rng), ry = ran2(rng);
      pk->pos = v3(src->p1[0] + rx * src->p2[0] + ry * src->p3[0],
                   src->p1[1] + rx * src->p2[1] + ry * src->p3[1],
                   src->p1[2] + rx * src->p2[2] + ry * src->p3[2]);
    } else {                                                         /* pencil :652-710 */
      pk->pos = v3(src->pos[0], src->pos[1], src->pos[2]);
      pk->layer = 1;  /* layer is not set by uniform/pencil; overwritten by the caller */
    }
    if (pk->pos.x == -xmax) pk->pos.x = pk->pos.x + 7.9e-7;
    else if (pk->pos.x == xmax) pk->pos.x = pk->pos.x - 7.9e-7;
    if (pk->pos.y == -ymax) pk->pos.y = pk->pos.y + 7.9e-7;
    else if (pk->pos.y == ymax) pk->pos.y = pk->pos.y - 7.9e-7;
    if (pk->pos.z == -zmax) pk->pos.z = pk->pos.z + 7.9e-7;
    else if (pk->pos.z == zmax) pk->pos.z = pk->pos.z - 7.9e-7;
    pk->n = v3(src->dir[0], src->dir[1], src->dir[2]);
  }
  pk->tflag = 0;
  pk->bounces = 0;
  pk->weight = 1.0;
  pk->xcell = vox_of(pk->pos.x, S->grid.nx, xmax);
  pk->ycell = vox_of(pk->pos.y, S->grid.ny, ymax);
  pk->zcell = vox_of(pk->pos.z, S->grid.nz, zmax);
}

static inline int cell_out(const scene_t* S, const packet_t* pk) {
  return pk->xcell < 1 || pk->xcell > S->grid.nx || pk->ycell < 1 || pk->ycell > S->grid.ny ||
         pk->zcell < 1 || pk->zcell > S->grid.nz;
}

static void add_cell(const scene_t* S, double* g, const packet_t* pk, double w, ctx_t* C) {
  if (cell_out(S, pk)) { C->fault = 1; return; }
  if (g) g[lin(S, pk->xcell, pk->ycell, pk->zcell)] += w;
}

/* one photon: noBiasPropagation / survivalBiasPropagation / test_kernel body */
static void run_photon(ctx_t* C, const smcrt_source* src, uint64_t pid, uint64_t seed,
                       double* ds, double* dsNew, smcrt_photon_record* rec) {
  const scene_t* S = C->S;
  rng_t rng = {pid, seed, 0};
  packet_t pk;
  memset(&pk, 0, sizeof pk);
  const int test_kernel = (C->flags & SMCRT_FLAG_TEST_KERNEL) != 0;
  uint32_t status = 0;
  C->fault = 0;
  emit(C, src, &pk, &rng);                                           /* kernelsMod.f90:1937 */
  if (!test_kernel) {
    int tries = 0;
    while (cell_out(S, &pk)) {                                       /* :1939-1943 */
      if (++tries > SMCRT_MAX_EMIT_TRIES) { C->fault = 1; break; }
      C->ctr[SMCRT_CTR_EMIT_RETRIES]++;
      emit(C, src, &pk, &rng);
    }
    if (!C->fault && (C->flags & SMCRT_FLAG_RENDER_SOURCE)) add_cell(S, C->emission, &pk, 1.0, C);  /* :1945 */
  }
  if (!C->fault) {
    uint64_t not_counted = 0;                                        /* outside packet%cnts */
    dsinfo I = eval_all(S, pk.pos, ds, &not_counted, test_kernel);   /* :1948-1952 */
    pk.layer = I.maxloc;
    if (pk.layer == 0) C->fault = 1;
  }
  if (!C->fault) {
    tauint2(C, &pk, &rng, ds, dsNew);
    uint64_t inter = 0;
    while (!pk.tflag && !C->fault) {                                 /* :1958-1975 */
      if (++inter > SMCRT_MAX_INTERACTIONS) { C->fault = 1; break; }
      double ran = ran2(&rng);
      int32_t L = pk.layer;
      if (C->flags & SMCRT_FLAG_SURVIVAL_BIAS) {                     /* :2041-2062 */
        double w_abs = pk.weight * (1.0 - S->albedo[L - 1]);
        pk.weight = pk.weight - w_abs;
        add_cell(S, C->absorb, &pk, w_abs, C);
        if (pk.weight < 0.01) {
          if (ran < 0.1) {
            pk.weight = pk.weight / 0.1;
          } else {
            pk.tflag = 1;
            status = 1;
            C->ctr[SMCRT_CTR_ABSORBED]++;
            break;
          }
        }
        scatter(C, &pk, S->hgg[L - 1], &rng);
        pk.nscatt++;
        C->nscatt += 1.0;
        C->ctr[SMCRT_CTR_SCATTERS]++;
      } else if (ran < S->albedo[L - 1]) {
        scatter(C, &pk, S->hgg[L - 1], &rng);
        pk.nscatt++;
        C->nscatt += 1.0;
        C->ctr[SMCRT_CTR_SCATTERS]++;
        if (test_kernel) {                                           /* :2142-2163 */
          uint32_t st = pk.nscatt;
          if (st >= 1 && st <= 4) {
            if (C->moments) {
              double* m = C->moments + 3 * (st - 1);
              double* m2 = C->moments + 12 + 3 * (st - 1);
              m[0] += pk.pos.x; m[1] += pk.pos.y; m[2] += pk.pos.z;
              m2[0] += pk.pos.x * pk.pos.x; m2[1] += pk.pos.y * pk.pos.y; m2[2] += pk.pos.z * pk.pos.z;
            }
          } else if (C->flags & SMCRT_FLAG_END_EARLY) {
            pk.tflag = 1;
            status = 4;
          }
        }
      } else {
        pk.tflag = 1;
        status = 1;
        C->ctr[SMCRT_CTR_ABSORBED]++;
        if (!test_kernel) add_cell(S, C->absorb, &pk, 1.0, C);       /* recordWeight(packet, 1.0) */
        break;
      }
      tauint2(C, &pk, &rng, ds, dsNew);
    }
  }
  if (C->fault) { status = 3; C->ctr[SMCRT_CTR_FAULTS]++; }
  else if (status == 0) { status = 2; C->ctr[SMCRT_CTR_ESCAPED]++; }
  C->ctr[SMCRT_CTR_PHOTONS]++;
  C->ctr[SMCRT_CTR_RNG_DRAWS] += rng.draws;
  if (rec) {
    rec->pos[0] = pk.pos.x; rec->pos[1] = pk.pos.y; rec->pos[2] = pk.pos.z;
    rec->dir[0] = pk.n.x; rec->dir[1] = pk.n.y; rec->dir[2] = pk.n.z;
    rec->weight = pk.weight;
    rec->cell[0] = pk.xcell; rec->cell[1] = pk.ycell; rec->cell[2] = pk.zcell;
    rec->layer = pk.layer;
    rec->nscatt = pk.nscatt;
    rec->bounces = pk.bounces;
    rec->draws = rng.draws;
    rec->status = status;
  }
}

/* ============================================================= entry points ===== */
static int build_scene(scene_t* S, const smcrt_sdf_node* nodes, int32_t n_nodes, const int32_t* top,
                       int32_t n_top, const smcrt_grid* grid, const smcrt_detector* dets, int32_t n_dets) {
  memset(S, 0, sizeof *S);
  if (!nodes || n_nodes < 1 || !top || n_top < 1 || !grid) return SMCRT_ERR_INVALID_ARG;
  if (grid->nx < 1 || grid->ny < 1 || grid->nz < 1) return SMCRT_ERR_INVALID_ARG;
  for (int32_t i = 0; i < n_top; ++i)
    if (top[i] < 0 || top[i] >= n_nodes) return SMCRT_ERR_INVALID_ARG;
  for (int32_t i = 0; i < n_dets; ++i)
    if (dets[i].kind == SMCRT_DET_FIBRE) return SMCRT_ERR_UNSUPPORTED;
  S->nodes = nodes; S->n_nodes = n_nodes; S->top = top; S->n_top = n_top; S->grid = *grid;
  S->dets = dets; S->n_dets = n_dets;
  S->kappa = calloc(6 * (size_t)n_top, sizeof(double));
  S->albedo = S->kappa + n_top; S->mua = S->albedo + n_top; S->hgg = S->mua + n_top;
  S->g2 = S->hgg + n_top; S->nidx = S->g2 + n_top;
  for (int32_t i = 0; i < n_top; ++i) {                              /* init_mono :107-125 */
    const smcrt_sdf_node* nd = &nodes[top[i]];
    S->kappa[i] = nd->mus + nd->mua;
    S->albedo[i] = (nd->mua < 1e-9) ? 1.0 : nd->mus / S->kappa[i];
    S->mua[i] = nd->mua; S->hgg[i] = nd->hgg; S->g2[i] = nd->hgg * nd->hgg; S->nidx[i] = nd->n;
  }
  S->xface = calloc((size_t)grid->nx + 1 + grid->ny + 1 + grid->nz + 2, sizeof(double));
  S->yface = S->xface + grid->nx + 1;
  S->zface = S->yface + grid->ny + 1;
  for (int32_t i = 0; i < grid->nx + 1; ++i) S->xface[i] = (double)i * 2.0 * grid->xmax / (double)grid->nx;  /* grid.f90:147-157 */
  for (int32_t i = 0; i < grid->ny + 1; ++i) S->yface[i] = (double)i * 2.0 * grid->ymax / (double)grid->ny;
  for (int32_t i = 0; i < grid->nz + 2; ++i) S->zface[i] = (double)i * 2.0 * grid->zmax / (double)grid->nz;
  S->det_off = calloc((size_t)n_dets + 1, sizeof(int64_t));
  for (int32_t i = 0; i < n_dets; ++i) {
    int64_t nb = dets[i].nbins;
    S->det_off[i + 1] = S->det_off[i] + (dets[i].kind == SMCRT_DET_CAMERA ? nb * nb : nb);
  }
  return SMCRT_OK;
}

static void free_scene(scene_t* S) { free(S->kappa); free(S->xface); free(S->det_off); }

/* SDF values at points (unit checks against test/SDF/test_SDF.f90) */
ORACLE_API int oracle_sdf_eval(const smcrt_sdf_node* nodes, int32_t n_nodes, int32_t node,
                               const double* pts, int64_t n_pts, double* out) {
  scene_t S;
  memset(&S, 0, sizeof S);
  S.nodes = nodes; S.n_nodes = n_nodes;
  if (node < 0 || node >= n_nodes) return SMCRT_ERR_INVALID_ARG;
  for (int64_t i = 0; i < n_pts; ++i)
    out[i] = sdf_eval_node(&S, node, v3(pts[3 * i], pts[3 * i + 1], pts[3 * i + 2]), 0);
  return SMCRT_OK;
}

ORACLE_API int oracle_calc_normal(const smcrt_sdf_node* nodes, int32_t n_nodes, int32_t node,
                                  const double* p, double* n) {
  scene_t S;
  memset(&S, 0, sizeof S);
  int32_t top = node;
  S.nodes = nodes; S.n_nodes = n_nodes; S.top = &top; S.n_top = 1;
  vec3 r = calc_normal(&S, v3(p[0], p[1], p[2]), 0);
  n[0] = r.x; n[1] = r.y; n[2] = r.z;
  return SMCRT_OK;
}

/* the photon loop of run_MCRT (serial, photon order), accumulating into `io` */
ORACLE_API int oracle_run(const smcrt_sdf_node* nodes, int32_t n_nodes, const int32_t* top, int32_t n_top,
                          const smcrt_grid* grid, const smcrt_detector* dets, int32_t n_dets,
                          const smcrt_source* src, const smcrt_run_config* cfg, smcrt_tallies* io) {
  scene_t S;
  int st = build_scene(&S, nodes, n_nodes, top, n_top, grid, dets, n_dets);
  if (st) return st;
  if (!src || !cfg || !io ||
      (src->kind != SMCRT_SRC_POINT && src->kind != SMCRT_SRC_UNIFORM && src->kind != SMCRT_SRC_PENCIL)) {
    free_scene(&S);
    return SMCRT_ERR_INVALID_ARG;
  }
  int64_t nv = (int64_t)grid->nx * grid->ny * grid->nz;
  ctx_t C;
  memset(&C, 0, sizeof C);
  C.S = &S;
  C.flags = cfg->flags;
  C.jmean = (io->jmean || io->jmean_f64) ? calloc((size_t)nv, sizeof(double)) : NULL;
  C.absorb = (io->absorb || io->absorb_f64) ? calloc((size_t)nv, sizeof(double)) : NULL;
  C.emission = (io->emission || io->emission_f64) ? calloc((size_t)nv, sizeof(double)) : NULL;
  C.det = io->det_bins;
  C.moments = io->moments;
  double* ds = calloc(2 * (size_t)n_top, sizeof(double));
  for (uint64_t j = 0; j < cfg->n_photons; ++j) {
    smcrt_photon_record* rec = (io->records && (cfg->flags & SMCRT_FLAG_RECORD_PHOTONS)) ? &io->records[j] : NULL;
    run_photon(&C, src, cfg->first_photon + j, cfg->seed, ds, ds + n_top, rec);
  }
  double* g[3] = {C.jmean, C.absorb, C.emission};
  float* gf[3] = {io->jmean, io->absorb, io->emission};
  double* gd[3] = {io->jmean_f64, io->absorb_f64, io->emission_f64};
  for (int t = 0; t < 3; ++t) {
    if (!g[t]) continue;
    for (int64_t i = 0; i < nv; ++i) {
      if (gf[t]) gf[t][i] = (float)((double)gf[t][i] + g[t][i]);
      if (gd[t]) gd[t][i] += g[t][i];
    }
    free(g[t]);
  }
  if (io->nscatt) *io->nscatt += C.nscatt;
  if (io->counters)
    for (int i = 0; i < SMCRT_NCOUNTERS; ++i) io->counters[i] += C.ctr[i];
  free(ds);
  free_scene(&S);
  return SMCRT_OK;
}

/* one record_hit call on a single detector (unit checks against test/detector) */
ORACLE_API int oracle_record_hit(const smcrt_detector* det, const double start[3], const double dir[3],
                                 double pointSep, int32_t layer, double weight, double* bins, uint64_t* hits) {
  scene_t S;
  memset(&S, 0, sizeof S);
  int64_t off[2] = {0, 0};
  S.dets = det; S.n_dets = 1; S.det_off = off;
  ctx_t C;
  memset(&C, 0, sizeof C);
  C.S = &S;
  C.det = bins;
  record_hits(&C, v3(start[0], start[1], start[2]), v3(dir[0], dir[1], dir[2]), pointSep, layer, weight);
  if (hits) *hits = C.ctr[SMCRT_CTR_DETECTOR_HITS];
  return SMCRT_OK;
}
