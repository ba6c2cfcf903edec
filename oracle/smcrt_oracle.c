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
 *   emitters              src/photon.f90:159-1043 (every source: point, uniform, pencil,
 *                         circular, focus, annulus, dslit, aperture, slm, ...)
 *   source spectra        src/piecewise.f90 (constant, 1-D and 2-D piecewise)
 *   spectral optical props src/opticalProps/opticalProperties.f90:127-201 (init_spectral,
 *                         updateSpectral; oracle_spectral_sample below)
 *   scatter               src/photon.f90:1045-1103
 *   detectors             src/detectors/detector_base.f90:137-235, detectors.f90:147-469,
 *                         src/geometryMod.f90:217-270 (circle, annulus, camera, fibre)
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

/* atan, fdlibm s_atan.c (Sun Microsystems, 1993): the fibre detector's acceptance angle */
ORACLE_API double oracle_atan(double x) {
  static const double atanhi[4] = {4.63647609000806093515e-01, 7.85398163397448278999e-01,
                                   9.82793723247329054082e-01, 1.57079632679489655800e+00};
  static const double atanlo[4] = {2.26987774529616870924e-17, 3.06161699786838301793e-17,
                                   1.39033110312309984516e-17, 6.12323399573676603587e-17};
  static const double aT[11] = {3.33333333333329318027e-01, -1.99999999998764832476e-01,
                                1.42857142725034663711e-01, -1.11111104054623557880e-01,
                                9.09088713343650656196e-02, -7.69187620504482999495e-02,
                                6.66107313738753120669e-02, -5.83357013379057348645e-02,
                                4.97687799461593236017e-02, -3.65315727442169155270e-02,
                                1.62858201153657823623e-02};
  uint64_t u = d2u(x);
  int32_t hx = (int32_t)(u >> 32);
  uint32_t ix = (uint32_t)hx & 0x7fffffffu;
  int id;
  if (ix >= 0x44100000u) {
    if (ix > 0x7ff00000u || (ix == 0x7ff00000u && (uint32_t)u != 0u)) return x + x;
    return hx > 0 ? atanhi[3] + atanlo[3] : -atanhi[3] - atanlo[3];
  }
  if (ix < 0x3fdc0000u) {
    if (ix < 0x3e200000u) return x;
    id = -1;
  } else {
    x = fabs(x);
    if (ix < 0x3ff30000u) {
      if (ix < 0x3fe60000u) { id = 0; x = (2.0 * x - 1.0) / (2.0 + x); }
      else { id = 1; x = (x - 1.0) / (x + 1.0); }
    } else if (ix < 0x40038000u) {
      id = 2; x = (x - 1.5) / (1.0 + 1.5 * x);
    } else {
      id = 3; x = -1.0 / x;
    }
  }
  double z = x * x, w = z * z;
  double s1 = z * (aT[0] + w * (aT[2] + w * (aT[4] + w * (aT[6] + w * (aT[8] + w * aT[10])))));
  double s2 = w * (aT[1] + w * (aT[3] + w * (aT[5] + w * (aT[7] + w * aT[9]))));
  if (id < 0) return x - x * (s1 + s2);
  z = atanhi[id] - ((x * (s1 + s2) - atanlo[id]) - x);
  return hx < 0 ? -z : z;
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
/* composites (models, modifiers) nest at most this many levels below a top, as the engine
 * accepts (geometry.h PROG_MAX_DEPTH); the reference's recursion has no limit */
#define ORACLE_MAX_NEST 32

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

/* sin and cos of a twist/bend/displacement angle of any sign: sin(-x) = -sin(x), cos(-x) =
 * cos(x), then oracle_sincos's reduction (the device's det_sincos_any, detmath.h) */
static void oracle_sincos_any(double x, double* s, double* c) {
  oracle_sincos(fabs(x), s, c);
  if (x < 0.0) *s = -*s;
}

static double sdf_eval_node(const scene_t* S, int32_t idx, vec3 pos, int depth) {
  const smcrt_sdf_node* nd = &S->nodes[idx];
  const double* P = nd->param;
  if (nd->kind == SMCRT_SDF_MODEL) {                                     /* eval_model sdf_base.f90:146-161 */
    if (depth >= ORACLE_MAX_NEST || nd->n_children < 1) return NAN;
    double res = sdf_eval_node(S, nd->first_child, pos, depth + 1);
    for (int32_t i = 1; i < nd->n_children; ++i)
      res = csg(nd->op, res, sdf_eval_node(S, nd->first_child + i, pos, depth + 1), nd->k);
    return res;
  }
  if (nd->kind > SMCRT_SDF_MODEL) {  /* the modifiers of sdfModifiers.f90: one wrapped node, own transform unused */
    if (depth >= ORACLE_MAX_NEST || nd->n_children != 1) return NAN;
    const int32_t ch = nd->first_child;
    switch (nd->kind) {
      case SMCRT_SDF_REVOLUTION: {                                       /* eval_revolution :303-321 */
        vec3 pin = vsub(pos, v3(P[1], P[2], P[3]));
        vec3 pxz = v3(pin.x, 0.0, pin.z);
        return sdf_eval_node(S, ch, v3(vlen(pxz) - P[0], pin.y, 0.0), depth + 1);
      }
      case SMCRT_SDF_EXTRUDE: {                                          /* eval_extrude :286-301 */
        double d = sdf_eval_node(S, ch, pos, depth + 1);
        vec3 w = v3(d, fabs(pos.z) - P[0], 0.0);
        return fmind(fmaxd(w.x, w.y), 0.0) + vlen(vmaxs(w, 0.0));
      }
      case SMCRT_SDF_ONION:                                              /* eval_onion :323-333 */
        return fabs(sdf_eval_node(S, ch, pos, depth + 1)) - P[0];
      case SMCRT_SDF_ELONGATE: {                                         /* eval_elongate :335-351 */
        vec3 q = vsub(vabs(pos), v3(P[0], P[1], P[2]));
        double w = fmind(fmaxd(q.x, fmaxd(q.y, q.z)), 0.0);
        return sdf_eval_node(S, ch, vmaxs(q, 0.0), depth + 1) + w;
      }
      case SMCRT_SDF_TWIST:                                              /* eval_twist :353-371 */
      case SMCRT_SDF_BEND: {                                             /* eval_bend :373-391 */
        double s, c;
        oracle_sincos_any(P[0] * (nd->kind == SMCRT_SDF_TWIST ? pos.z : pos.x), &s, &c);
        double x2 = c * pos.x - s * pos.y;
        double y2 = s * pos.x + c * pos.y;
        return sdf_eval_node(S, ch, v3(x2, y2, pos.z), depth + 1);
      }
      case SMCRT_SDF_DISPLACEMENT: {                                     /* eval_disp :393-408, built-in f */
        double d1 = sdf_eval_node(S, ch, pos, depth + 1);
        double sx, sy, sz, c;
        oracle_sincos_any(P[2] * pos.x, &sx, &c);
        oracle_sincos_any(P[3] * pos.y, &sy, &c);
        oracle_sincos_any(P[4] * pos.z, &sz, &c);
        return d1 + ((P[1] * sx) * sy) * sz;
      }
      default:
        return NAN;
    }
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
  const struct src_plan* plan; /* general emitter (sources beyond point/uniform/pencil, spectra) */
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
    else if (D->kind == SMCRT_DET_FIBRE) {                           /* detectors.f90:331-393 */
      const double* F = D->fibre;  /* f1, f2, f1Ap, f2Ap, frontOff, backOff, front2pin, pin2back, pinAp, accept, core */
      int hit = intersect_circle(ddir, vadd(dpos, vmul(ddir, F[4])), F[2], start, dir, &t, &value1D);
      if (hit && (t <= 0.0 || t > pointSep)) hit = 0;
      if (hit) {
        double costt = vdot(ddir, dir);
        if (costt > 1.0) costt = 1.0;
        double sintt = sqrt(1.0 - costt * costt);
        double gradient = sintt / costt;
        double radius = value1D;
        gradient = -radius / F[0] + gradient;                         /* thin lens 1 */
        radius = radius + gradient * F[6];                            /* to the pinhole */
        if (radius > F[8]) {
          hit = 0;
        } else {
          radius = radius + gradient * F[7];                          /* to lens 2 */
          if (radius > F[3]) {
            hit = 0;
          } else {
            gradient = -radius / F[1] + gradient;
            radius = radius + gradient * F[5];                        /* to the fibre */
            double angle = fabs(oracle_atan(gradient)) * 360.0 / 6.283185307179586;
            if (angle > F[9] || radius > (F[10] / 2.0)) hit = 0;
            value1D = fabs(radius);
          }
        }
      }
      if (hit) {
        int64_t idx = f_nint(value1D / D->bin_wid) + 1;
        if (idx > D->nbins) idx = D->nbins;
        if (idx >= 1) { if (data) data[idx - 1] += weight; C->ctr[SMCRT_CTR_DETECTOR_HITS]++; }
      }
    }
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

/* ======================================================= general emitter (f3) ===== */
/* The remaining sources of photon.f90 and the source spectrum of piecewise.f90. The
 * per-run constants (rotation/translation matrices, CDFs) are computed once per run with the
 * reference's operations in its order; the per-photon part follows each subroutine. */
typedef double m4[4][4]; /* m[r][c] = Fortran t(r+1, c+1) */

static void m4_identity(m4 a) { memset(a, 0, sizeof(m4)); for (int i = 0; i < 4; ++i) a[i][i] = 1.0; }
static void m4_matmul(const m4 A, const m4 B, m4 C) {                /* matmul intrinsic, k ascending */
  m4 T;
  for (int i = 0; i < 4; ++i)
    for (int j = 0; j < 4; ++j) {
      double acc = 0.0;
      for (int k = 0; k < 4; ++k) acc = acc + A[i][k] * B[k][j];
      T[i][j] = acc;
    }
  memcpy(C, T, sizeof(m4));
}
/* invert(translate(o)) with mat_class.f90:154-207's direct inverse, written out for a
 * translation (rows 1-3 identity, row 4 = o): the same products, most of them with 0/1 */
static void m4_invert(const m4 M, m4 B) {                            /* mat_class.f90:154-207 */
#define A(i, j) M[(i)-1][(j)-1]
  double detinv = 1.0 / (A(1,1)*(A(2,2)*(A(3,3)*A(4,4)-A(3,4)*A(4,3))+A(2,3)*(A(3,4)*A(4,2)-A(3,2)*A(4,4))+A(2,4)*(A(3,2)*A(4,3)-A(3,3)*A(4,2)))
                       - A(1,2)*(A(2,1)*(A(3,3)*A(4,4)-A(3,4)*A(4,3))+A(2,3)*(A(3,4)*A(4,1)-A(3,1)*A(4,4))+A(2,4)*(A(3,1)*A(4,3)-A(3,3)*A(4,1)))
                       + A(1,3)*(A(2,1)*(A(3,2)*A(4,4)-A(3,4)*A(4,2))+A(2,2)*(A(3,4)*A(4,1)-A(3,1)*A(4,4))+A(2,4)*(A(3,1)*A(4,2)-A(3,2)*A(4,1)))
                       - A(1,4)*(A(2,1)*(A(3,2)*A(4,3)-A(3,3)*A(4,2))+A(2,2)*(A(3,3)*A(4,1)-A(3,1)*A(4,3))+A(2,3)*(A(3,1)*A(4,2)-A(3,2)*A(4,1))));
  B[0][0] = detinv*(A(2,2)*(A(3,3)*A(4,4)-A(3,4)*A(4,3))+A(2,3)*(A(3,4)*A(4,2)-A(3,2)*A(4,4))+A(2,4)*(A(3,2)*A(4,3)-A(3,3)*A(4,2)));
  B[1][0] = detinv*(A(2,1)*(A(3,4)*A(4,3)-A(3,3)*A(4,4))+A(2,3)*(A(3,1)*A(4,4)-A(3,4)*A(4,1))+A(2,4)*(A(3,3)*A(4,1)-A(3,1)*A(4,3)));
  B[2][0] = detinv*(A(2,1)*(A(3,2)*A(4,4)-A(3,4)*A(4,2))+A(2,2)*(A(3,4)*A(4,1)-A(3,1)*A(4,4))+A(2,4)*(A(3,1)*A(4,2)-A(3,2)*A(4,1)));
  B[3][0] = detinv*(A(2,1)*(A(3,3)*A(4,2)-A(3,2)*A(4,3))+A(2,2)*(A(3,1)*A(4,3)-A(3,3)*A(4,1))+A(2,3)*(A(3,2)*A(4,1)-A(3,1)*A(4,2)));
  B[0][1] = detinv*(A(1,2)*(A(3,4)*A(4,3)-A(3,3)*A(4,4))+A(1,3)*(A(3,2)*A(4,4)-A(3,4)*A(4,2))+A(1,4)*(A(3,3)*A(4,2)-A(3,2)*A(4,3)));
  B[1][1] = detinv*(A(1,1)*(A(3,3)*A(4,4)-A(3,4)*A(4,3))+A(1,3)*(A(3,4)*A(4,1)-A(3,1)*A(4,4))+A(1,4)*(A(3,1)*A(4,3)-A(3,3)*A(4,1)));
  B[2][1] = detinv*(A(1,1)*(A(3,4)*A(4,2)-A(3,2)*A(4,4))+A(1,2)*(A(3,1)*A(4,4)-A(3,4)*A(4,1))+A(1,4)*(A(3,2)*A(4,1)-A(3,1)*A(4,2)));
  B[3][1] = detinv*(A(1,1)*(A(3,2)*A(4,3)-A(3,3)*A(4,2))+A(1,2)*(A(3,3)*A(4,1)-A(3,1)*A(4,3))+A(1,3)*(A(3,1)*A(4,2)-A(3,2)*A(4,1)));
  B[0][2] = detinv*(A(1,2)*(A(2,3)*A(4,4)-A(2,4)*A(4,3))+A(1,3)*(A(2,4)*A(4,2)-A(2,2)*A(4,4))+A(1,4)*(A(2,2)*A(4,3)-A(2,3)*A(4,2)));
  B[1][2] = detinv*(A(1,1)*(A(2,4)*A(4,3)-A(2,3)*A(4,4))+A(1,3)*(A(2,1)*A(4,4)-A(2,4)*A(4,1))+A(1,4)*(A(2,3)*A(4,1)-A(2,1)*A(4,3)));
  B[2][2] = detinv*(A(1,1)*(A(2,2)*A(4,4)-A(2,4)*A(4,2))+A(1,2)*(A(2,4)*A(4,1)-A(2,1)*A(4,4))+A(1,4)*(A(2,1)*A(4,2)-A(2,2)*A(4,1)));
  B[3][2] = detinv*(A(1,1)*(A(2,3)*A(4,2)-A(2,2)*A(4,3))+A(1,2)*(A(2,1)*A(4,3)-A(2,3)*A(4,1))+A(1,3)*(A(2,2)*A(4,1)-A(2,1)*A(4,2)));
  B[0][3] = detinv*(A(1,2)*(A(2,4)*A(3,3)-A(2,3)*A(3,4))+A(1,3)*(A(2,2)*A(3,4)-A(2,4)*A(3,2))+A(1,4)*(A(2,3)*A(3,2)-A(2,2)*A(3,3)));
  B[1][3] = detinv*(A(1,1)*(A(2,3)*A(3,4)-A(2,4)*A(3,3))+A(1,3)*(A(2,4)*A(3,1)-A(2,1)*A(3,4))+A(1,4)*(A(2,1)*A(3,3)-A(2,3)*A(3,1)));
  B[2][3] = detinv*(A(1,1)*(A(2,4)*A(3,2)-A(2,2)*A(3,4))+A(1,2)*(A(2,1)*A(3,4)-A(2,4)*A(3,1))+A(1,4)*(A(2,2)*A(3,1)-A(2,1)*A(3,2)));
  B[3][3] = detinv*(A(1,1)*(A(2,2)*A(3,3)-A(2,3)*A(3,2))+A(1,2)*(A(2,3)*A(3,1)-A(2,1)*A(3,3))+A(1,3)*(A(2,1)*A(3,2)-A(2,2)*A(3,1)));
#undef A
}
static void m4_translate(vec3 o, m4 a) { m4_identity(a); a[3][0] = o.x; a[3][1] = o.y; a[3][2] = o.z; } /* sdfHelpers.f90:169-182 */
static vec3 vcross(vec3 a, vec3 b) { return v3(a.y * b.z - a.z * b.y, -a.x * b.z + a.z * b.x, a.x * b.y - a.y * b.x); }
static vec3 vmagnitude(vec3 a) { double t = vlen(a); return v3(a.x / t, a.y / t, a.z / t); }  /* vector_class.f90:392-402 */
static int veq(vec3 a, vec3 b) { return a.x == b.x && a.y == b.y && a.z == b.z; }
static void rotation_align(vec3 a, vec3 b, m4 r) {                   /* sdfHelpers.f90:114-140 */
  vec3 v = vcross(a, b);
  double c = vdot(a, b);
  double k = 1.0 / (1.0 + c);
  m4 vx, vx2, I;
  memset(vx, 0, sizeof vx);
  vx[1][0] = -1.0 * v.z; vx[2][0] = v.y;
  vx[0][1] = v.z;        vx[2][1] = -1.0 * v.x;
  vx[0][2] = -1.0 * v.y; vx[1][2] = v.x;
  m4_matmul(vx, vx, vx2);
  m4_identity(I);
  for (int i = 0; i < 4; ++i)
    for (int j = 0; j < 4; ++j) r[i][j] = (I[i][j] + vx[i][j]) + vx2[i][j] * k;
}
static void m4_colmajor(const m4 a, double* o) { for (int c = 0; c < 4; ++c) for (int r = 0; r < 4; ++r) o[c * 4 + r] = a[r][c]; }

typedef struct src_plan {
  smcrt_source src;
  int spec_kind;
  int circ_z;
  double T[16], R[16];
  double wavelength;
  int64_t n;         /* 1-D rows / 2-D CDF entries */
  double* x;         /* 1-D abscissae */
  double* cdf;
  int32_t xoff, yoff;
  double cw, ch;
} src_plan_t;

static uint32_t pack_bits(uint64_t x) {                              /* piecewise.f90:296-315 */
  x &= 0x5555555555555555ull;
  x = (x >> 1) | x; x &= 0x3333333333333333ull;
  x = (x >> 2) | x; x &= 0x0F0F0F0F0F0F0F0Full;
  x = (x >> 4) | x; x &= 0x00FF00FF00FF00FFull;
  x = (x >> 8) | x; x &= 0x0000FFFF0000FFFFull;
  x = (x >> 16) | x;
  return (uint32_t)x;
}
static int32_t nextpwr2(int32_t v) {                                 /* piecewise.f90:238-252 */
  uint32_t r = (uint32_t)v - 1u;
  r |= r >> 1; r |= r >> 2; r |= r >> 4; r |= r >> 8; r |= r >> 16;
  return (int32_t)(r + 1u);
}

static void free_plan(src_plan_t* P) { free(P->x); free(P->cdf); P->x = P->cdf = NULL; }

static int build_plan(src_plan_t* P, const smcrt_source* s) {
  memset(P, 0, sizeof *P);
  P->src = *s;
  P->wavelength = 500.0;                                             /* parse_spectrum.f90:55 */
  m4 T, R;
  m4_identity(T); m4_identity(R);
  if (s->kind == SMCRT_SRC_CIRCULAR) {                               /* photon.f90:239-264 */
    vec3 a = vmagnitude(v3(1.0, 0.0, 0.0));
    vec3 b = vmagnitude(v3(s->dir[0], s->dir[1], s->dir[2]));
    if (veq(vabs(a), vabs(b))) { a = vmagnitude(v3(0.0, 0.0, 1.0)); P->circ_z = 1; }
    m4 ra, tr, inv;
    rotation_align(a, b, ra);
    m4_translate(v3(s->pos[0], s->pos[1], s->pos[2]), tr);
    m4_invert(tr, inv);
    m4_matmul(ra, inv, T);
  } else if (s->kind == SMCRT_SRC_FOCUS || s->kind == SMCRT_SRC_ANNULUS) {  /* :445-485, :917-957 */
    if (s->kind == SMCRT_SRC_FOCUS && s->beam != SMCRT_BEAM_SQUARE && s->beam != SMCRT_BEAM_CIRCLE &&
        s->beam != SMCRT_BEAM_GAUSSIAN) return SMCRT_ERR_INVALID_ARG;
    if (s->kind == SMCRT_SRC_ANNULUS && s->beam != SMCRT_BEAM_TOPHAT && s->beam != SMCRT_BEAM_BESSEL &&
        s->beam != SMCRT_BEAM_GAUSSIAN) return SMCRT_ERR_INVALID_ARG;
    vec3 rot = v3(s->rotation[0], s->rotation[1], s->rotation[2]);
    if (vlen(rot) < 1e-8) return SMCRT_ERR_INVALID_ARG;              /* parse_source.f90:84-88 */
    vec3 a = vmagnitude(v3(0.0, 0.0, -1.0)), b = vmagnitude(rot);
    vec3 start = v3(-s->pos[0], -s->pos[1], -s->pos[2]);
    m4 t;
    int flip = veq(vabs(a), vabs(b));
    if (veq(a, b)) m4_identity(t);
    else if (flip) { m4_identity(t); t[2][2] = -1.0; }
    else rotation_align(a, b, t);
    memcpy(R, t, sizeof(m4));
    if (flip && !veq(a, b)) t[2][2] = 1.0;
    m4 tr, inv;
    m4_translate(start, tr);
    m4_invert(tr, inv);
    m4_matmul(t, inv, T);
  } else if (s->kind < SMCRT_SRC_POINT || s->kind > SMCRT_SRC_APERTURE) {
    return SMCRT_ERR_INVALID_ARG;
  }
  m4_colmajor(T, P->T);
  m4_colmajor(R, P->R);
  const smcrt_spectrum* sp = s->spectrum;
  P->spec_kind = sp ? sp->kind : SMCRT_SPEC_CONSTANT;
  if (sp && sp->kind == SMCRT_SPEC_CONSTANT) {
    P->wavelength = sp->wavelength;
  } else if (sp && sp->kind == SMCRT_SPEC_1D) {                      /* init_piecewise1D :140-168 */
    int64_t n = sp->n;
    if (n < 2 || !sp->array) return SMCRT_ERR_INVALID_ARG;
    const double* x = sp->array;
    const double* y = sp->array + n;
    P->x = malloc((size_t)n * sizeof(double));
    P->cdf = calloc((size_t)n, sizeof(double));
    memcpy(P->x, x, (size_t)n * sizeof(double));
    double sumer = 0.0;
    for (int64_t i = 1; i < n; ++i) {                                /* do i = 2, length */
      /* trapz_weights (stdlib): ends 0.5*(x2-x1), 0.5*(xn-xn-1); inside 0.5*(x(i+1)-x(i-1)) */
      double w = (n == 2 || i == n - 1) ? 0.5 * (x[n - 1] - x[n - 2]) : 0.5 * (x[i + 1] - x[i - 1]);
      sumer = sumer + w * y[i];
      P->cdf[i] = sumer;
    }
    double last = P->cdf[n - 1];
    for (int64_t i = 0; i < n; ++i) P->cdf[i] = P->cdf[i] / last;
    P->n = n;
  } else if (sp && sp->kind == SMCRT_SPEC_2D) {                      /* init_piecewise2D :190-236 */
    int32_t width = sp->width, height = sp->height;
    if (width < 1 || height < 1 || !sp->image) return SMCRT_ERR_INVALID_ARG;
    int32_t w2 = nextpwr2(width), h2 = nextpwr2(height);
    P->xoff = (h2 - height) / 2;
    P->yoff = (w2 - width) / 2;
    int32_t x0 = P->xoff > 0 ? P->xoff - 1 : 0, y0 = P->yoff > 0 ? P->yoff - 1 : 0;
    if (x0 + width > w2 || y0 + height > h2) return SMCRT_ERR_INVALID_ARG;
    int64_t N = (int64_t)w2 * h2;
    double* img = calloc((size_t)N, sizeof(double));
    for (int32_t j = 0; j < height; ++j)
      for (int32_t i = 0; i < width; ++i)
        img[(size_t)(x0 + i) + (size_t)w2 * (size_t)(y0 + j)] = sp->image[(size_t)i + (size_t)width * j];
    P->cdf = calloc((size_t)N, sizeof(double));
    for (int64_t i = 0; i < N; ++i) {
      uint64_t li = (uint64_t)pack_bits((uint64_t)i) + (uint64_t)w2 * pack_bits((uint64_t)i >> 1);
      double h = li < (uint64_t)N ? img[li] : 0.0;
      P->cdf[i] = i == 0 ? h : P->cdf[i - 1] + h;
    }
    free(img);
    double last = P->cdf[N - 1];
    for (int64_t i = 0; i < N; ++i) P->cdf[i] = P->cdf[i] / last;
    P->n = N;
    P->cw = sp->cell_width; P->ch = sp->cell_height;
  } else if (sp) {
    return SMCRT_ERR_INVALID_ARG;
  }
  if (s->kind == SMCRT_SRC_SLM && P->spec_kind == SMCRT_SPEC_1D) { free_plan(P); return SMCRT_ERR_INVALID_ARG; }
  return SMCRT_OK;
}

static int64_t search_1d(const double* a, int64_t n, double v) {     /* piecewise.f90:254-275 */
  int64_t nup = n, nlow = 1;
  while ((nup - nlow) > 1) {
    int64_t middle = (int64_t)((float)(nup + nlow) / 2.0f);            /* int((nup+nlow)/2.), default real */
    if (v > a[middle - 1]) nlow = middle; else nup = middle;
  }
  return nlow;
}
static double ranu(rng_t* r, double a, double b) { return a + ran2(r) * (b - a); }  /* random_mod.f90:93-103 */

static void spec_sample(const src_plan_t* P, rng_t* r, double* x, double* y) {
  if (P->spec_kind == SMCRT_SPEC_1D) {                               /* sample1D :109-137 */
    double val = ran2(r);
    int64_t i = search_1d(P->cdf, P->n, val);
    *x = P->x[i - 1] + ((val - P->cdf[i - 1]) * (P->x[i] - P->x[i - 1])) / (P->cdf[i] - P->cdf[i - 1]);
    *y = 0.0;
  } else if (P->spec_kind == SMCRT_SPEC_2D) {                        /* sample2D :171-188 */
    double val = ran2(r);
    int64_t i = search_1d(P->cdf, P->n, val);
    int32_t xr = (int32_t)pack_bits((uint64_t)i), yr = (int32_t)pack_bits((uint64_t)i >> 1);
    *x = (double)(xr - P->xoff) + ranu(r, -P->cw, P->cw);
    *y = (double)(yr - P->yoff) + ranu(r, -P->ch, P->ch);
  } else {                                                           /* getValue :93-107 */
    *x = P->wavelength;
    *y = -9999.0;
  }
}

static void nudge(const scene_t* S, vec3* p) {                       /* e.g. photon.f90:614-628 */
  const double xmax = S->grid.xmax, ymax = S->grid.ymax, zmax = S->grid.zmax;
  if (p->x == -xmax) p->x = p->x + 7.9e-7; else if (p->x == xmax) p->x = p->x - 7.9e-7;
  if (p->y == -ymax) p->y = p->y + 7.9e-7; else if (p->y == ymax) p->y = p->y - 7.9e-7;
  if (p->z == -zmax) p->z = p->z + 7.9e-7; else if (p->z == zmax) p->z = p->z - 7.9e-7;
}

static void emit_ext(ctx_t* C, packet_t* pk, rng_t* rng) {
  const scene_t* S = C->S;
  const src_plan_t* P = C->plan;
  const smcrt_source* s = &P->src;
  const double TWOPI = 6.283185307179586;
  double wl, tmp;
  switch (s->kind) {
    case SMCRT_SRC_POINT: {                                          /* photon.f90:311-359 */
      pk->pos = v3(s->pos[0], s->pos[1], s->pos[2]);
      double phi = ran2(rng) * TWOPI, sinp, cosp;
      oracle_sincos(phi, &sinp, &cosp);
      double cost = 2.0 * ran2(rng) - 1.0;
      double sint = sqrt(1.0 - cost * cost);
      pk->n = v3(sint * cosp, sint * sinp, cost);
      pk->layer = 1;
      spec_sample(P, rng, &wl, &tmp);
      break;
    }
    case SMCRT_SRC_UNIFORM: {                                        /* :566-649 */
      double rx = ran2(rng), ry = ran2(rng);
      pk->n = v3(s->dir[0], s->dir[1], s->dir[2]);
      pk->pos = v3(s->p1[0] + rx * s->p2[0] + ry * s->p3[0], s->p1[1] + rx * s->p2[1] + ry * s->p3[1],
                   s->p1[2] + rx * s->p2[2] + ry * s->p3[2]);
      nudge(S, &pk->pos);
      spec_sample(P, rng, &wl, &tmp);
      break;
    }
    case SMCRT_SRC_PENCIL: {                                         /* :652-710 */
      pk->pos = v3(s->pos[0], s->pos[1], s->pos[2]);
      nudge(S, &pk->pos);
      pk->n = v3(s->dir[0], s->dir[1], s->dir[2]);
      pk->layer = 1;
      spec_sample(P, rng, &wl, &tmp);
      break;
    }
    case SMCRT_SRC_CIRCULAR: {                                       /* :214-308 */
      pk->n = v3(s->dir[0], s->dir[1], s->dir[2]);
      double r = s->radius * sqrt(ran2(rng));
      double theta = ran2(rng) * TWOPI, st, ct;
      oracle_sincos(theta, &st, &ct);
      vec3 q = P->circ_z ? v3(r * ct, r * st, 0.0) : v3(0.0, r * ct, r * st);
      vec3 t = vdotmat(q, P->T);
      pk->pos = v3(-t.x, -t.y, -t.z);
      nudge(S, &pk->pos);
      spec_sample(P, rng, &wl, &tmp);
      pk->layer = 1;
      break;
    }
    case SMCRT_SRC_FOCUS:                                            /* :361-563 */
    case SMCRT_SRC_ANNULUS: {                                        /* :850-1043 */
      vec3 q, qd;
      if (s->kind == SMCRT_SRC_FOCUS) {
        if (s->beam == SMCRT_BEAM_SQUARE) {
          double x = ranu(rng, -s->beam_size, s->beam_size);
          double y = ranu(rng, -s->beam_size, s->beam_size);
          q = v3(x, y, 0.0);
        } else {
          double radius = s->beam == SMCRT_BEAM_CIRCLE ? s->beam_size * sqrt(ran2(rng))
                                                       : s->beam_size * sqrt(-oracle_log(1.0 - ran2(rng)));
          double phi = TWOPI * ran2(rng), sinp, cosp;
          oracle_sincos(phi, &sinp, &cosp);
          q = v3(radius * cosp, radius * sinp, 0.0);
        }
        qd = q;
      } else {
        double radius, mid;
        if (s->beam == SMCRT_BEAM_TOPHAT) {
          radius = sqrt(s->rlo * s->rlo + (s->rhi * s->rhi - s->rlo * s->rlo) * ran2(rng));
          mid = (s->rhi + s->rlo) / 2.0;
        } else if (s->beam == SMCRT_BEAM_BESSEL) {
          radius = s->rlo + (s->rhi - s->rlo) * ran2(rng);
          mid = (s->rhi + s->rlo) / 2.0;
        } else {                                                     /* rang, random_mod.f90:105-127 */
          mid = (s->rhi + s->rlo) / 2.0;
          double x = 0.0, y = 0.0, sq = 1.0;
          int tries = 0;
          while (sq >= 1.0) {
            if (++tries > 1000) { C->fault = 1; break; }
            x = ranu(rng, -1.0, 1.0);
            y = ranu(rng, -1.0, 1.0);
            sq = y * y + x * x;
          }
          radius = mid + s->sigma * (x * sqrt(-2.0 * oracle_log(sq) / sq));
        }
        double phi = TWOPI * ran2(rng), sinp, cosp;
        oracle_sincos(phi, &sinp, &cosp);
        q = v3(radius * cosp, radius * sinp, 0.0);
        qd = v3(mid * cosp, mid * sinp, 0.0);
      }
      /* dir = magnitude(sign(1,f)*((-1)*(q - targ)/dist)), rotated, renormalised */
      vec3 d0 = vsub(qd, v3(0.0, 0.0, -s->focal_length));
      double dist = vlen(d0);
      vec3 d = smul(-1.0, d0);
      d = v3(d.x / dist, d.y / dist, d.z / dist);
      d = vmul(d, copysign(1.0, s->focal_length));
      d = vmagnitude(d);
      pk->n = vmagnitude(vdotmat(d, P->R));
      pk->pos = vdotmat(q, P->T);
      spec_sample(P, rng, &wl, &tmp);
      /* step into the grid, photon.f90:505-556 (focus: counter > 4; annulus :985-1036: > 3) */
      int cap = s->kind == SMCRT_SRC_FOCUS ? 4 : 3;
      int inX = 0, inY = 0, inZ = 0, tX = 0, tY = 0, tZ = 0, counter = 0;
      const double xmax = S->grid.xmax, ymax = S->grid.ymax, zmax = S->grid.zmax;
      vec3* p = &pk->pos;
      vec3 dd = pk->n;
      while (!inX || !inY || !inZ) {
        double st;
        if (p->x <= -xmax) { st = (-xmax - p->x + 9e-7) / dd.x; *p = v3(p->x + dd.x * st, p->y + dd.y * st, p->z + dd.z * st); tX = 1; }
        else if (p->x >= xmax) { st = (xmax - p->x - 9e-7) / dd.x; *p = v3(p->x + dd.x * st, p->y + dd.y * st, p->z + dd.z * st); tX = 1; }
        else inX = 1;
        if (p->y <= -ymax) { st = (-ymax - p->y + 9e-7) / dd.y; *p = v3(p->x + dd.x * st, p->y + dd.y * st, p->z + dd.z * st); tY = 1; }
        else if (p->y >= ymax) { st = (ymax - p->y - 9e-7) / dd.y; *p = v3(p->x + dd.x * st, p->y + dd.y * st, p->z + dd.z * st); tY = 1; }
        else inY = 1;
        if (p->z <= -zmax) { st = (-zmax - p->z + 9e-7) / dd.z; *p = v3(p->x + dd.x * st, p->y + dd.y * st, p->z + dd.z * st); tZ = 1; }
        else if (p->z >= zmax) { st = (zmax - p->z - 9e-7) / dd.z; *p = v3(p->x + dd.x * st, p->y + dd.y * st, p->z + dd.z * st); tZ = 1; }
        else inZ = 1;
        if ((tX && tY && tZ) || counter > cap) break;
        counter = counter + 1;
      }
      break;
    }
    case SMCRT_SRC_SLM: {                                            /* :159-212 */
      double x, y;
      spec_sample(P, rng, &x, &y);
      pk->pos = v3((x - 100.0) / ((double)S->grid.nx / (2.0 * S->grid.xmax)),
                   (y - 100.0) / ((double)S->grid.ny / (2.0 * S->grid.ymax)), s->pos[2]);
      pk->n = v3(s->dir[0], s->dir[1], s->dir[2]);
      pk->layer = 1;
      break;
    }
    default: {                                                       /* dslit :712-780, aperture :782-848 */
      spec_sample(P, rng, &wl, &tmp);
      double x1, y1, z1, x2, y2, z2;
      if (s->kind == SMCRT_SRC_DSLIT) {
        double a = 60.0 * wl, b = 20.0 * wl;
        if (ran2(rng) > 0.5) { x1 = ranu(rng, a / 2.0, a / 2.0 + b); y1 = ranu(rng, -b * 0.5, b * 0.5); }
        else { x1 = ranu(rng, -a / 2.0, -a / 2.0 - b); y1 = ranu(rng, -b * 0.5, b * 0.5); }
        z2 = 5.0 - (1.e-5 * (2.0 * (5.0 / 400.0)));
        x2 = ranu(rng, -5.0, 5.0);
        y2 = ranu(rng, -5.0, 5.0);
        z1 = (10000.0 * wl) - 5.0;
      } else {
        double apwid = 200e-6, b = apwid / 2.0, F = 4.95;
        x1 = ranu(rng, -b, b);
        y1 = ranu(rng, -b, b);
        double fa = F / apwid;
        z1 = (1.0 / (((fa * fa) / 2.0) * wl)) - 0.5;
        x2 = ranu(rng, -0.5, 0.5);
        y2 = ranu(rng, -0.5, 0.5);
        z2 = 0.5 - (1.e-5 * (2.0 * 0.5 / 400.0));
      }
      pk->pos = v3(x2, y2, z2);
      double dx = x2 - x1, dy = y2 - y1, dz = z2 - z1;
      double phase = sqrt(dx * dx + dy * dy + dz * dz);
      pk->n = v3(dx / phase, dy / phase, -fabs(dz) / phase);
      break;
    }
  }
}

/* ==================================================================== emit ===== */
static void emit(ctx_t* C, const smcrt_source* src, packet_t* pk, rng_t* rng) {
  const scene_t* S = C->S;
  const double xmax = S->grid.xmax, ymax = S->grid.ymax, zmax = S->grid.zmax;
  if (C->plan) {
    emit_ext(C, pk, rng);
  } else if (src->kind == SMCRT_SRC_POINT) {                         /* photon.f90:311-359 */
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
  S->nodes = nodes; S->n_nodes = n_nodes; S->top = top; S->n_top = n_top; S->grid = *grid;
  S->dets = dets; S->n_dets = n_dets;
  S->kappa = calloc(6 * (size_t)n_top, sizeof(double));
  S->albedo = S->kappa + n_top; S->mua = S->albedo + n_top; S->hgg = S->mua + n_top;
  S->g2 = S->hgg + n_top; S->nidx = S->g2 + n_top;
  for (int32_t i = 0; i < n_top; ++i) {                              /* init_mono :107-125 */
    const smcrt_sdf_node* nd = &nodes[top[i]];
    S->kappa[i] = nd->mus + nd->mua;
    if (nd->flags & SMCRT_NODE_ALBEDO_UNGUARDED) S->albedo[i] = nd->mus / S->kappa[i];  /* updateSpectral :198-199 */
    else S->albedo[i] = (nd->mua < 1e-9) ? 1.0 : nd->mus / S->kappa[i];
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
  if (!src || !cfg || !io || src->kind < SMCRT_SRC_POINT || src->kind > SMCRT_SRC_APERTURE) {
    free_scene(&S);
    return SMCRT_ERR_INVALID_ARG;
  }
  src_plan_t plan;
  const int use_plan = src->kind > SMCRT_SRC_PENCIL || (src->spectrum && src->spectrum->kind != SMCRT_SPEC_CONSTANT);
  if (use_plan && (st = build_plan(&plan, src)) != SMCRT_OK) {
    free_scene(&S);
    return st;
  }
  int64_t nv = (int64_t)grid->nx * grid->ny * grid->nz;
  ctx_t C;
  memset(&C, 0, sizeof C);
  C.S = &S;
  C.flags = cfg->flags;
  /* A grid asked for in fp64 only is accumulated in place: no per-call scratch grid, so a
   * caller that runs a job in many small calls (bench.py's CPU legs) pays nothing per call.
   * fp32 grids get a scratch fp64 sum that is added once at the end, as smcrt_run does. */
  float* gf[3] = {io->jmean, io->absorb, io->emission};
  double* gd[3] = {io->jmean_f64, io->absorb_f64, io->emission_f64};
  double* g[3] = {NULL, NULL, NULL};
  int own[3] = {0, 0, 0};
  for (int t = 0; t < 3; ++t) {
    if (gf[t]) { g[t] = calloc((size_t)nv, sizeof(double)); own[t] = 1; }
    else g[t] = gd[t];
  }
  C.jmean = g[0];
  C.absorb = g[1];
  C.emission = g[2];
  C.det = io->det_bins;
  C.moments = io->moments;
  C.plan = use_plan ? &plan : NULL;
  double* ds = calloc(2 * (size_t)n_top, sizeof(double));
  for (uint64_t j = 0; j < cfg->n_photons; ++j) {
    smcrt_photon_record* rec = (io->records && (cfg->flags & SMCRT_FLAG_RECORD_PHOTONS)) ? &io->records[j] : NULL;
    run_photon(&C, src, cfg->first_photon + j, cfg->seed, ds, ds + n_top, rec);
  }
  for (int t = 0; t < 3; ++t) {
    if (!own[t]) continue;
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
  if (use_plan) free_plan(&plan);
  free_scene(&S);
  return SMCRT_OK;
}

/* One emission (no re-emission loop) of photons [first, first+n): pos/dir (3 each),
 * cells (3) and RNG draws per photon, for the source unit checks of test/photon. */
ORACLE_API int oracle_emit(const smcrt_grid* grid, const smcrt_source* src, uint64_t seed, uint64_t first,
                           int64_t n, double* pos, double* dir, int32_t* cells, uint32_t* draws) {
  static const int32_t top0 = 0;
  smcrt_sdf_node nd;
  memset(&nd, 0, sizeof nd);
  nd.kind = SMCRT_SDF_SPHERE; nd.param[0] = 1.0; nd.n = 1.0;
  for (int i = 0; i < 4; ++i) nd.transform[i * 5] = 1.0;
  scene_t S;
  int st = build_scene(&S, &nd, 1, &top0, 1, grid, NULL, 0);
  if (st) return st;
  src_plan_t plan;
  if ((st = build_plan(&plan, src)) != SMCRT_OK) { free_scene(&S); return st; }
  ctx_t C;
  memset(&C, 0, sizeof C);
  C.S = &S;
  C.plan = &plan;
  for (int64_t j = 0; j < n; ++j) {
    rng_t rng = {first + (uint64_t)j, seed, 0};
    packet_t pk;
    memset(&pk, 0, sizeof pk);
    emit(&C, src, &pk, &rng);
    pos[3 * j] = pk.pos.x; pos[3 * j + 1] = pk.pos.y; pos[3 * j + 2] = pk.pos.z;
    dir[3 * j] = pk.n.x; dir[3 * j + 1] = pk.n.y; dir[3 * j + 2] = pk.n.z;
    cells[3 * j] = pk.xcell; cells[3 * j + 1] = pk.ycell; cells[3 * j + 2] = pk.zcell;
    draws[j] = rng.draws;
  }
  free_plan(&plan);
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

/* n samples of a source spectrum (sample of piecewise.f90; unit checks of test/optical_props) */
ORACLE_API int oracle_spectrum_sample(const smcrt_source* src, uint64_t seed, uint64_t first, int64_t n,
                                      double* x, double* y, uint32_t* draws) {
  src_plan_t plan;
  int st = build_plan(&plan, src);
  if (st) return st;
  for (int64_t j = 0; j < n; ++j) {
    rng_t rng = {first + (uint64_t)j, seed, 0};
    spec_sample(&plan, &rng, &x[j], &y[j]);
    if (draws) draws[j] = rng.draws;
  }
  free_plan(&plan);
  return SMCRT_OK;
}

/* ===================================================== spectral optical properties ===== */
/* The `spectral` type (opticalProperties.f90:127-201) over five piecewise1D tables.
 * Its ran2 draws come from the host stream family 2: draw d is the (d & 1) half of Philox block
 * (d >> 1, 2, 0, 0xFFFFFFFF) under (seed_lo, seed_hi) (the library's smcrt_spectral_sample
 * documents the same stream). mode 0: init_spectral as documented (properties at the sampled
 * wavelength, albedo guarded); 1: updateSpectral (albedo unguarded); 2: init_spectral as
 * compiled (sample(x, y) without a value: each property is an x-axis draw of its own table).
 * out[8] = mus, mua, hgg, g2, n, kappa, albedo, wavelength. */
static double spectral_ran2(uint64_t seed, uint64_t* d) {
  uint32_t ctr[4] = {(uint32_t)(*d >> 1), 2u, 0u, 0xFFFFFFFFu};
  uint32_t key[2] = {(uint32_t)seed, (uint32_t)(seed >> 32)};
  uint32_t o[4];
  oracle_philox4x32_10(ctr, key, o);
  uint64_t u = (*d & 1u) ? (((uint64_t)o[3] << 32) | o[2]) : (((uint64_t)o[1] << 32) | o[0]);
  *d += 1;
  return (double)(u >> 11) * 0x1.0p-53;
}

/* init_piecewise1D (piecewise.f90:142-168): cdf(1) = 0, cdf(i) = sum_{k=2..i} w(k) y(k) with
 * stdlib's trapz_weights, then res%cdf = res%cdf / res%cdf(length) */
static double* pw1d_cdf(const double* a, int64_t n) {
  const double* x = a;
  const double* y = a + n;
  double* cdf = calloc((size_t)n, sizeof(double));
  double sumer = 0.0;
  for (int64_t i = 1; i < n; ++i) {
    double w = (n == 2 || i == n - 1) ? 0.5 * (x[n - 1] - x[n - 2]) : 0.5 * (x[i + 1] - x[i - 1]);
    sumer = sumer + w * y[i];
    cdf[i] = sumer;
  }
  double last = cdf[n - 1];
  for (int64_t i = 0; i < n; ++i) cdf[i] = cdf[i] / last;
  return cdf;
}

/* sample1D without value (:124-131) */
static double pw1d_draw(const double* a, int64_t n, uint64_t seed, uint64_t* d) {
  double* cdf = pw1d_cdf(a, n);
  double val = spectral_ran2(seed, d);
  int64_t idx = search_1d(cdf, n, val);
  double x = a[idx - 1] + ((val - cdf[idx - 1]) * (a[idx] - a[idx - 1])) / (cdf[idx] - cdf[idx - 1]);
  free(cdf);
  return x;
}

/* sample1D with value (:132-137); search_2D (:288-312) bisects the first column */
static double pw1d_at(const double* a, int64_t n, double value) {
  int64_t idx = search_1d(a, n, value);
  const double* y = a + n;
  return y[idx - 1] + (y[idx] - y[idx - 1]) * ((value - a[idx - 1]) / (a[idx] - a[idx - 1]));
}

ORACLE_API int oracle_spectral_sample(const smcrt_spectral* sp, int32_t mode, uint64_t seed, uint64_t* draw,
                                      double out[8]) {
  if (!sp || !draw || !out || mode < 0 || mode > 2) return SMCRT_ERR_INVALID_ARG;
  if (!sp->mus || !sp->mua || !sp->hgg || !sp->n || !sp->flux) return SMCRT_ERR_INVALID_ARG;
  if (sp->n_mus < 2 || sp->n_mua < 2 || sp->n_hgg < 2 || sp->n_n < 2 || sp->n_flux < 2) return SMCRT_ERR_INVALID_ARG;
  uint64_t d = *draw;
  double wave = pw1d_draw(sp->flux, sp->n_flux, seed, &d);          /* flux%sample(wave, tmp) */
  double mus, mua, hgg, n;
  if (mode == 2) {                                                   /* :144-148 as compiled */
    mus = pw1d_draw(sp->mus, sp->n_mus, seed, &d);
    mua = pw1d_draw(sp->mua, sp->n_mua, seed, &d);
    hgg = pw1d_draw(sp->hgg, sp->n_hgg, seed, &d);
    n = pw1d_draw(sp->n, sp->n_n, seed, &d);
  } else {                                                           /* :184-195 */
    mus = pw1d_at(sp->mus, sp->n_mus, wave);
    mua = pw1d_at(sp->mua, sp->n_mua, wave);
    hgg = pw1d_at(sp->hgg, sp->n_hgg, wave);
    n = pw1d_at(sp->n, sp->n_n, wave);
  }
  double kappa = mus + mua, albedo;
  if (mode == 1) albedo = mus / kappa;                               /* :198-199 */
  else albedo = (mua < 1e-9) ? 1.0 : mus / kappa;                    /* :150-155 */
  out[0] = mus; out[1] = mua; out[2] = hgg; out[3] = hgg * hgg; out[4] = n;
  out[5] = kappa; out[6] = albedo; out[7] = wave;
  *draw = d;
  return SMCRT_OK;
}
