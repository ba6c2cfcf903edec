// detmath.h — device-side RNG and elementary functions with fixed, portable arithmetic.
//
// The reference draws from the compiler intrinsic random_number (src/random_mod.f90:83-90)
// and calls the compiler's log/sin/cos. Here every draw is Philox4x32-10 keyed by
// (seed, photon index) and log/sin/cos are fixed fdlibm-style polynomials evaluated with
// plain IEEE operations (compiled with -ffp-contract=off), so a photon's trajectory does
// not depend on the GPU, the launch geometry, or the number of GPUs.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace smcrt {

// ------------------------------------------------------------------ Philox4x32-10 --
struct Philox4 {
  uint32_t v[4];
};

__device__ __forceinline__ Philox4 philox4x32_10(uint32_t c0, uint32_t c1, uint32_t c2, uint32_t c3,
                                                 uint32_t k0, uint32_t k1) {
  // The key is wave-uniform. Make it opaque here so the ten round keys are derived at each
  // call (two scalar adds per round) instead of being hoisted into twenty long-lived scalar
  // registers, which the kernel cannot afford and would spill.
  asm volatile("" : "+s"(k0), "+s"(k1));
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    if (r > 0) { k0 += 0x9E3779B9u; k1 += 0xBB67AE85u; }
    // one 32x32->64 multiply (v_mad_u64_u32) per product instead of separate lo/hi multiplies
    const uint64_t p0 = (uint64_t)0xD2511F53u * c0, p1 = (uint64_t)0xCD9E8D57u * c2;
    const uint32_t lo0 = (uint32_t)p0, hi0 = (uint32_t)(p0 >> 32);
    const uint32_t lo1 = (uint32_t)p1, hi1 = (uint32_t)(p1 >> 32);
    const uint32_t n0 = hi1 ^ c1 ^ k0, n2 = hi0 ^ c3 ^ k1;
    c0 = n0; c1 = lo1; c2 = n2; c3 = lo0;
  }
  Philox4 o;
  o.v[0] = c0; o.v[1] = c1; o.v[2] = c2; o.v[3] = c3;
  return o;
}

// Per-photon stream: draw d is the (d&1) half of Philox block d>>1, counter
// (d>>1, 0, pid_lo, pid_hi), key (seed_lo, seed_hi); 53-bit double in [0,1).
// The key is launch-uniform and passed in, so it stays in scalar registers.
struct Rng {
  uint32_t pid_lo, pid_hi;
  uint32_t draws;
  double cached;

  __device__ __forceinline__ void init(uint64_t pid) {
    pid_lo = (uint32_t)pid; pid_hi = (uint32_t)(pid >> 32);
    draws = 0; cached = 0.0;
  }
  __device__ __forceinline__ double next(uint32_t key0, uint32_t key1) {
    const uint32_t d = draws++;
    if (d & 1u) return cached;
    const Philox4 o = philox4x32_10(d >> 1, 0u, pid_lo, pid_hi, key0, key1);
    const uint64_t u0 = ((uint64_t)o.v[1] << 32) | o.v[0];
    const uint64_t u1 = ((uint64_t)o.v[3] << 32) | o.v[2];
    cached = (double)(u1 >> 11) * 0x1.0p-53;
    return (double)(u0 >> 11) * 0x1.0p-53;
  }
};

// --------------------------------------------------------------- elementary math --
__host__ __device__ __forceinline__ uint64_t d2u(double x) { return __builtin_bit_cast(uint64_t, x); }
__host__ __device__ __forceinline__ double u2d(uint64_t u) { return __builtin_bit_cast(double, u); }

// IEEE fp64 division split in two. For `n / d` the compiler emits (gfx950):
//   D = v_div_scale(d); r = v_rcp(D); twice { e = fma(-D, r, 1); r = fma(r, e, r) };
//   q = N*r; res = fma(-D, q, N); v_div_fmas(res, r, q); v_div_fixup(.., d, n)
// with N = v_div_scale(n). While 2^-500 <= |n|, |d| <= 4 neither operand is scaled, vcc
// stays 0 (v_div_fmas is a plain fma) and v_div_fixup passes the quotient through, so the
// two halves below give the correctly rounded n / d bit for bit. The first half depends
// on d only and can be shared by every division by the same d.
__device__ __forceinline__ double ieee_rcp_f64(double d) {
  double r = __builtin_amdgcn_rcp(d);
  double e = __builtin_fma(-d, r, 1.0);
  r = __builtin_fma(r, e, r);
  e = __builtin_fma(-d, r, 1.0);
  return __builtin_fma(r, e, r);
}
__device__ __forceinline__ double ieee_div_tail_f64(double n, double d, double r) {
  const double q = n * r;
  const double res = __builtin_fma(-d, q, n);
  return __builtin_fma(res, r, q);
}

// natural log: fdlibm e_log.c algorithm (identical operation sequence to the oracle)
__device__ inline double det_log(double x) {
  const double ln2_hi = 6.93147180369123816490e-01, ln2_lo = 1.90821492927058770002e-10,
               two54 = 1.80143985094819840000e+16, Lg1 = 6.666666666666735130e-01,
               Lg2 = 3.999999999940941908e-01, Lg3 = 2.857142874366239149e-01,
               Lg4 = 2.222219843214978396e-01, Lg5 = 1.818357216161805012e-01,
               Lg6 = 1.531383769920937332e-01, Lg7 = 1.479819860511658591e-01;
  uint64_t ux = d2u(x);
  int32_t hx = (int32_t)(ux >> 32);
  const uint32_t lx = (uint32_t)ux;
  int32_t k = 0;
  if (hx < 0x00100000) {
    if (((hx & 0x7fffffff) | lx) == 0) return -__builtin_inf();
    if (hx < 0) return __builtin_nan("");
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
  x = u2d(((uint64_t)(uint32_t)(hx | (i ^ 0x3ff00000)) << 32) | (ux & 0xffffffffull));
  k += (i >> 20);
  const double f = x - 1.0;
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
  const double s = f / (2.0 + f);
  dk = (double)k;
  const double z = s * s;
  i = hx - 0x6147a;
  const double w = z * z;
  const int32_t j = 0x6b851 - hx;
  const double t1 = w * (Lg2 + w * (Lg4 + w * Lg6));
  const double t2 = z * (Lg1 + w * (Lg3 + w * (Lg5 + w * Lg7)));
  i |= j;
  R = t2 + t1;
  if (i > 0) {
    const double hfsq = 0.5 * f * f;
    if (k == 0) return f - (hfsq - s * (hfsq + R));
    return dk * ln2_hi - ((hfsq - (s * (hfsq + R) + dk * ln2_lo)) - f);
  }
  if (k == 0) return f - s * (f - R);
  return dk * ln2_hi - ((s * (f - R) - dk * ln2_lo) - f);
}

__host__ __device__ __forceinline__ double ksin(double x) {
  const double S1 = -1.66666666666666324348e-01, S2 = 8.33333333332248946124e-03,
               S3 = -1.98412698298579493134e-04, S4 = 2.75573137070700676789e-06,
               S5 = -2.50507602534068634195e-08, S6 = 1.58969099521155010221e-10;
  const double z = x * x;
  const double v = z * x;
  const double r = S2 + z * (S3 + z * (S4 + z * (S5 + z * S6)));
  return x + v * (S1 + z * r);
}

__host__ __device__ __forceinline__ double kcos(double x) {
  const double C1 = 4.16666666666666019037e-02, C2 = -1.38888888888741095749e-03,
               C3 = 2.48015872894767294178e-05, C4 = -2.75573143513906633035e-07,
               C5 = 2.08757232129817482790e-09, C6 = -1.13596475577881948265e-11;
  const uint32_t ix = (uint32_t)(d2u(x) >> 32) & 0x7fffffffu;
  if (ix < 0x3e400000u) return 1.0;
  const double z = x * x;
  const double r = z * (C1 + z * (C2 + z * (C3 + z * (C4 + z * (C5 + z * C6)))));
  if (ix < 0x3FD33333u) return 1.0 - (0.5 * z - z * r);
  const double qx = (ix > 0x3fe90000u) ? 0.28125 : u2d((uint64_t)(ix - 0x00200000u) << 32);
  const double hz = 0.5 * z - qx;
  const double a = 1.0 - qx;
  return a - (hz - z * r);
}

// sin and cos of x in [0, 4pi] (fdlibm medium Cody-Waite reduction)
__host__ __device__ __forceinline__ void det_sincos(double x, double* s, double* c) {
  const double invpio2 = 6.36619772367581382433e-01, pio2_1 = 1.57079632673412561417e+00,
               pio2_1t = 6.07710050650619224932e-11;
  const int32_t n = (int32_t)(x * invpio2 + 0.5);
  const double fn = (double)n;
  const double r = x - fn * pio2_1;
  const double w = fn * pio2_1t;
  const double y = r - w;
  const double sy = ksin(y), cy = kcos(y);
  switch (n & 3) {
    case 0: *s = sy; *c = cy; break;
    case 1: *s = cy; *c = -sy; break;
    case 2: *s = -sy; *c = -cy; break;
    default: *s = -cy; *c = sy; break;
  }
}

// sin and cos of any angle of the twist and bend modifiers (k * p, sdfModifiers.f90:363-364,
// :383-384): sin(-x) = -sin(x), cos(-x) = cos(x), then det_sincos's reduction, whose
// fn * pio2_1 stays exact while |x| < 2^19 pi/2 (larger angles stay deterministic, with less
// accuracy). The oracle restates it (oracle_sincos_any).
__host__ __device__ __forceinline__ void det_sincos_any(double x, double* s, double* c) {
  det_sincos(fabs(x), s, c);
  if (x < 0.0) *s = -*s;
}

// atan (fdlibm s_atan.c), for the fibre detector's acceptance angle (detectors.f90:386).

__device__ inline double det_atan(double x) {
  const double atanhi[4] = {4.63647609000806093515e-01, 7.85398163397448278999e-01, 9.82793723247329054082e-01,
                            1.57079632679489655800e+00};
  const double atanlo[4] = {2.26987774529616870924e-17, 3.06161699786838301793e-17, 1.39033110312309984516e-17,
                            6.12323399573676603587e-17};
  const double aT0 = 3.33333333333329318027e-01, aT1 = -1.99999999998764832476e-01,
               aT2 = 1.42857142725034663711e-01, aT3 = -1.11111104054623557880e-01,
               aT4 = 9.09088713343650656196e-02, aT5 = -7.69187620504482999495e-02,
               aT6 = 6.66107313738753120669e-02, aT7 = -5.83357013379057348645e-02,
               aT8 = 4.97687799461593236017e-02, aT9 = -3.65315727442169155270e-02,
               aT10 = 1.62858201153657823623e-02;
  const uint64_t u = d2u(x);
  const int32_t hx = (int32_t)(u >> 32);
  const uint32_t ix = (uint32_t)hx & 0x7fffffffu;
  int id;
  if (ix >= 0x44100000u) {  // |x| >= 2^66 (or NaN)
    if (ix > 0x7ff00000u || (ix == 0x7ff00000u && (uint32_t)u != 0u)) return x + x;
    return hx > 0 ? atanhi[3] + atanlo[3] : -atanhi[3] - atanlo[3];
  }
  if (ix < 0x3fdc0000u) {  // |x| < 0.4375
    if (ix < 0x3e200000u) return x;  // |x| < 2^-29
    id = -1;
  } else {
    x = fabs(x);
    if (ix < 0x3ff30000u) {    // |x| < 1.1875
      if (ix < 0x3fe60000u) {  // 7/16 <= |x| < 11/16
        id = 0; x = (2.0 * x - 1.0) / (2.0 + x);
      } else {
        id = 1; x = (x - 1.0) / (x + 1.0);
      }
    } else if (ix < 0x40038000u) {  // |x| < 2.4375
      id = 2; x = (x - 1.5) / (1.0 + 1.5 * x);
    } else {
      id = 3; x = -1.0 / x;
    }
  }
  const double z = x * x, w = z * z;
  const double s1 = z * (aT0 + w * (aT2 + w * (aT4 + w * (aT6 + w * (aT8 + w * aT10)))));
  const double s2 = w * (aT1 + w * (aT3 + w * (aT5 + w * (aT7 + w * aT9))));
  if (id < 0) return x - x * (s1 + s2);
  const double r = atanhi[id] - ((x * (s1 + s2) - atanlo[id]) - x);
  return hx < 0 ? -r : r;
}

}  // namespace smcrt
