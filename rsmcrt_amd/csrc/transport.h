// transport.h — the per-photon hot path as CDNA4 device code.
//
// One wavefront lane carries one photon packet (fp64 state in VGPRs). The SDF table is
// wave-uniform (every lane evaluates SDF i at the same time), so node parameters come in
// through scalar loads and the per-SDF `switch` never diverges. The functions below follow
// the reference line by line (file:line cited at each) so that, with -ffp-contract=off,
// a photon's trajectory is bit-identical to the CPU restatement in oracle/.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/smcrt.h"
#include "detmath.h"

namespace smcrt {

// Unbounded loops of the reference are capped; the CPU restatement uses the same caps.
constexpr int64_t MAX_EMIT_TRIES = 100000;
constexpr int64_t MAX_HOP_ITERS = 1000000;
constexpr int64_t MAX_MARCH_ITERS = 10000000;
constexpr int64_t MAX_GLANCE_ITERS = 100000;
constexpr int64_t MAX_DDA_ITERS = 10000000;
constexpr int MAX_RENORM_ITERS = 64;
constexpr int64_t MAX_INTERACTIONS = 100000000;

// Optical properties of a top-level SDF, derived as init_mono does
// (opticalProperties.f90:107-125).
struct TopProps {
  double kappa, albedo, hgg, n;
};

// Everything a launch needs; passed by value (kernel arguments live in SGPRs).
struct KParams {
  const smcrt_sdf_node* __restrict__ nodes;
  const int32_t* __restrict__ top;
  const TopProps* __restrict__ props;
  const double* __restrict__ xface;  // nx+1
  const double* __restrict__ yface;  // ny+1
  const double* __restrict__ zface;  // nz+2
  const smcrt_detector* __restrict__ dets;
  const int64_t* __restrict__ det_off;
  int32_t n_top, n_dets;
  int32_t nx, ny, nz;
  uint32_t flags;
  double xmax, ymax, zmax;
  smcrt_source src;
  uint64_t n_photons, first_photon, seed;
  double* jmean;
  double* absorb;
  double* emission;
  double* det_bins;
  double* nscatt;
  double* moments;
  unsigned long long* counters;
  smcrt_photon_record* records;
  unsigned long long* queue;  // photon work-queue head (zeroed before launch)
};

// ------------------------------------------------------------------ vec3 ---------
struct V3 {
  double x, y, z;
};
__device__ __forceinline__ V3 v3(double x, double y, double z) { return V3{x, y, z}; }
__device__ __forceinline__ V3 operator+(V3 a, V3 b) { return v3(a.x + b.x, a.y + b.y, a.z + b.z); }
__device__ __forceinline__ V3 operator-(V3 a, V3 b) { return v3(a.x - b.x, a.y - b.y, a.z - b.z); }
__device__ __forceinline__ V3 mul(V3 a, double s) { return v3(a.x * s, a.y * s, a.z * s); }   // vec*scal
__device__ __forceinline__ V3 smul(double s, V3 a) { return v3(s * a.x, s * a.y, s * a.z); }  // scal*vec
__device__ __forceinline__ double dot(V3 a, V3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
__device__ __forceinline__ double len(V3 a) { return sqrt(a.x * a.x + a.y * a.y + a.z * a.z); }
__device__ __forceinline__ V3 vabs(V3 a) { return v3(fabs(a.x), fabs(a.y), fabs(a.z)); }
__device__ __forceinline__ double dmax(double a, double b) { return a > b ? a : b; }
__device__ __forceinline__ double dmin(double a, double b) { return a < b ? a : b; }
__device__ __forceinline__ double clampd(double v, double lo, double hi) { return dmin(dmax(v, lo), hi); }

// vec_dot_mat, vector_class.f90:292-304 (transform column-major)
__device__ __forceinline__ V3 dotmat(V3 a, const double* t) {
  return v3(t[0] * a.x + t[1] * a.y + t[2] * a.z + t[3], t[4] * a.x + t[5] * a.y + t[6] * a.z + t[7],
            t[8] * a.x + t[9] * a.y + t[10] * a.z + t[11]);
}

// ------------------------------------------------------------------ SDFs ---------
__device__ __forceinline__ double csg(int32_t op, double d1, double d2, double k) {
  switch (op) {
    case SMCRT_OP_UNION: return dmin(d1, d2);  // sdfModifiers.f90:428-440
    case SMCRT_OP_SMOOTH_UNION: {              // :442-456
      const double h = dmax(k - fabs(d1 - d2), 0.0) / k;
      return dmin(d1, d2) - h * h * h * k * (1.0 / 6.0);
    }
    case SMCRT_OP_SUBTRACTION: return dmax(-d1, d2);  // :458-473
    default: return dmax(d1, d2);                     // :475-491
  }
}

// One primitive (sdfs.f90:494-735). `nd` is wave-uniform.
__device__ __forceinline__ double sdf_prim(const smcrt_sdf_node* __restrict__ nd, V3 pos) {
  const double* P = nd->param;
  const V3 p = dotmat(pos, nd->transform);
  switch (nd->kind) {
    case SMCRT_SDF_SPHERE:  // :494-508
      return sqrt(p.x * p.x + p.y * p.y + p.z * p.z) - P[0];
    case SMCRT_SDF_BOX: {  // :510-525
      const V3 q = vabs(p) - v3(P[0], P[1], P[2]);
      return len(v3(dmax(q.x, 0.0), dmax(q.y, 0.0), dmax(q.z, 0.0))) + dmin(dmax(q.x, dmax(q.y, q.z)), 0.0);
    }
    case SMCRT_SDF_TORUS: {  // :527-542
      const V3 q = v3(len(v3(p.x, 0.0, p.z)) - P[0], p.y, 0.0);
      return len(q) - P[1];
    }
    case SMCRT_SDF_CYLINDER: {  // :544-581
      const V3 a = v3(P[0], P[1], P[2]), b = v3(P[3], P[4], P[5]);
      const V3 ba = b - a, pa = p - a;
      const double baba = dot(ba, ba), paba = dot(pa, ba);
      const double x = len(mul(pa, baba) - mul(ba, paba)) - P[6] * baba;
      const double y = fabs(paba - baba * 0.5) - baba * 0.5;
      const double x2 = x * x, y2 = (y * y) * baba;
      double d;
      if (dmax(x, y) < 0.0) d = -dmin(x2, y2);
      else if (x > 0.0 && y > 0.0) d = x2 + y2;
      else if (x > 0.0) d = x2;
      else if (y > 0.0) d = y2;
      else d = 0.0;
      return copysign(sqrt(fabs(d)) / baba, d);
    }
    case SMCRT_SDF_TRIPRISM: {  // :583-597
      const V3 q = vabs(p);
      return dmax(q.z - P[1], dmax(q.x * 0.866025 + p.y * 0.5, -p.y) - P[0] * 0.5);
    }
    case SMCRT_SDF_SEGMENT: {  // :599-626
      const V3 a = v3(P[0], P[1], P[2]), b = v3(P[3], P[4], P[5]);
      const V3 pa = p - a, ba = b - a;
      const double h = clampd(dot(pa, ba) / dot(ba, ba), 0.0, 1.0);
      return len(pa - mul(ba, h)) - 0.1;
    }
    case SMCRT_SDF_CAPSULE: {  // :628-648
      const V3 a = v3(P[0], P[1], P[2]), b = v3(P[3], P[4], P[5]);
      const V3 pa = p - a, ba = b - a;
      const double h = clampd(dot(pa, ba) / dot(ba, ba), 0.0, 1.0);
      return len(pa - mul(ba, h)) - P[6];
    }
    case SMCRT_SDF_CONE: {  // :650-686
      const V3 a = v3(P[0], P[1], P[2]), b = v3(P[3], P[4], P[5]);
      const double ra = P[6], rb = P[7];
      const double rba = rb - ra;
      const double baba = dot(b - a, b - a);
      const double papa = dot(p - a, p - a);
      const double paba = dot(p - a, b - a) / baba;
      const double x = sqrt(papa - baba * (paba * paba));
      const double cax = (paba < 0.5) ? dmax(0.0, x - ra) : dmax(0.0, x - rb);
      const double cay = fabs(paba - 0.5) - 0.5;
      const double k = rba * rba + baba;
      const double f = clampd((rba * (x - ra) + paba * baba) / k, 0.0, 1.0);
      const double cbx = x - ra - f * rba;
      const double cby = paba - f;
      const double s = (cbx < 0.0 && cay < 0.0) ? -1.0 : 1.0;
      return s * sqrt(dmin(cax * cax + baba * (cay * cay), cbx * cbx + baba * (cby * cby)));
    }
    case SMCRT_SDF_EGG: {  // :688-718
      const double r1 = P[0], r2 = P[1], hh = P[2];
      const V3 pin = v3(fabs(p.x), p.y, p.z);
      const double r = r1 - r2;
      const double h_in = hh + r;
      const double l = (h_in * h_in - r * r) / (2.0 * r);
      if (pin.y <= 0.0) return len(pin) - r1;
      if ((pin.y - h_in) * l > pin.x * h_in) return len(pin - v3(0.0, h_in, 0.0)) - ((r1 + l) - len(v3(h_in, l, 0.0)));
      return len(pin + v3(l, 0.0, 0.0)) - (r1 + l);
    }
    case SMCRT_SDF_PLANE:  // :720-735
      return dot(p, v3(P[0], P[1], P[2]));
    default:
      return __builtin_nan("");
  }
}

// sdf_evaluate / eval_model (sdf_base.f90:146-161, 273-281). Models hold primitives
// (one level; checked at scene creation).
__device__ __forceinline__ double sdf_node(const smcrt_sdf_node* __restrict__ nodes, int32_t idx, V3 pos) {
  const smcrt_sdf_node* nd = nodes + idx;
  if (nd->kind != SMCRT_SDF_MODEL) return sdf_prim(nd, pos);
  const int32_t c0 = nd->first_child, nc = nd->n_children, op = nd->op;
  const double k = nd->k;
  double res = sdf_prim(nodes + c0, pos);
  for (int32_t i = 1; i < nc; ++i) res = csg(op, res, sdf_prim(nodes + c0 + i, pos), k);
  return res;
}

__device__ __forceinline__ double sdf_top(const KParams& K, int32_t i, V3 pos) {
  return sdf_node(K.nodes, K.top[i], pos);
}

// The reductions tauint2 takes over ds(:): minval(abs(ds)), minval(ds),
// maxloc(ds, mask=ds<0) (first maximum; 0 when no SDF contains the point).
struct DsInfo {
  double minabs, minv;
  int32_t maxloc;
};

__device__ __forceinline__ DsInfo eval_all(const KParams& K, V3 pos, uint32_t& cnt, bool mask_le = false) {
  DsInfo r;
  r.minabs = __builtin_inf();
  r.minv = __builtin_inf();
  r.maxloc = 0;
  double best = -__builtin_inf();
  for (int32_t i = 0; i < K.n_top; ++i) {
    const double d = sdf_top(K, i, pos);
    const double a = fabs(d);
    if (a < r.minabs) r.minabs = a;
    if (d < r.minv) r.minv = d;
    const bool neg = mask_le ? (d <= 0.0) : (d < 0.0);
    if (neg && (r.maxloc == 0 || d > best)) { best = d; r.maxloc = i + 1; }
  }
  cnt += (uint32_t)K.n_top;
  return r;
}

// ------------------------------------------------------------------ packet -------
struct Packet {
  V3 pos, n;
  int32_t xcell, ycell, zcell;
  int32_t layer;
  double weight;
  uint32_t bounces, nscatt;
  bool tflag;
};

// Per-lane counters, reduced across the wave once at the end of the launch.
struct LaneCounters {
  uint32_t v[SMCRT_NCOUNTERS];
};

struct Lane {
  LaneCounters c;
  double nscatt;
  bool fault;
};

// update_voxels, inttau2.f90:587-614 (corner coordinates)
__device__ __forceinline__ int32_t cell_of(double p, int32_t n, double max) {
  const double f = floor(((double)n * p) / (2.0 * max));
  if (!(f >= 0.0 && f < (double)n)) return -1;
  return (int32_t)f + 1;
}
// get_voxel_cart, grid.f90:51-78 (centred coordinates)
__device__ __forceinline__ int32_t vox_of(double p, int32_t n, double max) {
  const double f = floor(((double)n * (p + max)) / (2.0 * max));
  if (!(f >= 0.0 && f < (double)n)) return -1;
  return (int32_t)f + 1;
}

__device__ __forceinline__ int64_t lin(const KParams& K, int32_t i, int32_t j, int32_t k) {
  return (int64_t)(i - 1) + (int64_t)K.nx * ((int64_t)(j - 1) + (int64_t)K.ny * (int64_t)(k - 1));
}

__device__ __forceinline__ void atomic_add_nr(double* p, double v) {
  __hip_atomic_fetch_add(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// jmean(cell) += real(dcell,sp)*weight (inttau2.f90:427,434)
__device__ __forceinline__ void deposit(const KParams& K, Lane& L, int32_t i, int32_t j, int32_t k, double dcell,
                                        double weight) {
  L.c.v[SMCRT_CTR_DEPOSITS]++;
  if (K.jmean) atomic_add_nr(K.jmean + lin(K, i, j, k), (double)(float)dcell * weight);
}

// update_grids + wall_dist + update_pos (inttau2.f90:367-584)
__device__ void update_grids(const KParams& K, Lane& L, V3 pos, V3 dir, double d_sdf, Packet& pk) {
  L.c.v[SMCRT_CTR_GRID_UPDATES]++;
  V3 old = v3(pos.x + K.xmax, pos.y + K.ymax, pos.z + K.zmax);
  int32_t ci = cell_of(old.x, K.nx, K.xmax), cj = cell_of(old.y, K.ny, K.ymax), ck = cell_of(old.z, K.nz, K.zmax);
  pk.xcell = ci; pk.ycell = cj; pk.zcell = ck;
  if (!(K.flags & SMCRT_FLAG_PATHLENGTH)) {  // :446-463
    old.x = old.x + dir.x * d_sdf;
    old.y = old.y + dir.y * d_sdf;
    old.z = old.z + dir.z * d_sdf;
    ci = cell_of(old.x, K.nx, K.xmax); cj = cell_of(old.y, K.ny, K.ymax); ck = cell_of(old.z, K.nz, K.zmax);
    if (ci == -1 || cj == -1 || ck == -1) pk.tflag = true;
    pk.xcell = ci; pk.ycell = cj; pk.zcell = ck;
    return;
  }
  const double delta = 1e-8;  // :393
  double d = 0.0;
  if (ci == -1 || cj == -1 || ck == -1) { pk.tflag = true; return; }
  for (int64_t it = 0;; ++it) {
    if (it >= MAX_DDA_ITERS) { L.fault = true; pk.tflag = true; break; }
    // wall_dist :467-521
    double dx = -999.0, dy = -999.0, dz = -999.0;
    if (dir.x > 0.0) dx = (K.xface[ci] - old.x) / dir.x;
    else if (dir.x < 0.0) dx = (K.xface[ci - 1] - old.x) / dir.x;
    else if (dir.x == 0.0) dx = 100000.0;
    if (dir.y > 0.0) dy = (K.yface[cj] - old.y) / dir.y;
    else if (dir.y < 0.0) dy = (K.yface[cj - 1] - old.y) / dir.y;
    else if (dir.y == 0.0) dy = 100000.0;
    if (dir.z > 0.0) dz = (K.zface[ck] - old.z) / dir.z;
    else if (dir.z < 0.0) dz = (K.zface[ck - 1] - old.z) / dir.z;
    else if (dir.z == 0.0) dz = 100000.0;
    double dcell = dmin(dmin(dx, dy), dz);
    if (dcell < 0.0) { L.fault = true; pk.tflag = true; break; }  // error stop :510-516
    const bool lx = (dcell == dx), ly = (dcell == dy), lz = (dcell == dz);
    if (d + dcell > d_sdf) {  // :421-429
      dcell = d_sdf - d;
      d = d_sdf;
      deposit(K, L, ci, cj, ck, dcell, pk.weight);
      old.x = old.x + dir.x * dcell;
      old.y = old.y + dir.y * dcell;
      old.z = old.z + dir.z * dcell;
      break;
    }
    d = d + dcell;
    deposit(K, L, ci, cj, ck, dcell, pk.weight);
    if (lx) {  // update_pos :538-582
      if (dir.x > 0.0) old.x = K.xface[ci] + delta;
      else if (dir.x < 0.0) old.x = K.xface[ci - 1] - delta;
      old.y = old.y + dir.y * dcell;
      old.z = old.z + dir.z * dcell;
    } else if (ly) {
      if (dir.y > 0.0) old.y = K.yface[cj] + delta;
      else if (dir.y < 0.0) old.y = K.yface[cj - 1] - delta;
      old.x = old.x + dir.x * dcell;
      old.z = old.z + dir.z * dcell;
    } else if (lz) {
      if (dir.z > 0.0) old.z = K.zface[ck] + delta;
      else if (dir.z < 0.0) old.z = K.zface[ck - 1] - delta;
      old.x = old.x + dir.x * dcell;
      old.y = old.y + dir.y * dcell;
    } else {  // error stop :570-573
      L.fault = true; pk.tflag = true; break;
    }
    ci = cell_of(old.x, K.nx, K.xmax); cj = cell_of(old.y, K.ny, K.ymax); ck = cell_of(old.z, K.nz, K.zmax);
    if (ci == -1 || cj == -1 || ck == -1) { pk.tflag = true; break; }
  }
  pk.xcell = ci; pk.ycell = cj; pk.zcell = ck;
}

// ------------------------------------------------------------------ detectors ----
// intersectCircle, geometryMod.f90:217-270
__device__ __forceinline__ bool intersect_circle(V3 n, V3 p0, double radius, V3 l0, V3 l, double& t, double& d2) {
  t = 0.0;
  const double denom = dot(n, l);
  if (denom > 1e-6) {
    const V3 p0l0 = p0 - l0;
    double tt = dot(p0l0, n);
    tt = tt / denom;
    t = tt;
    if (tt > -1e-6) {
      const V3 p = l0 + mul(l, tt);
      const V3 v = p - p0;
      d2 = sqrt(dot(v, v));
      if (d2 <= radius) return true;
    }
  }
  return false;
}

__device__ __forceinline__ int64_t f_nint(double x) {
  if (!(fabs(x) < 4.0e18)) return x > 0 ? (int64_t)4e18 : -(int64_t)4e18;
  return (int64_t)round(x);
}
__device__ __forceinline__ int64_t f_int(double x) {
  if (!(fabs(x) < 4.0e18)) return x > 0 ? (int64_t)4e18 : -(int64_t)4e18;
  return (int64_t)x;
}

// record_hit on every detector for one path segment (detector_base.f90:137-235)
__device__ void record_hits(const KParams& K, Lane& L, V3 start, V3 dir, double pointSep, int32_t layer,
                            double weight) {
  double value1D = (double)layer;  // hit_t%value1D <- packet%layer
  for (int32_t di = 0; di < K.n_dets; ++di) {
    const smcrt_detector* D = K.dets + di;
    const V3 dpos = v3(D->pos[0], D->pos[1], D->pos[2]);
    const V3 ddir = v3(D->dir[0], D->dir[1], D->dir[2]);
    double* data = K.det_bins ? K.det_bins + K.det_off[di] : nullptr;
    double t;
    if (D->kind == SMCRT_DET_CIRCLE) {  // detectors.f90:147-164
      bool hit = intersect_circle(ddir, dpos, D->radius, start, dir, t, value1D);
      if (hit && (t <= 0.0 || t > pointSep)) hit = false;
      if (hit) {
        int64_t idx = f_nint(value1D / D->bin_wid) + 1;
        if (idx > D->nbins) idx = D->nbins;
        if (idx >= 1) {
          if (data) atomic_add_nr(data + idx - 1, weight);
          L.c.v[SMCRT_CTR_DETECTOR_HITS]++;
        }
      }
    } else if (D->kind == SMCRT_DET_ANNULUS) {  // detectors.f90:212-244
      const bool h1 = intersect_circle(ddir, dpos, D->r1, start, dir, t, value1D);
      const bool h2 = intersect_circle(ddir, dpos, D->r2, start, dir, t, value1D);
      bool hit = false;
      if (!h1 && h2) hit = !(t <= 0.0 || t > pointSep);
      value1D = value1D - D->r1;
      if (hit) {
        int64_t idx = f_nint(value1D / D->bin_wid) + 1;
        if (idx > D->nbins) idx = D->nbins;
        if (idx >= 1) {
          if (data) atomic_add_nr(data + idx - 1, weight);
          L.c.v[SMCRT_CTR_DETECTOR_HITS]++;
        }
      }
    } else if (D->kind == SMCRT_DET_CAMERA) {  // detectors.f90:447-469
      const V3 e1 = v3(D->e1[0], D->e1[1], D->e1[2]), e2 = v3(D->e2[0], D->e2[1], D->e2[2]);
      const double tt = dot(dpos - start, ddir) / dot(dir, ddir);
      if (tt >= 0.0) {
        const V3 v = (start + smul(tt, dir)) - dpos;
        const double proj1 = dot(v, e1) / D->width;
        const double proj2 = dot(v, e2) / D->height;
        if ((proj1 < D->width && proj1 > 0.0) && (proj2 < D->height && proj2 > 0.0)) {
          const double x = start.z + D->pos[0];  // record_hit_2D_sub :206-235
          const double y = start.y + D->pos[1];
          int64_t idx = f_int(x / D->bin_wid) + 1;
          int64_t idy = f_int(y / D->bin_wid_y) + 1;
          if (idx > D->nbins) idx = D->nbins;
          if (idy > D->nbins) idy = D->nbins;
          if (idx < 1) idx = D->nbins;
          if (idy < 1) idy = D->nbins;
          if (data) atomic_add_nr(data + (idx - 1) + (int64_t)D->nbins * (idy - 1), 1.0);
          L.c.v[SMCRT_CTR_DETECTOR_HITS]++;
        }
      }
    }
  }
}

// ------------------------------------------------------------------ surfaces -----
// fresnel, surfaces.f90:86-127
__device__ __forceinline__ double fresnel(V3 I, V3 N, double n1, double n2) {
  double costt = fabs(dot(I, N));
  if (costt > 1.0) costt = 1.0;
  const double sintt = sqrt(1.0 - costt * costt);
  double sint2 = n1 / n2 * sintt;
  if (sint2 > 1.0) return 1.0;
  if (costt == 1.0) return 0.0;
  sint2 = (n1 / n2) * sintt;
  const double cost2 = sqrt(1.0 - sint2 * sint2);
  const double a = (n1 * costt - n2 * cost2) / (n1 * costt + n2 * cost2);
  const double b = (n1 * cost2 - n2 * costt) / (n1 * cost2 + n2 * costt);
  const double f1 = fabs(a) * fabs(a), f2 = fabs(b) * fabs(b);
  return 0.5 * (f1 + f2);
}

// calcNormal, sdf_base.f90:166-190
__device__ V3 calc_normal(const KParams& K, V3 p, int32_t top0) {
  const double h = 1e-6;
  const V3 xyy = v3(1.0, -1.0, -1.0), yyx = v3(-1.0, -1.0, 1.0), yxy = v3(-1.0, 1.0, -1.0), xxx = v3(1.0, 1.0, 1.0);
  const double e1 = sdf_top(K, top0, p + mul(xyy, h));
  const double e2 = sdf_top(K, top0, p + mul(yyx, h));
  const double e3 = sdf_top(K, top0, p + mul(yxy, h));
  const double e4 = sdf_top(K, top0, p + mul(xxx, h));
  const V3 n = ((mul(xyy, e1) + mul(yyx, e2)) + mul(yxy, e3)) + mul(xxx, e4);
  const double ln = len(n);
  return v3(n.x / ln, n.y / ln, n.z / ln);
}

__device__ __forceinline__ double pointsep(V3 a, V3 b) {
  const double dx = a.x - b.x, dy = a.y - b.y, dz = a.z - b.z;
  return sqrt(dx * dx + dy * dy + dz * dz);
}

// ------------------------------------------------------------------ tauint2 ------
// inttau2.f90:15-364
__device__ void tauint2(const KParams& K, Lane& L, Packet& pk, Rng& rng) {
  V3 pos = pk.pos, oldpos = pos, startPos = pos, dir = pk.n;
  const double eps = 1e-8;
  uint32_t& cnt = L.c.v[SMCRT_CTR_SDF_EVALS];
  L.c.v[SMCRT_CTR_TAUINT]++;
  const double tau = -det_log(rng.next());  // :58
  double taurun = 0.0, d_sdf, t_sdf;
  DsInfo I;
  const bool has_det = K.n_dets > 0;
  int64_t hop = 0;
  while (taurun <= tau) {  // :61
    if (++hop > MAX_HOP_ITERS) { L.fault = true; pk.tflag = true; break; }
    I = eval_all(K, pos, cnt);
    d_sdf = I.minabs;
    if (d_sdf < eps) {  // :73-146
      d_sdf = I.minabs + 2.0 * eps;
      const V3 ssp = pos + smul(d_sdf, dir);
      const DsInfo J = eval_all(K, ssp, cnt);
      const double kap = K.props[pk.layer - 1].kappa;
      oldpos = pos;
      t_sdf = d_sdf * kap;
      if (J.maxloc == pk.layer) {  // forward
        if (taurun + t_sdf < tau) {
          pos = pos + smul(d_sdf, dir);
          taurun = taurun + t_sdf;
          update_grids(K, L, oldpos, dir, d_sdf, pk);
        } else {
          d_sdf = (tau - taurun) / kap;
          taurun = taurun + t_sdf;
          update_grids(K, L, oldpos, dir, d_sdf, pk);
        }
      } else {  // backward
        if (taurun + t_sdf < tau) {
          pos = pos - smul(d_sdf, dir);
          taurun = taurun + t_sdf;
          update_grids(K, L, oldpos, dir, d_sdf, pk);
        } else {
          d_sdf = (tau - taurun) / kap;
          pos = pos - smul(d_sdf, dir);
          update_grids(K, L, oldpos, dir, d_sdf, pk);
        }
      }
      if (has_det) record_hits(K, L, startPos, dir, pointsep(pos, startPos), pk.layer, pk.weight);
      startPos = pos;
      I = eval_all(K, pos, cnt);
      d_sdf = I.minabs;
      if (I.minv > 0.0) pk.tflag = true;
    }
    if (taurun >= tau || pk.tflag) break;
    int64_t march = 0;
    while (d_sdf >= eps) {  // :155-192
      if (++march > MAX_MARCH_ITERS) { L.fault = true; pk.tflag = true; break; }
      const double kap = K.props[pk.layer - 1].kappa;
      t_sdf = d_sdf * kap;
      if (taurun + t_sdf < tau) {
        taurun = taurun + t_sdf;
        oldpos = pos;
        update_grids(K, L, oldpos, dir, d_sdf, pk);
        pos = pos + smul(d_sdf, dir);
      } else {
        d_sdf = (tau - taurun) / kap;
        taurun = tau;
        oldpos = pos;
        pos = pos + smul(d_sdf, dir);
        update_grids(K, L, oldpos, dir, d_sdf, pk);
        break;
      }
      I = eval_all(K, pos, cnt);
      d_sdf = I.minabs;
      if (I.minv > 0.0) { pk.tflag = true; break; }
    }
    if (has_det) record_hits(K, L, startPos, dir, pointsep(pos, startPos), pk.layer, pk.weight);
    startPos = pos;
    if (taurun >= tau || pk.tflag) break;
    // boundary crossing :213-235
    d_sdf = I.minabs + 2.0 * eps;
    V3 ssp = pos + smul(d_sdf, dir);
    DsInfo Nw = eval_all(K, ssp, cnt);
    int32_t new_layer = Nw.maxloc;
    double glancing = Nw.minabs;
    const int32_t old_layer = pk.layer;
    int64_t gl = 0;
    while (new_layer == old_layer && glancing < eps) {
      if (++gl > MAX_GLANCE_ITERS) { L.fault = true; pk.tflag = true; break; }
      d_sdf = d_sdf + eps;
      ssp = pos + smul(d_sdf, dir);
      Nw = eval_all(K, ssp, cnt);
      new_layer = Nw.maxloc;
      glancing = Nw.minabs;
    }
    if (pk.tflag) break;
    if (new_layer == 0) { pk.tflag = true; break; }  // :237-241
    const double n1 = K.props[pk.layer - 1].n, n2 = K.props[new_layer - 1].n;
    if (n1 != n2) {  // :248-317
      // ds/dsNew entries of the two layers involved, re-evaluated (same values as the
      // arrays the reference keeps)
      const double ds_new = sdf_top(K, new_layer - 1, pos), ds_old = sdf_top(K, old_layer - 1, pos);
      const double dn_new = sdf_top(K, new_layer - 1, ssp), dn_old = sdf_top(K, old_layer - 1, ssp);
      int32_t Ls;
      if (dn_new < 0.0 && ds_new >= 0.0) Ls = new_layer;
      else if (dn_old >= 0.0 && ds_old < 0.0) Ls = old_layer;
      else if (dn_new < 0.0 && dn_old < 0.0) Ls = new_layer;
      else if (ds_old >= 0.0 && dn_old >= 0.0) Ls = old_layer;
      else { L.fault = true; pk.tflag = true; break; }  // error stop :264-277
      const V3 N = calc_normal(K, pos, Ls - 1);
      L.c.v[SMCRT_CTR_FRESNEL]++;
      const double R = fresnel(dir, N, n1, n2);  // reflect_refract :14-40
      if (rng.next() <= R) {                     // reflect :42-55
        const double s = 2.0 * dot(N, dir);
        dir = dir - smul(s, N);
        L.c.v[SMCRT_CTR_REFLECTIONS]++;
        oldpos = pos;
        startPos = pos;
        pk.bounces += 1;
        if (pk.bounces > 1000) {  // :313-315, return without write-back
          L.c.v[SMCRT_CTR_BOUNCE_ABORTS]++;
          return;
        }
      } else {  // refract :57-84, then transmit :284-303
        const double eta = n1 / n2;
        V3 Nt = N;
        double c1 = dot(Nt, dir);
        if (c1 < 0.0) c1 = -c1;
        else Nt = smul(-1.0, N);
        const double c2 = sqrt(1.0 - (eta * eta) * (1.0 - c1 * c1));
        dir = smul(eta, dir) + smul(eta * c1 - c2, Nt);
        pk.layer = new_layer;
        oldpos = pos;
        update_grids(K, L, oldpos, dir, d_sdf, pk);
        t_sdf = d_sdf * K.props[pk.layer - 1].kappa;
        taurun = taurun + t_sdf;
        pos = ssp;
        if (has_det) record_hits(K, L, startPos, dir, pointsep(pos, startPos), pk.layer, pk.weight);
        startPos = pos;
      }
    } else {  // :318-336
      pk.layer = new_layer;
      oldpos = pos;
      update_grids(K, L, oldpos, dir, d_sdf, pk);
      t_sdf = d_sdf * K.props[pk.layer - 1].kappa;
      taurun = taurun + t_sdf;
      pos = ssp;
      if (has_det) record_hits(K, L, startPos, dir, pointsep(pos, startPos), pk.layer, pk.weight);
      startPos = pos;
    }
    if (pk.tflag) break;
  }
  pk.pos = pos;  // :341-362
  pk.n = dir;
  if (fabs(pk.pos.x) > K.xmax) pk.tflag = true;
  if (fabs(pk.pos.y) > K.ymax) pk.tflag = true;
  if (fabs(pk.pos.z) > K.zmax) pk.tflag = true;
}

// ------------------------------------------------------------------ scatter ------
// photon.f90:1045-1103
__device__ void scatter(Lane& L, Packet& pk, double hgg, Rng& rng) {
  double cost, temp;
  if (hgg == 0.0) {
    cost = 2.0 * rng.next() - 1.0;
  } else {
    temp = (1.0 - hgg * hgg) / (1.0 - hgg + 2.0 * hgg * rng.next());
    cost = (1.0 + hgg * hgg - temp * temp) / (2.0 * hgg);
  }
  const double sint = sqrt(1.0 - cost * cost);
  const double phi = 6.283185307179586 * rng.next();
  double sinp, cosp;
  det_sincos(phi, &sinp, &cosp);
  const double nxp = pk.n.x, nyp = pk.n.y, nzp = pk.n.z;
  double uxx, uyy, uzz;
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
    if (++it > MAX_RENORM_ITERS) { L.fault = true; pk.tflag = true; break; }
    uxx = uxx / temp; uyy = uyy / temp; uzz = uzz / temp;
    temp = sqrt(uxx * uxx + uyy * uyy + uzz * uzz);
  }
  pk.n = v3(uxx, uyy, uzz);
}

// ------------------------------------------------------------------ emit ---------
__device__ void emit(const KParams& K, Packet& pk, Rng& rng) {
  const smcrt_source& s = K.src;
  if (s.kind == SMCRT_SRC_POINT) {  // photon.f90:311-359
    pk.pos = v3(s.pos[0], s.pos[1], s.pos[2]);
    const double phi = rng.next() * 6.283185307179586;
    double sinp, cosp;
    det_sincos(phi, &sinp, &cosp);
    const double cost = 2.0 * rng.next() - 1.0;
    const double sint = sqrt(1.0 - cost * cost);
    pk.n = v3(sint * cosp, sint * sinp, cost);
    pk.layer = 1;
  } else {
    if (s.kind == SMCRT_SRC_UNIFORM) {  // photon.f90:566-649
      const double rx = rng.next(), ry = rng.next();
      pk.pos = v3(s.p1[0] + rx * s.p2[0] + ry * s.p3[0], s.p1[1] + rx * s.p2[1] + ry * s.p3[1],
                  s.p1[2] + rx * s.p2[2] + ry * s.p3[2]);
    } else {  // pencil :652-710
      pk.pos = v3(s.pos[0], s.pos[1], s.pos[2]);
      pk.layer = 1;
    }
    if (pk.pos.x == -K.xmax) pk.pos.x = pk.pos.x + 7.9e-7;
    else if (pk.pos.x == K.xmax) pk.pos.x = pk.pos.x - 7.9e-7;
    if (pk.pos.y == -K.ymax) pk.pos.y = pk.pos.y + 7.9e-7;
    else if (pk.pos.y == K.ymax) pk.pos.y = pk.pos.y - 7.9e-7;
    if (pk.pos.z == -K.zmax) pk.pos.z = pk.pos.z + 7.9e-7;
    else if (pk.pos.z == K.zmax) pk.pos.z = pk.pos.z - 7.9e-7;
    pk.n = v3(s.dir[0], s.dir[1], s.dir[2]);
  }
  pk.tflag = false;
  pk.bounces = 0;
  pk.weight = 1.0;
  pk.xcell = vox_of(pk.pos.x, K.nx, K.xmax);
  pk.ycell = vox_of(pk.pos.y, K.ny, K.ymax);
  pk.zcell = vox_of(pk.pos.z, K.nz, K.zmax);
}

__device__ __forceinline__ bool cell_out(const KParams& K, const Packet& pk) {
  return pk.xcell < 1 || pk.xcell > K.nx || pk.ycell < 1 || pk.ycell > K.ny || pk.zcell < 1 || pk.zcell > K.nz;
}

__device__ __forceinline__ void add_cell(const KParams& K, double* g, const Packet& pk, double w, Lane& L) {
  if (cell_out(K, pk)) { L.fault = true; return; }
  if (g) atomic_add_nr(g + lin(K, pk.xcell, pk.ycell, pk.zcell), w);
}

// One photon: noBiasPropagation (kernelsMod.f90:1901-1976), survivalBiasPropagation
// (:1979-2067) or the test_kernel body (:2124-2171).
__device__ void run_photon(const KParams& K, Lane& L, uint64_t pid, smcrt_photon_record* rec) {
  Rng rng;
  rng.init(pid, K.seed);
  Packet pk;
  pk.layer = 0; pk.nscatt = 0; pk.xcell = pk.ycell = pk.zcell = 0;
  pk.pos = v3(0.0, 0.0, 0.0); pk.n = pk.pos; pk.weight = 1.0; pk.bounces = 0; pk.tflag = false;
  const bool test_kernel = (K.flags & SMCRT_FLAG_TEST_KERNEL) != 0;
  uint32_t status = 0;
  L.fault = false;
  emit(K, pk, rng);
  if (!test_kernel) {
    int64_t tries = 0;
    while (cell_out(K, pk)) {  // :1939-1943
      if (++tries > MAX_EMIT_TRIES) { L.fault = true; break; }
      L.c.v[SMCRT_CTR_EMIT_RETRIES]++;
      emit(K, pk, rng);
    }
    if (!L.fault && (K.flags & SMCRT_FLAG_RENDER_SOURCE)) add_cell(K, K.emission, pk, 1.0, L);
  }
  if (!L.fault) {
    uint32_t not_counted = 0;
    const DsInfo I = eval_all(K, pk.pos, not_counted, test_kernel);  // :1948-1952
    pk.layer = I.maxloc;
    if (pk.layer == 0) L.fault = true;
  }
  if (!L.fault) {
    tauint2(K, L, pk, rng);
    int64_t inter = 0;
    while (!pk.tflag && !L.fault) {  // :1958-1975
      if (++inter > MAX_INTERACTIONS) { L.fault = true; break; }
      const double ran = rng.next();
      const TopProps pr = K.props[pk.layer - 1];
      if (K.flags & SMCRT_FLAG_SURVIVAL_BIAS) {
        const double w_abs = pk.weight * (1.0 - pr.albedo);
        pk.weight = pk.weight - w_abs;
        add_cell(K, K.absorb, pk, w_abs, L);
        if (pk.weight < 0.01) {
          if (ran < 0.1) {
            pk.weight = pk.weight / 0.1;
          } else {
            pk.tflag = true;
            status = 1;
            L.c.v[SMCRT_CTR_ABSORBED]++;
            break;
          }
        }
        scatter(L, pk, pr.hgg, rng);
        pk.nscatt++;
        L.nscatt += 1.0;
        L.c.v[SMCRT_CTR_SCATTERS]++;
      } else if (ran < pr.albedo) {
        scatter(L, pk, pr.hgg, rng);
        pk.nscatt++;
        L.nscatt += 1.0;
        L.c.v[SMCRT_CTR_SCATTERS]++;
        if (test_kernel) {  // :2142-2163
          const uint32_t st = pk.nscatt;
          if (st >= 1 && st <= 4) {
            if (K.moments) {
              double* m = K.moments + 3 * (st - 1);
              double* m2 = K.moments + 12 + 3 * (st - 1);
              atomic_add_nr(m + 0, pk.pos.x); atomic_add_nr(m + 1, pk.pos.y); atomic_add_nr(m + 2, pk.pos.z);
              atomic_add_nr(m2 + 0, pk.pos.x * pk.pos.x);
              atomic_add_nr(m2 + 1, pk.pos.y * pk.pos.y);
              atomic_add_nr(m2 + 2, pk.pos.z * pk.pos.z);
            }
          } else if (K.flags & SMCRT_FLAG_END_EARLY) {
            pk.tflag = true;
            status = 4;
          }
        }
      } else {
        pk.tflag = true;
        status = 1;
        L.c.v[SMCRT_CTR_ABSORBED]++;
        if (!test_kernel) add_cell(K, K.absorb, pk, 1.0, L);  // recordWeight(packet, 1.0)
        break;
      }
      tauint2(K, L, pk, rng);
    }
  }
  if (L.fault) { status = 3; L.c.v[SMCRT_CTR_FAULTS]++; }
  else if (status == 0) { status = 2; L.c.v[SMCRT_CTR_ESCAPED]++; }
  L.c.v[SMCRT_CTR_PHOTONS]++;
  L.c.v[SMCRT_CTR_RNG_DRAWS] += rng.draws;
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

}  // namespace smcrt
