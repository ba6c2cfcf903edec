// transport.h — the per-photon hot path as a CDNA4 per-lane state machine.
//
// One wavefront lane carries one photon packet (fp64 state in VGPRs). The reference's
// nested loops (noBiasPropagation kernelsMod.f90:1901-1976 -> tauint2 inttau2.f90:15-364
// -> update_grids :367-465) are unrolled into program points ("states"); every iteration of
// the kernel's single loop does, per lane:
//   1. DDA:     up to DDA_PER_ITER voxel crossings of the lane's pending deposit segment;
//   2. EVAL:    one evaluation of the whole SDF array at the lane's query point, if its
//               state asked for one (the only copy of the SDF code in the kernel: wave-
//               uniform loop, scalar-loaded parameters, no divergence);
//   3. ADVANCE: the control logic of the reference from the current program point to the
//               next one that needs an EVAL or a DDA segment.
// A lane whose photon terminates fetches the next photon index (wave-aggregated atomic on a
// work queue) without waiting for the rest of its wave (persistent-threads regeneration).
//
// Each program point cites the reference lines it restates. Arithmetic is in the
// reference's order with -ffp-contract=off, so every photon's trajectory, tallies and RNG
// consumption are bit-identical to the CPU restatement.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/smcrt.h"
#include "detmath.h"
#include "geometry.h"
#include "srcplan.h"
#include "cull.h"

namespace smcrt {

// Unbounded loops of the reference are capped; the CPU restatement uses the same caps.
constexpr int64_t MAX_EMIT_TRIES = 100000;
constexpr int64_t MAX_HOP_ITERS = 1000000;
constexpr int64_t MAX_MARCH_ITERS = 10000000;
constexpr int64_t MAX_GLANCE_ITERS = 100000;
constexpr int64_t MAX_DDA_ITERS = 10000000;
constexpr int MAX_RENORM_ITERS = 64;
constexpr int64_t MAX_INTERACTIONS = 100000000;

// transport_kernel walks at most this many crossings of a lane's segment per trip (round 2:
// more while many lanes still walk was box-dependent, profiles/r02_s3/dda_schedule_ab.txt)
#define SMCRT_DDA_PER_ITER 3
// photons a wave takes from the work queue with one atomic
#define SMCRT_FETCH_CHUNK 64
// transport_kernel runs its photon-event phase once this many lanes wait for it (or no lane
// has anything else to do)
#define SMCRT_EVENT_LANES 16

// Optical properties of a top-level SDF, derived as init_mono does
// (opticalProperties.f90:107-125).
struct TopProps {
  double kappa, albedo, hgg, n;
};

// Launch parameters read only at rare program points (fetch of a new photon chunk,
// emission, interactions, completion). They live in device memory behind a pointer and are
// loaded where used, so they do not occupy scalar registers for the whole kernel.
struct KCold {
  smcrt_source src;
  uint64_t n_photons, first_photon;
  double* absorb;
  double* emission;
  double* det_bins;
  double* nscatt;
  double* moments;
  unsigned long long* counters;
  smcrt_photon_record* records;
  unsigned long long* queue;  // photon work-queue head (zeroed before launch)
  double* jmean;              // fp64 atomics: the unbinned path and pool overflow
  uint32_t* chunk_fill;       // records in each used chunk (deposit.h)
  uint32_t* dep_ctl;          // [0] next chunk, [1] overflowed deposits
  uint32_t* bin_counts;       // fused tile histogram, counts[tile][chunk % BIN_BLOCKS]
  uint32_t* bucket_tile;      // bucketed path: tile of each bucket id (TILE_INVALID: unused)
  uint32_t* bucket_fill;      // bucketed path: records in each bucket
  uint32_t* tile_nb;          // bucketed path: buckets claimed per tile
  unsigned long long* far_steps;  // march steps taken by the far-field march (far.h), running total
  unsigned long long* lean_hazards;  // deferred lean segments ending in tflag / a fault (lean.h), running total
  double* lane_scratch;       // ws_kernel's per-photon-lane Fresnel/detector state (ws.h WX_*), or null
  // the watchdog (round 6): every cross-wave wait of the kernels is bounded by watchdog_ticks of
  // s_memrealtime (SMCRT_WATCHDOG_MS; 0 = unbounded); the first wait past it stores
  // site | (block + 1) << 8 here (smcrt_scene_check / smcrt_run return SMCRT_ERR_DEVICE_FAULT
  // naming the site) and its wave gives up the wait, so the grid drains instead of hanging
  uint32_t* watchdog;
  uint64_t watchdog_ticks;
#ifdef SMCRT_DIAG
  // diagnostic builds: each photon's completion time (s_memrealtime) at done_time[pid - done_base]
  // (smcrt_diag_done_times; SMCRT_DIAG_DONE=1), or null
  unsigned long long* done_time;
  uint64_t done_base;
#endif
  SrcPlan plan;               // the general emitter's constants (XSRC instantiations only)
};

// watchdog sites (KCold::watchdog bits 0-7; smcrt.hip names them)
enum : uint32_t {
  WDOG_PHOTON_WAVE = 1,  // ws_kernel photon wave: every live lane waited (event, segment, slot)
  WDOG_RING = 2,         // ws_kernel ring producer: its word's previous lap was never consumed
  WDOG_EVENT_QUEUE = 3,  // ws_kernel event-queue producer: likewise
  WDOG_BUCKET = 4        // deposit.h bucket wait: the pending claim never rebased the tile word
};
// true once a wait that started at t0 has run past the budget; the first such wait of the
// launch records its site
__device__ __forceinline__ bool watchdog_expired(const KCold* __restrict__ C, uint64_t t0, uint32_t site) {
  const uint64_t budget = C->watchdog_ticks;
  if (budget == 0 || __builtin_amdgcn_s_memrealtime() - t0 <= budget) return false;
  atomicCAS(C->watchdog, 0u, site | ((blockIdx.x + 1u) << 8));
  return true;
}

struct KParams {
  const smcrt_sdf_node* __restrict__ nodes;
  const ProgOp* __restrict__ prog;
  const TopProps* __restrict__ props;
  const double* __restrict__ xface;  // nx+1
  const double* __restrict__ yface;  // ny+1
  const double* __restrict__ zface;  // nz+2
  const smcrt_detector* __restrict__ dets;
  const int64_t* __restrict__ det_off;
  int32_t n_prog, n_top, n_dets;
  int32_t coop_lanes;  // cooperative EVAL when at most this many lanes need one (0 = never)
  int32_t nx, ny, nz;
  uint32_t flags;
  double xmax, ymax, zmax;
  // exact reciprocal of 2*max when that is a power of two (else 0): n*p/(2*max) == n*p*inv
  double inv2x, inv2y, inv2z;
  int32_t fex, fey, fez;  // GM == 2: face k = k * 2^fe (see face())
  uint32_t key0, key1;  // Philox key = seed words
  // binned jmean deposition (deposit.h): record log in chunks
  unsigned long long* rec_pool;  // CHUNK_RECORDS records per chunk; NULL -> fp64 atomics into jmean
  uint32_t n_chunks;
  // fused tile histogram (deposit.h): counts[tile][chunk % BIN_BLOCKS] built by the
  // transport kernel from a per-wave LDS histogram; hist_tiles == 0 -> bin_hist does it
  uint32_t hist_tiles;
  // bucketed deposition (deposit.h): records go straight into per-tile buckets of the pool;
  // bucket_tiles != 0 selects it (and is the tile count), n_buckets is the pool's size
  uint32_t bucket_tiles, n_buckets;
  // debug knob (SMCRT_DEBUG_CLAIM_DELAY, tests only): s_sleep 127 this many times before a
  // bucket claim's CAS, so that other waves fill both buckets of the tile and wait (deposit.h)
  uint32_t claim_delay;
  // debug knob (SMCRT_DEBUG_LEAN_MARGIN, tests only), bits 0-1: 0 = lean.h's margin; 1 = no
  // margin; 2 = every segment that starts in the grid is deferred, so escapes become counted
  // hazards. Bit 2 (SMCRT_DEBUG_DROP_EVENT, tests only): photon lane 0 of block 0 marks its first
  // event queued without queueing it (the hang class the watchdog turns into a counted fault)
  uint32_t lean_debug;
  // the lean path's deferral box (lean.h lean_margin, corner coordinates), formed on the host so
  // that the photon waves read six wave-uniform doubles with scalar loads instead of keeping
  // them in VGPRs (they were spilled to scratch and reloaded at every hand-out)
  double lean_lo[3], lean_hi[3];
  // exact SDF culling (cull.h), many-top scenes in the COOP instantiation; NULL = off
  const CullGrid* __restrict__ cull;
  // the cooperative EVAL's table of primitives (CTAB_ROWS x 64 doubles, column = top - 1),
  // staged in LDS by the COOP instantiation; NULL when the scene does not qualify
  const double* __restrict__ ctab;
  // far-field march (far.h), COOP instantiation with ctab: the absolute error bound of a
  // computed top-level SDF value and the per-step bound on the rounding of p + d*dir (both
  // from the scene's extent); fm_err == 0 turns it off
  double fm_err, fm_step;
};

// ------------------------------------------------------------------ voxels -------
// update_voxels, inttau2.f90:587-614 (corner coordinates): floor(n*p/(2*max))+1, -1 outside
// GM >= 1: every axis has 2*max a power of two, so the division is an exact multiply (the kernel
// is instantiated for it; the general case keeps a per-axis uniform branch).
template <int GM>
__device__ __forceinline__ double cell_floor(double p, int32_t n, double max, double inv, int32_t fe) {
  if constexpr (GM == 2) return floor(ldexp(p, -fe));  // n/(2*max) == 2^-fe: one exact scaling
  const double a = (double)n * p;
  return floor(GM >= 1 ? a * inv : (inv != 0.0 ? a * inv : a / (2.0 * max)));
}
// v_cvt_i32_f64 saturates out-of-range values (a C++ conversion of those is undefined)
__device__ __forceinline__ int32_t cvt_sat_i32(double f) {
  int32_t r;
  asm("v_cvt_i32_f64 %0, %1" : "=v"(r) : "v"(f));
  return r;
}
template <int GM>
__device__ __forceinline__ int32_t cell_of(double p, int32_t n, double max, double inv, int32_t fe) {
  const double f = cell_floor<GM>(p, n, max, inv, fe);
  if (!(f >= 0.0 && f < (double)n)) return -1;
  return (int32_t)f + 1;
}
// get_voxel_cart, grid.f90:51-78 (centred coordinates)
template <int GM>
__device__ __forceinline__ int32_t vox_of(double p, int32_t n, double max, double inv, int32_t fe) {
  return cell_of<GM>(p + max, n, max, inv, fe);
}

template <int GM>
__device__ __forceinline__ double face(const double* __restrict__ f, int32_t k, int32_t ex) {
  if constexpr (GM == 2) return ldexp((double)k, ex);
  else return f[k];
}

__device__ __forceinline__ void atomic_add_nr(double* p, double v) {
  __hip_atomic_fetch_add(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
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

// record_hit on every detector for one path segment (detector_base.f90:137-235,
// detectors.f90:147-469). Returns the number of bin increments.
// `totals` (batched point sources): add each hit to totals[detector] (total_dect,
// detector_base.f90) instead of to its bin.
__device__ __forceinline__ uint32_t record_hits(const KParams& K, double* det_bins,
                                                const smcrt_detector* __restrict__ dets,
                                                const int64_t* __restrict__ det_off, V3 start, V3 dir,
                                                double pointSep, int32_t layer, double weight,
                                                double* totals = nullptr) {
  uint32_t hits = 0;
  double value1D = (double)layer;  // hit_t%value1D <- packet%layer
  for (int32_t di = 0; di < K.n_dets; ++di) {
    const smcrt_detector* D = dets + di;
    const V3 dpos = v3(D->pos[0], D->pos[1], D->pos[2]);
    const V3 ddir = v3(D->dir[0], D->dir[1], D->dir[2]);
    double* data = det_bins ? det_bins + det_off[di] : nullptr;
    double t;
    int64_t bin = -1;
    double w = weight;
    if (D->kind == SMCRT_DET_CIRCLE || D->kind == SMCRT_DET_ANNULUS) {
      // A hit needs 0 < t <= pointSep for t = dot(pos - start, dir) / dot(dir, dir of the ray)
      // as intersect_circle rounds it (numerator and denominator computed the same way here):
      // a segment that cannot reach the detector's plane skips the intersection (no bin, and
      // value1D is only read after a hit). The 1e-9 margin covers the quotient's rounding.
      const double den = dot(ddir, dir);
      const double num = dot(dpos - start, ddir);
      if (!(den > 1e-6) || !(num > 0.0) || num > pointSep * den * (1.0 + 1e-9)) continue;
    }
    if (D->kind == SMCRT_DET_CIRCLE) {
      bool hit = intersect_circle(ddir, dpos, D->radius, start, dir, t, value1D);
      if (hit && (t <= 0.0 || t > pointSep)) hit = false;
      if (hit) {
        int64_t idx = f_nint(value1D / D->bin_wid) + 1;
        if (idx > D->nbins) idx = D->nbins;
        if (idx >= 1) bin = idx - 1;
      }
    } else if (D->kind == SMCRT_DET_ANNULUS) {
      const bool h1 = intersect_circle(ddir, dpos, D->r1, start, dir, t, value1D);
      const bool h2 = intersect_circle(ddir, dpos, D->r2, start, dir, t, value1D);
      bool hit = false;
      if (!h1 && h2) hit = !(t <= 0.0 || t > pointSep);
      value1D = value1D - D->r1;
      if (hit) {
        int64_t idx = f_nint(value1D / D->bin_wid) + 1;
        if (idx > D->nbins) idx = D->nbins;
        if (idx >= 1) bin = idx - 1;
      }
    } else if (D->kind == SMCRT_DET_CAMERA) {
      const V3 e1 = v3(D->e1[0], D->e1[1], D->e1[2]), e2 = v3(D->e2[0], D->e2[1], D->e2[2]);
      const double tt = dot(dpos - start, ddir) / dot(dir, ddir);
      if (tt >= 0.0) {
        const V3 v = (start + smul(tt, dir)) - dpos;
        const double proj1 = dot(v, e1) / D->width;
        const double proj2 = dot(v, e2) / D->height;
        if ((proj1 < D->width && proj1 > 0.0) && (proj2 < D->height && proj2 > 0.0)) {
          const double x = start.z + D->pos[0];  // record_hit_2D_sub uses hit%pos
          const double y = start.y + D->pos[1];
          int64_t idx = f_int(x / D->bin_wid) + 1;
          int64_t idy = f_int(y / D->bin_wid_y) + 1;
          if (idx > D->nbins) idx = D->nbins;
          if (idy > D->nbins) idy = D->nbins;
          if (idx < 1) idx = D->nbins;
          if (idy < 1) idy = D->nbins;
          bin = (idx - 1) + (int64_t)D->nbins * (idy - 1);
          w = 1.0;
        }
      }
    } else if (D->kind == SMCRT_DET_FIBRE) {  // check_hit_fibre, detectors.f90:331-393 (4f thin-lens chain)
      const double* F = D->fibre;  // focalLength1, focalLength2, f1Aperture, f2Aperture, frontOffset,
                                   // backOffset, frontToPinSep, pinToBackSep, pinAperture, acceptAngle, core
      bool hit = intersect_circle(ddir, dpos + mul(ddir, F[4]), F[2], start, dir, t, value1D);
      if (hit && (t <= 0.0 || t > pointSep)) hit = false;
      if (hit) {
        double costt = dot(ddir, dir);
        if (costt > 1.0) costt = 1.0;
        const double sintt = sqrt(1.0 - costt * costt);
        double gradient = sintt / costt;
        double radius = value1D;
        gradient = -radius / F[0] + gradient;    // front lens
        radius = radius + gradient * F[6];       // to the pinhole
        if (radius > F[8]) {
          hit = false;
        } else {
          radius = radius + gradient * F[7];     // to the back lens
          if (radius > F[3]) {
            hit = false;
          } else {
            gradient = -radius / F[1] + gradient;
            radius = radius + gradient * F[5];   // to the fibre
            const double angle = fabs(det_atan(gradient)) * 360.0 / 6.283185307179586;
            if (angle > F[9] || radius > (F[10] / 2.0)) hit = false;
            value1D = fabs(radius);
          }
        }
      }
      if (hit) {
        int64_t idx = f_nint(value1D / D->bin_wid) + 1;
        if (idx > D->nbins) idx = D->nbins;
        if (idx >= 1) bin = idx - 1;
      }
    }
    if (bin >= 0) {
      if (totals) atomic_add_nr(totals + di, w);
      else if (data) atomic_add_nr(data + bin, w);
      ++hits;
    }
  }
  return hits;
}

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

__device__ __forceinline__ double pointsep(V3 a, V3 b) {
  const double dx = a.x - b.x, dy = a.y - b.y, dz = a.z - b.z;
  return sqrt(dx * dx + dy * dy + dz * dz);
}

// ------------------------------------------------------------------ lane state ---
enum : uint32_t {
  ST_IDLE = 0,   // no photon and the queue is empty
  ST_FETCH,      // needs a photon index (fetched wave-wide at the end of ADVANCE)
  ST_EMIT,       // emit (+ re-emission), kernelsMod.f90:1937-1945
  ST_LAYER,      // EVAL at pos: initial layer = maxloc(ds, mask ds<0), :1948-1952
  ST_T2,         // tauint2 entry, inttau2.f90:48-60
  ST_H0,         // hop-loop head, EVAL at pos, :61-73
  ST_H1,         // on-surface micro-step, EVAL at smallStepPos, :77-123
  ST_H2,         // after its deposit: detectors, :125-131
  ST_H3,         // EVAL at pos, :133-146
  ST_M0,         // march-loop head, :155-176
  ST_M1,         // EVAL at pos after a march step, :177-191
  ST_B0,         // after the march: detectors, boundary probe, :195-214
  ST_G0,         // EVAL at smallStepPos (+ glancing loop), :214-245
  ST_X1,         // after a crossing deposit: tau, pos, detectors, :294-303 / :326-335
  ST_F0,         // Fresnel: ds(new), ds(old) at pos (EVAL, capture)
  ST_F1,         // Fresnel: dsNew(new), dsNew(old) at smallStepPos (EVAL, capture), :250-277
  ST_N1,         // calcNormal taps 1..4 (EVAL, capture), sdf_base.f90:166-190
  ST_N2,
  ST_N3,
  ST_N4,
  ST_T2END,      // tauint2 write-back checks, :341-362
  ST_DONE,       // photon finished: tallies, record, next photon
  ST_INTERACT,   // albedo roulette / survival bias + scatter, kernelsMod.f90:1958-1975, 2036-2065
};

// Per-lane state kept in VGPRs. Rarely touched values (tauint2 entry pos/dir for the
// bounce abort, most counters) live in LDS (LaneShared) instead.
struct Lane {
  // photon packet
  V3 pos, dir;
  double weight;
  int32_t xcell, ycell, zcell, layer;
  bool tflag, fault;  // bounces, nscatt, status: LDS (LaneShared::u)
  Rng rng;
  // tauint2 locals
  double tau, taurun, d;
  V3 ssp;              // startPos: LDS (LaneShared::start)
  double minabs;       // minval(abs(ds)) of the last EVAL at pos
  int32_t old_layer, new_layer, Ls;
  uint32_t hop, loopc;  // hop / march-or-glance loop guards (interactions: LDS)
  // state machine
  uint32_t st;
  bool pend;  // an EVAL was requested for the current state
  // deposit segment (update_grids in progress). While no segment is active (the Fresnel
  // sequence F0..N4), old/sd/slen hold the captured SDF values instead.
  bool seg;
  V3 old;  // DDA position, corner coordinates
  double sd, slen;
  uint32_t dda_it;  // (the DDA's voxel is xcell/ycell/zcell)
};

// LDS-resident per-lane values, [field][threadIdx] so lanes never share a bank.
// Everything here is touched at most a few times per photon, so it lives in LDS instead of
// costing a register for the whole kernel.
enum : int { LC_PHOTONS = 0, LC_RETRIES, LC_SCATTERS, LC_ABSORBED, LC_TAU, LC_FRES, LC_REFL, LC_BABORT,
             LC_FAULTS, LC_DRAWS, LC_HITS, LC_ESCAPED, LC_UPD, LC_N };
enum : int { LU_INTER = 0, LU_BOUNCES, LU_NSCATT, LU_STATUS, LU_ORIGIN, LU_N };  // per-photon fields
struct LaneShared {
  uint32_t ctr[LC_N][256];
  uint32_t u[LU_N][256];
  double entry[6][256];  // tauint2 entry pos/dir, restored on a bounce abort (inttau2.f90:313-315)
  // (startPos of the detector segments, inttau2.f90:59,125-131, is in dynamic LDS and only
  // allocated when the scene has detectors)
};
#define LCTR(c) (sh->ctr[(c)][threadIdx.x])
#define LU(f) (sh->u[(f)][threadIdx.x])

__device__ __forceinline__ bool is_eval_state(uint32_t s) {
  return s == ST_LAYER || s == ST_H0 || s == ST_H1 || s == ST_H3 || s == ST_M1 || s == ST_G0 || s == ST_F0 ||
         s == ST_F1 || s == ST_N1 || s == ST_N2 || s == ST_N3 || s == ST_N4;
}

__device__ __forceinline__ bool cell_out(const KParams& K, const Lane& L) {
  return L.xcell < 1 || L.xcell > K.nx || L.ycell < 1 || L.ycell > K.ny || L.zcell < 1 || L.zcell > K.nz;
}

// Voxel index, x fastest (Fortran order). Grids are limited to < 2^32 voxels (scene_create).
__device__ __forceinline__ uint32_t lin(const KParams& K, int32_t i, int32_t j, int32_t k) {
  return (uint32_t)(i - 1) + (uint32_t)K.nx * ((uint32_t)(j - 1) + (uint32_t)K.ny * (uint32_t)(k - 1));
}

__device__ __forceinline__ void add_cell(const KParams& K, double* g, Lane& L, double w) {
  if (cell_out(K, L)) { L.fault = true; return; }
  if (g) atomic_add_nr(g + lin(K, L.xcell, L.ycell, L.zcell), w);
}

// ------------------------------------------------------------------ general emitter ----
// Kernels instantiated with XSRC run every source of photon.f90 and sample the source
// spectrum (piecewise.f90); the others keep the three-source emitter below it. The launch-
// invariant parts (matrices, CDFs) come from the host (srcplan.h).

// search_1D, piecewise.f90:254-275: bisection with middle = int((nup+nlow)/2.) in default
// (single) precision; returns the 1-based nlow.
__device__ __forceinline__ int64_t search_1d(const double* __restrict__ a, int64_t n, double v) {
  int64_t nup = n, nlow = 1;
  while ((nup - nlow) > 1) {
    const int64_t middle = (int64_t)((float)(nup + nlow) / 2.0f);
    if (v > a[middle - 1]) nlow = middle;
    else nup = middle;
  }
  return nlow;
}
__device__ __forceinline__ uint32_t pack_bits(uint64_t x) {  // piecewise.f90:296-315
  x &= 0x5555555555555555ull;
  x = (x >> 1) | x; x &= 0x3333333333333333ull;
  x = (x >> 2) | x; x &= 0x0F0F0F0F0F0F0F0Full;
  x = (x >> 4) | x; x &= 0x00FF00FF00FF00FFull;
  x = (x >> 8) | x; x &= 0x0000FFFF0000FFFFull;
  x = (x >> 16) | x;
  return (uint32_t)x;
}
// ranu(a, b) = a + ran2()*(b - a), random_mod.f90:93-103
__device__ __forceinline__ double ranu(const KParams& K, Lane& L, double a, double b) {
  return a + L.rng.next(K.key0, K.key1) * (b - a);
}
// spectrum%p%sample(x, y): constant getValue :93-107, sample1D :109-137, sample2D :171-188
__device__ __forceinline__ void spec_sample(const KParams& K, const SrcPlan& P, Lane& L, double& x, double& y) {
  if (P.spec_kind == SMCRT_SPEC_1D) {
    const double val = L.rng.next(K.key0, K.key1);
    const int64_t i = search_1d(P.cdf, P.spec_n, val);  // 1-based
    const double* a = P.spec_x;
    x = a[i - 1] + ((val - P.cdf[i - 1]) * (a[i] - a[i - 1])) / (P.cdf[i] - P.cdf[i - 1]);
    y = 0.0;  // (undefined in the reference; never used)
  } else if (P.spec_kind == SMCRT_SPEC_2D) {
    const double val = L.rng.next(K.key0, K.key1);
    const int64_t i = search_1d(P.cdf, P.spec_n, val);
    const int32_t xr = (int32_t)pack_bits((uint64_t)i), yr = (int32_t)pack_bits((uint64_t)i >> 1);
    x = (double)(xr - P.xoff) + ranu(K, L, -P.cell_w, P.cell_w);
    y = (double)(yr - P.yoff) + ranu(K, L, -P.cell_h, P.cell_h);
  } else {
    x = P.wavelength;
    y = -9999.0;
  }
}
__device__ __forceinline__ void nudge_faces(const KParams& K, V3& p) {  // e.g. photon.f90:614-628
  if (p.x == -K.xmax) p.x = p.x + 7.9e-7;
  else if (p.x == K.xmax) p.x = p.x - 7.9e-7;
  if (p.y == -K.ymax) p.y = p.y + 7.9e-7;
  else if (p.y == K.ymax) p.y = p.y - 7.9e-7;
  if (p.z == -K.zmax) p.z = p.z + 7.9e-7;
  else if (p.z == K.zmax) p.z = p.z - 7.9e-7;
}
__device__ __forceinline__ V3 magnitude(V3 a) {  // vector_class.f90:392-402
  const double t = len(a);
  return v3(a.x / t, a.y / t, a.z / t);
}
// focus/annulus: dir = magnitude(sign(1,f) * (-(p - targ)/|p - targ|)) with targ = (0,0,-f),
// then rotated and renormalised (photon.f90:430-472 / :902-944)
__device__ __forceinline__ V3 beam_dir(const SrcPlan& P, V3 q) {
  const V3 d0 = q - v3(0.0, 0.0, -P.focal);
  const double dist = len(d0);
  V3 d = smul(-1.0, d0);
  d = v3(d.x / dist, d.y / dist, d.z / dist);
  d = mul(d, copysign(1.0, P.focal));
  d = magnitude(d);
  return magnitude(dotmat(d, P.R));
}
// the step back into the grid of focus (cap 4) and annulus (cap 3), photon.f90:505-556
__device__ __forceinline__ void step_into_grid(const KParams& K, Lane& L, int cap) {
  bool inX = false, inY = false, inZ = false, tX = false, tY = false, tZ = false;
  int counter = 0;
  V3& p = L.pos;
  const V3 d = L.dir;
  while (!inX || !inY || !inZ) {
    double st;
    if (p.x <= -K.xmax) { st = (-K.xmax - p.x + 9e-7) / d.x; p = v3(p.x + d.x * st, p.y + d.y * st, p.z + d.z * st); tX = true; }
    else if (p.x >= K.xmax) { st = (K.xmax - p.x - 9e-7) / d.x; p = v3(p.x + d.x * st, p.y + d.y * st, p.z + d.z * st); tX = true; }
    else inX = true;
    if (p.y <= -K.ymax) { st = (-K.ymax - p.y + 9e-7) / d.y; p = v3(p.x + d.x * st, p.y + d.y * st, p.z + d.z * st); tY = true; }
    else if (p.y >= K.ymax) { st = (K.ymax - p.y - 9e-7) / d.y; p = v3(p.x + d.x * st, p.y + d.y * st, p.z + d.z * st); tY = true; }
    else inY = true;
    if (p.z <= -K.zmax) { st = (-K.zmax - p.z + 9e-7) / d.z; p = v3(p.x + d.x * st, p.y + d.y * st, p.z + d.z * st); tZ = true; }
    else if (p.z >= K.zmax) { st = (K.zmax - p.z - 9e-7) / d.z; p = v3(p.x + d.x * st, p.y + d.y * st, p.z + d.z * st); tZ = true; }
    else inZ = true;
    if ((tX && tY && tZ) || counter > cap) break;
    counter = counter + 1;
  }
}

constexpr int MAX_RANG_TRIES = 1000;  // rang's rejection loop (random_mod.f90:116-121), capped

// pos/dir of one emission for every source kind (the cells are set by the caller)
// `oidx`: the lane's origin in a batched point-source run (SrcPlan::origins).
__device__ __forceinline__ void emit_ext(const KParams& K, const SrcPlan& P, Lane& L, uint32_t oidx) {
  const double TWOPI = 6.283185307179586;
  double wl, tmp;
  switch (P.kind) {
    case SMCRT_SRC_POINT: {  // photon.f90:311-359
      if (P.origins) {  // set_photon(voxel centre) before each run_MCRT, kernelsMod.f90:579-580
        const double* o = P.origins + 3 * (uint64_t)oidx;
        L.pos = v3(o[0], o[1], o[2]);
      } else {
        L.pos = v3(P.origin[0], P.origin[1], P.origin[2]);
      }
      const double phi = L.rng.next(K.key0, K.key1) * TWOPI;
      double sinp, cosp;
      det_sincos(phi, &sinp, &cosp);
      const double cost = 2.0 * L.rng.next(K.key0, K.key1) - 1.0;
      const double sint = sqrt(1.0 - cost * cost);
      L.dir = v3(sint * cosp, sint * sinp, cost);
      L.layer = 1;
      spec_sample(K, P, L, wl, tmp);
      break;
    }
    case SMCRT_SRC_UNIFORM: {  // :566-649
      const double rx = L.rng.next(K.key0, K.key1), ry = L.rng.next(K.key0, K.key1);
      L.dir = v3(P.dir[0], P.dir[1], P.dir[2]);
      L.pos = v3(P.p1[0] + rx * P.p2[0] + ry * P.p3[0], P.p1[1] + rx * P.p2[1] + ry * P.p3[1],
                 P.p1[2] + rx * P.p2[2] + ry * P.p3[2]);
      nudge_faces(K, L.pos);
      spec_sample(K, P, L, wl, tmp);
      break;
    }
    case SMCRT_SRC_PENCIL: {  // :652-710
      L.pos = v3(P.origin[0], P.origin[1], P.origin[2]);
      nudge_faces(K, L.pos);
      L.dir = v3(P.dir[0], P.dir[1], P.dir[2]);
      L.layer = 1;
      spec_sample(K, P, L, wl, tmp);
      break;
    }
    case SMCRT_SRC_CIRCULAR: {  // :214-308
      L.dir = v3(P.dir[0], P.dir[1], P.dir[2]);
      const double r = P.radius * sqrt(L.rng.next(K.key0, K.key1));
      const double theta = L.rng.next(K.key0, K.key1) * TWOPI;
      double st, ct;
      det_sincos(theta, &st, &ct);
      const V3 q = P.circ_z ? v3(r * ct, r * st, 0.0) : v3(0.0, r * ct, r * st);
      const V3 t = dotmat(q, P.T);
      L.pos = v3(-t.x, -t.y, -t.z);
      nudge_faces(K, L.pos);
      spec_sample(K, P, L, wl, tmp);
      L.layer = 1;
      break;
    }
    case SMCRT_SRC_FOCUS:      // :361-563
    case SMCRT_SRC_ANNULUS: {  // :850-1043
      V3 q, qd;
      if (P.kind == SMCRT_SRC_FOCUS) {
        if (P.beam == SMCRT_BEAM_SQUARE) {
          const double x = ranu(K, L, -P.beam_size, P.beam_size);
          const double y = ranu(K, L, -P.beam_size, P.beam_size);
          q = v3(x, y, 0.0);
        } else {
          double radius;
          if (P.beam == SMCRT_BEAM_CIRCLE) radius = P.beam_size * sqrt(L.rng.next(K.key0, K.key1));
          else radius = P.beam_size * sqrt(-det_log(1.0 - L.rng.next(K.key0, K.key1)));
          const double phi = TWOPI * L.rng.next(K.key0, K.key1);
          double sinp, cosp;
          det_sincos(phi, &sinp, &cosp);
          q = v3(radius * cosp, radius * sinp, 0.0);
        }
        qd = q;
      } else {
        double radius, mid;
        if (P.beam == SMCRT_BEAM_TOPHAT) {
          radius = sqrt(P.rlo * P.rlo + (P.rhi * P.rhi - P.rlo * P.rlo) * L.rng.next(K.key0, K.key1));
          mid = (P.rhi + P.rlo) / 2.0;
        } else if (P.beam == SMCRT_BEAM_BESSEL) {
          radius = P.rlo + (P.rhi - P.rlo) * L.rng.next(K.key0, K.key1);
          mid = (P.rhi + P.rlo) / 2.0;
        } else {  // gaussian: rang(radius, tmp, mid, sigma), random_mod.f90:105-127
          mid = (P.rhi + P.rlo) / 2.0;
          double x = 0.0, y = 0.0, s = 1.0;
          int tries = 0;
          while (s >= 1.0) {
            if (++tries > MAX_RANG_TRIES) { L.fault = true; break; }
            x = ranu(K, L, -1.0, 1.0);
            y = ranu(K, L, -1.0, 1.0);
            s = y * y + x * x;
          }
          radius = mid + P.sigma * (x * sqrt(-2.0 * det_log(s) / s));
        }
        const double phi = TWOPI * L.rng.next(K.key0, K.key1);
        double sinp, cosp;
        det_sincos(phi, &sinp, &cosp);
        q = v3(radius * cosp, radius * sinp, 0.0);
        qd = v3(mid * cosp, mid * sinp, 0.0);
      }
      L.dir = beam_dir(P, qd);
      L.pos = dotmat(q, P.T);
      spec_sample(K, P, L, wl, tmp);
      step_into_grid(K, L, P.kind == SMCRT_SRC_FOCUS ? 4 : 3);
      break;
    }
    case SMCRT_SRC_SLM: {  // :159-212
      double x, y;
      spec_sample(K, P, L, x, y);
      L.pos = v3((x - 100.0) / ((double)P.nx / (2.0 * P.xmax)), (y - 100.0) / ((double)P.ny / (2.0 * P.ymax)),
                 P.origin[2]);
      L.dir = v3(P.dir[0], P.dir[1], P.dir[2]);
      L.layer = 1;
      break;
    }
    default: {  // dslit :712-780, aperture :782-848
      spec_sample(K, P, L, wl, tmp);
      double x1, y1, z1, x2, y2, z2;
      if (P.kind == SMCRT_SRC_DSLIT) {
        const double a = 60.0 * wl, b = 20.0 * wl;
        if (L.rng.next(K.key0, K.key1) > 0.5) {
          x1 = ranu(K, L, a / 2.0, a / 2.0 + b);
          y1 = ranu(K, L, -b * 0.5, b * 0.5);
        } else {
          x1 = ranu(K, L, -a / 2.0, -a / 2.0 - b);
          y1 = ranu(K, L, -b * 0.5, b * 0.5);
        }
        z2 = 5.0 - (1.e-5 * (2.0 * (5.0 / 400.0)));
        x2 = ranu(K, L, -5.0, 5.0);
        y2 = ranu(K, L, -5.0, 5.0);
        z1 = (10000.0 * wl) - 5.0;
      } else {
        const double apwid = 200e-6, b = apwid / 2.0, F = 4.95;
        x1 = ranu(K, L, -b, b);
        y1 = ranu(K, L, -b, b);
        const double fa = F / apwid;
        z1 = (1.0 / (((fa * fa) / 2.0) * wl)) - 0.5;
        x2 = ranu(K, L, -0.5, 0.5);
        y2 = ranu(K, L, -0.5, 0.5);
        z2 = 0.5 - (1.e-5 * (2.0 * 0.5 / 400.0));
      }
      L.pos = v3(x2, y2, z2);
      const double dx = x2 - x1, dy = y2 - y1, dz = z2 - z1;
      const double phase = sqrt(dx * dx + dy * dy + dz * dz);
      L.dir = v3(dx / phase, dy / phase, -fabs(dz) / phase);
      break;
    }
  }
}

// emit: point photon.f90:311-359 / uniform :566-649 / pencil :652-710
template <int GM, bool XSRC>
__device__ __forceinline__ void emit(const KParams& K, const KCold* __restrict__ C, Lane& L, uint32_t oidx) {
  const smcrt_source& s = C->src;
  if constexpr (XSRC) {
    emit_ext(K, C->plan, L, oidx);
  } else if (s.kind == SMCRT_SRC_POINT) {
    L.pos = v3(s.pos[0], s.pos[1], s.pos[2]);
    const double phi = L.rng.next(K.key0, K.key1) * 6.283185307179586;
    double sinp, cosp;
    det_sincos(phi, &sinp, &cosp);
    const double cost = 2.0 * L.rng.next(K.key0, K.key1) - 1.0;
    const double sint = sqrt(1.0 - cost * cost);
    L.dir = v3(sint * cosp, sint * sinp, cost);
    L.layer = 1;
  } else {
    if (s.kind == SMCRT_SRC_UNIFORM) {
      const double rx = L.rng.next(K.key0, K.key1), ry = L.rng.next(K.key0, K.key1);
      L.pos = v3(s.p1[0] + rx * s.p2[0] + ry * s.p3[0], s.p1[1] + rx * s.p2[1] + ry * s.p3[1],
                 s.p1[2] + rx * s.p2[2] + ry * s.p3[2]);
    } else {
      L.pos = v3(s.pos[0], s.pos[1], s.pos[2]);
      L.layer = 1;
    }
    if (L.pos.x == -K.xmax) L.pos.x = L.pos.x + 7.9e-7;
    else if (L.pos.x == K.xmax) L.pos.x = L.pos.x - 7.9e-7;
    if (L.pos.y == -K.ymax) L.pos.y = L.pos.y + 7.9e-7;
    else if (L.pos.y == K.ymax) L.pos.y = L.pos.y - 7.9e-7;
    if (L.pos.z == -K.zmax) L.pos.z = L.pos.z + 7.9e-7;
    else if (L.pos.z == K.zmax) L.pos.z = L.pos.z - 7.9e-7;
    L.dir = v3(s.dir[0], s.dir[1], s.dir[2]);
  }
  L.tflag = false;
  L.weight = 1.0;
  L.xcell = vox_of<GM>(L.pos.x, K.nx, K.xmax, K.inv2x, K.fex);
  L.ycell = vox_of<GM>(L.pos.y, K.ny, K.ymax, K.inv2y, K.fey);
  L.zcell = vox_of<GM>(L.pos.z, K.nz, K.zmax, K.inv2z, K.fez);
}

// scatter, photon.f90:1045-1103
__device__ __forceinline__ void scatter(const KParams& K, Lane& L, double hgg) {
  double cost, temp;
  if (hgg == 0.0) {
    cost = 2.0 * L.rng.next(K.key0, K.key1) - 1.0;
  } else {
    temp = (1.0 - hgg * hgg) / (1.0 - hgg + 2.0 * hgg * L.rng.next(K.key0, K.key1));
    cost = (1.0 + hgg * hgg - temp * temp) / (2.0 * hgg);
  }
  const double sint = sqrt(1.0 - cost * cost);
  const double phi = 6.283185307179586 * L.rng.next(K.key0, K.key1);
  double sinp, cosp;
  det_sincos(phi, &sinp, &cosp);
  const double nxp = L.dir.x, nyp = L.dir.y, nzp = L.dir.z;
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
    if (++it > MAX_RENORM_ITERS) { L.fault = true; L.tflag = true; break; }
    uxx = uxx / temp; uyy = uyy / temp; uzz = uzz / temp;
    temp = sqrt(uxx * uxx + uyy * uyy + uzz * uzz);
  }
  L.dir = v3(uxx, uyy, uzz);
}

// update_grids entry (inttau2.f90:401-415): start a deposit segment from `p` (centred) of
// length `dlen` along L.dir; the segment itself runs in the DDA phase. Returns true if the
// lane must wait for the DDA.
template <int GM>
__device__ __forceinline__ bool start_segment(const KParams& K, Lane& L, LaneShared* sh, V3 p, double dlen) {
  LCTR(LC_UPD)++;
  V3 old = v3(p.x + K.xmax, p.y + K.ymax, p.z + K.zmax);
  int32_t ci = cell_of<GM>(old.x, K.nx, K.xmax, K.inv2x, K.fex), cj = cell_of<GM>(old.y, K.ny, K.ymax, K.inv2y, K.fey),
          ck = cell_of<GM>(old.z, K.nz, K.zmax, K.inv2z, K.fez);
  L.xcell = ci; L.ycell = cj; L.zcell = ck;
  if (!(K.flags & SMCRT_FLAG_PATHLENGTH)) {  // :446-463
    old.x = old.x + L.dir.x * dlen;
    old.y = old.y + L.dir.y * dlen;
    old.z = old.z + L.dir.z * dlen;
    ci = cell_of<GM>(old.x, K.nx, K.xmax, K.inv2x, K.fex); cj = cell_of<GM>(old.y, K.ny, K.ymax, K.inv2y, K.fey);
    ck = cell_of<GM>(old.z, K.nz, K.zmax, K.inv2z, K.fez);
    if (ci == -1 || cj == -1 || ck == -1) L.tflag = true;
    L.xcell = ci; L.ycell = cj; L.zcell = ck;
    return false;
  }
  if (ci == -1 || cj == -1 || ck == -1) { L.tflag = true; return false; }
  L.old = old; L.sd = 0.0; L.slen = dlen; L.dda_it = 0;
  L.seg = true;
  return true;
}

// One voxel crossing of the pending segment: wall_dist + deposit + update_pos
// (inttau2.f90:417-441, 467-584). Clears L.seg when the segment ends. `L` is any state with
// the segment fields of Lane (old, sd, slen, xcell/ycell/zcell, dda_it, seg, tflag, fault):
// the photon's own Lane, or a walker's segment (lean.h); `dir` is the segment's direction.
// (dda_step_r: the same crossing with the direction's refined reciprocals (ieee_rcp_f64 of
// each component) supplied by the caller, e.g. kept by a walker for its whole segment.)
template <int GM, class S>
__device__ __forceinline__ void dda_step_r(const KParams& K, S& L, const V3 dir, const V3 rcp,
                                           const double* __restrict__ xf, const double* __restrict__ yf,
                                           const double* __restrict__ zf, bool& dep, uint32_t& dep_vox,
                                           double& dep_val, double weight);
template <int GM, class S>
__device__ __forceinline__ void dda_step(const KParams& K, S& L, const V3 dir, const double* __restrict__ xf,
                                         const double* __restrict__ yf, const double* __restrict__ zf,
                                         bool& dep, uint32_t& dep_vox, double& dep_val, double weight) {
  const V3 rcp = v3(ieee_rcp_f64(dir.x), ieee_rcp_f64(dir.y), ieee_rcp_f64(dir.z));
  dda_step_r<GM>(K, L, dir, rcp, xf, yf, zf, dep, dep_vox, dep_val, weight);
}
template <int GM, class S>
__device__ __forceinline__ void dda_step_r(const KParams& K, S& L, const V3 dir, const V3 rcp3,
                                           const double* __restrict__ xf, const double* __restrict__ yf,
                                           const double* __restrict__ zf, bool& dep, uint32_t& dep_vox,
                                           double& dep_val, double weight) {
#ifdef SMCRT_ASM_MARKERS
  asm volatile("; @@DDA_BEGIN");
#endif
  const bool capped = ++L.dda_it > (uint32_t)MAX_DDA_ITERS;  // runaway guard: fault
  // wall_dist, :467-521: d_a = (face_a - old_a)/dir_a, dcell = min, ldir_a = (dcell == d_a).
  // Only the smallest quotient is needed exactly: the three are ranked by products with
  // the refined reciprocals (relative error far below the 2^-16 margin required), and the
  // one winner is divided exactly. If the ranking is not clear-cut by that margin (near-ties, zero
  // or negative distances, a zero direction component, NaN), all three are divided exactly
  // as the reference does. Both paths give the reference's dcell and ldir bit for bit.
  // the wall each axis moves towards: xface(ci+1) going +, xface(ci) going - (0-based here)
  const double fx = face<GM>(xf, dir.x > 0.0 ? L.xcell : L.xcell - 1, K.fex);
  const double fy = face<GM>(yf, dir.y > 0.0 ? L.ycell : L.ycell - 1, K.fey);
  const double fz = face<GM>(zf, dir.z > 0.0 ? L.zcell : L.zcell - 1, K.fez);
  const double nx = fx - L.old.x;
  const double ny = fy - L.old.y;
  const double nz = fz - L.old.z;
  // The reciprocal half of the IEEE fp64 division sequence (v_rcp_f64 + two Newton steps, as
  // the compiler expands `n / d`) depends on the direction only, so it is computed once per
  // trip (the compiler hoists it out of the unrolled crossings); per crossing only the
  // numerator half (mul, residual fma, correction fma) remains.
  const double rx = rcp3.x, ry = rcp3.y, rz = rcp3.z;
  const double ax = nx * rx;
  const double ay = ny * ry;
  const double az = nz * rz;
  // Clear-cut: exactly two estimates lie above the margin over the smallest. (A NaN is
  // above nothing, so it can never leave two above: such lanes take the exact path.)
  const double amin = fmin(fmin(ax, ay), az);
  const double thr = amin * (1.0 + 0x1.0p-16);
  const bool ux = ax > thr, uy = ay > thr, uz = az > thr;
  const bool two = ((ux ^ uy) ^ uz) == false && (ux || uy || uz);
  // (the magnitude bounds keep the operands where the division sequence does no scaling)
  const bool fast0 = two && amin > 0.0 && fabs(dir.x) >= 0x1.0p-500 && fabs(dir.y) >= 0x1.0p-500 &&
                     fabs(dir.z) >= 0x1.0p-500;
  bool lx = !ux, ly = !uy, lz = !uz;
  const double num = lx ? nx : (ly ? ny : nz), den = lx ? dir.x : (ly ? dir.y : dir.z);
  const double rcp = lx ? rx : (ly ? ry : rz);
  const bool fast = fast0 && fabs(num) >= 0x1.0p-500;
  double dcell;
  if (fast) {
    dcell = ieee_div_tail_f64(num, den, rcp);  // == num / den bit for bit
  } else {
    double dx = -999.0, dy = -999.0, dz = -999.0;
    if (dir.x > 0.0 || dir.x < 0.0) dx = nx / dir.x;
    else if (dir.x == 0.0) dx = 100000.0;
    if (dir.y > 0.0 || dir.y < 0.0) dy = ny / dir.y;
    else if (dir.y == 0.0) dy = 100000.0;
    if (dir.z > 0.0 || dir.z < 0.0) dz = nz / dir.z;
    else if (dir.z == 0.0) dz = 100000.0;
    dcell = dmin(dmin(dx, dy), dz);
    lx = (dcell == dx); ly = (dcell == dy); lz = (dcell == dz);
  }
  // The rest of the crossing is written as selects, not branches: lanes of a wave reach
  // different outcomes here on almost every step, and divergent branches cost more than
  // computing both sides.
  const bool neg = dcell < 0.0;  // error stop :510-516
  const bool ok = !capped && !neg;
  const double sdn = L.sd + dcell;
  const bool last = sdn > L.slen;
  const double dc = last ? L.slen - L.sd : dcell;
  // jmean(cell) += real(dcell,sp)*weight (inttau2.f90:427,434): handed to the caller,
  // which appends a deposit record (binned path) or adds it atomically
  dep = ok;
  dep_vox = lin(K, L.xcell, L.ycell, L.zcell);
  dep_val = (double)(float)dc * weight;
  // update_pos (:524-584): .false. (last step) advances all three coordinates by dc;
  // .true. snaps the first axis with ldir set to its wall +- delta (unchanged if its
  // direction is 0) and advances the other two.
  const double delta = 1e-8;  // local delta, :393
  const double vx = L.old.x + dir.x * dc, vy = L.old.y + dir.y * dc, vz = L.old.z + dir.z * dc;
  // (face - delta == face + (-delta) exactly, so one add with a signed delta)
  const double sx = dir.x > 0.0 || dir.x < 0.0 ? fx + (dir.x > 0.0 ? delta : -delta) : L.old.x;
  const double sy = dir.y > 0.0 || dir.y < 0.0 ? fy + (dir.y > 0.0 ? delta : -delta) : L.old.y;
  const double sz = dir.z > 0.0 || dir.z < 0.0 ? fz + (dir.z > 0.0 ? delta : -delta) : L.old.z;
  const bool noaxis = !(lx || ly || lz);  // error stop :570-573
  const bool snap = ok && !last && !noaxis;
  const bool snx = lx, sny = !lx && ly, snz = !lx && !ly;
  // Without a snap the segment ends here and the DDA position is dead, so only the snap
  // case is selected (a zero direction component keeps its coordinate: vx == old.x then).
  const double px = snx && (dir.x > 0.0 || dir.x < 0.0) ? sx : vx;
  const double py = sny && (dir.y > 0.0 || dir.y < 0.0) ? sy : vy;
  const double pz = snz && (dir.z > 0.0 || dir.z < 0.0) ? sz : vz;
  // update_voxels, :587-614 (an out-of-range floor converts to an out-of-range integer)
  const int32_t gx = cvt_sat_i32(cell_floor<GM>(px, K.nx, K.xmax, K.inv2x, K.fex));
  const int32_t gy = cvt_sat_i32(cell_floor<GM>(py, K.ny, K.ymax, K.inv2y, K.fey));
  const int32_t gz = cvt_sat_i32(cell_floor<GM>(pz, K.nz, K.zmax, K.inv2z, K.fez));
  const bool inx = (uint32_t)gx < (uint32_t)K.nx, iny = (uint32_t)gy < (uint32_t)K.ny,
             inz = (uint32_t)gz < (uint32_t)K.nz;
  const bool left = snap && !(inx && iny && inz);  // left the grid, :437-440
  L.old = v3(px, py, pz);
  L.sd = sdn;  // (dead once the segment ends, as old is)
  L.xcell = snap ? (inx ? gx + 1 : -1) : L.xcell;
  L.ycell = snap ? (iny ? gy + 1 : -1) : L.ycell;
  L.zcell = snap ? (inz ? gz + 1 : -1) : L.zcell;
  const bool bad = capped || neg || (ok && !last && noaxis);
  if (bad || left) {  // error stops and leaving the grid: rare, so a (skipped) branch
    L.fault = L.fault || bad;
    L.tflag = true;
  }
  L.seg = !(bad || (ok && last) || left);
#ifdef SMCRT_ASM_MARKERS
  asm volatile("; @@DDA_END");
#endif
}

#ifndef SMCRT_EVAL_PAIRS
#define SMCRT_EVAL_PAIRS 1
#endif
// The EVAL phase: ds(i) for every top-level SDF at L.q, reduced to minval(abs(ds)),
// minval(ds), maxloc(ds, mask) and the captured ds(capi), ds(capj).
struct EvalOut {
  double minabs, minv, va, vb;
  int32_t maxloc;
};

// `nodes` and `prog` must come from `const __restrict__` kernel parameters: that is what lets
// the compiler prove them unclobbered and keep the wave-uniform loads on the scalar path.
// NEST: the program may hold nested-model ops (PROG_SUB); only the general instantiation
// evaluates such scenes (smcrt.hip), so every other caller compiles without them.
// PAIRS: two consecutive top-level spheres or boxes at a time (see below); transport_kernel
// (M5 46.3-47.6 vs 43.4-43.8 M photons/s) but not ws_kernel's photon waves (M1 -1.4 %, M0
// -2.3 %), profiles/r06_s6/ab_eval_pairs.txt
template <bool NEST = false, bool PAIRS = false>
__device__ __forceinline__ EvalOut eval_sdfs(const smcrt_sdf_node* __restrict__ nodes,
                                             const ProgOp* __restrict__ prog, int32_t n_prog, V3 q,
                                             bool mask_le, int32_t capi, int32_t capj) {
  EvalOut r;
  r.minabs = __builtin_inf();
  r.minv = __builtin_inf();
  r.va = 0.0; r.vb = 0.0;
  r.maxloc = 0;
  double best = -__builtin_inf();
  double acc = 0.0;
  for (int32_t ip = 0; ip < n_prog; ++ip) {
    const ProgOp op = prog[ip];
#if SMCRT_EVAL_PAIRS
    // two consecutive top-level spheres or boxes (any order) as straight-line code: the kinds
    // are constants there (sdf_prim_s: the same operations), so the two evaluations' latency
    // chains overlap; folded in program order, as below (wave-uniform branch)
    if (PAIRS && !NEST && ip + 1 < n_prog && op.action == PROG_TOP && op.top > 0) {
      const ProgOp op2 = prog[ip + 1];
      if (op2.action == PROG_TOP && op2.top > 0) {
        const smcrt_sdf_node* n1 = nodes + __builtin_amdgcn_readfirstlane(op.node);
        const smcrt_sdf_node* n2 = nodes + __builtin_amdgcn_readfirstlane(op2.node);
        const int32_t k1 = n1->kind, k2 = n2->kind;
        const bool t1 = op.translate_only != 0, t2 = op2.translate_only != 0;
        double v1 = 0.0, v2 = 0.0;
        bool pair = true;
        if (k1 == SMCRT_SDF_SPHERE && k2 == SMCRT_SDF_BOX) {
          v1 = sdf_prim_s<1>(SMCRT_SDF_SPHERE, n1->transform, n1->param, q, t1);
          v2 = sdf_prim_s<1>(SMCRT_SDF_BOX, n2->transform, n2->param, q, t2);
        } else if (k1 == SMCRT_SDF_BOX && k2 == SMCRT_SDF_BOX) {
          v1 = sdf_prim_s<1>(SMCRT_SDF_BOX, n1->transform, n1->param, q, t1);
          v2 = sdf_prim_s<1>(SMCRT_SDF_BOX, n2->transform, n2->param, q, t2);
        } else if (k1 == SMCRT_SDF_BOX && k2 == SMCRT_SDF_SPHERE) {
          v1 = sdf_prim_s<1>(SMCRT_SDF_BOX, n1->transform, n1->param, q, t1);
          v2 = sdf_prim_s<1>(SMCRT_SDF_SPHERE, n2->transform, n2->param, q, t2);
        } else if (k1 == SMCRT_SDF_SPHERE && k2 == SMCRT_SDF_SPHERE) {
          v1 = sdf_prim_s<1>(SMCRT_SDF_SPHERE, n1->transform, n1->param, q, t1);
          v2 = sdf_prim_s<1>(SMCRT_SDF_SPHERE, n2->transform, n2->param, q, t2);
        } else {
          pair = false;
        }
        if (pair) {
          const double dv[2] = {v1, v2};
          const int32_t tv[2] = {op.top, op2.top};
#pragma unroll
          for (int u = 0; u < 2; ++u) {
            const double d = dv[u];
            const int32_t i = tv[u];
            const double a = fabs(d);
            if (a < r.minabs) r.minabs = a;
            if (d < r.minv) r.minv = d;
            const bool neg = mask_le ? (d <= 0.0) : (d < 0.0);
            if (neg && (r.maxloc == 0 || d > best)) { best = d; r.maxloc = i; }
            if (i == capi) r.va = d;
            if (i == capj) r.vb = d;
          }
          ++ip;
          continue;
        }
      }
    }
#endif
    // the program is wave-uniform: keep node parameters on the scalar path
    const int32_t node = __builtin_amdgcn_readfirstlane(op.node);
    const double v = prog_value<NEST>(nodes, node, op.action, op.translate_only != 0, q);
    if ((op.action & 3) == PROG_TOP) acc = v;
    else if ((op.action & 3) == PROG_CHILD_FIRST) acc = v;
    else acc = csg(op.op, acc, v, op.k);
    if (op.top > 0) {  // a top-level ds(i) is complete
      const double d = acc;
      const int32_t i = op.top;
      const double a = fabs(d);
      if (a < r.minabs) r.minabs = a;
      if (d < r.minv) r.minv = d;
      const bool neg = mask_le ? (d <= 0.0) : (d < 0.0);
      if (neg && (r.maxloc == 0 || d > best)) { best = d; r.maxloc = i; }
      if (i == capi) r.va = d;
      if (i == capj) r.vb = d;
    }
  }
  return r;
}

// Cooperative EVAL: the whole wave evaluates the SDF array for one lane's query point `q`.
// Lane j runs the programs of tops j+1, j+65, ... (prog[n_prog + i].node holds the first op
// of top i+1, prog[n_prog + n_top].node == n_prog), then the wave reduces the partials. Used
// in a launch's tail, where a wave has only a few live photons and eval_sdfs' serial chain of
// dependent scalar loads and fp64 ops over every top is pure latency (one sphere ~1000
// cycles). Results equal eval_sdfs': min/abs-min are exact, maxloc ties go to the lowest top
// index as eval_sdfs' strict compares do, and the captured values come from the owning lane.
// (minv may differ from eval_sdfs' in the sign of a zero; it is only ever tested with > 0.)
template <bool NEST = false>
__device__ __forceinline__ EvalOut eval_sdfs_coop(const smcrt_sdf_node* __restrict__ nodes,
                                                           const ProgOp* __restrict__ prog, int32_t n_prog,
                                                           int32_t n_top, V3 q, bool mask_le, int32_t capi,
                                                           int32_t capj) {
  const int32_t lane = (int32_t)(threadIdx.x & 63);
  double minabs = __builtin_inf(), minv = __builtin_inf(), best = -__builtin_inf();
  double va = 0.0, vb = 0.0;
  int32_t loc = 0;
  for (int32_t i = lane; i < n_top; i += 64) {
    const int32_t b = prog[n_prog + i].node, e = prog[n_prog + i + 1].node;
    if (b == e) continue;  // an empty model never completes its ds(i)
    double acc = 0.0;
    for (int32_t ip = b; ip < e; ++ip) {
      const ProgOp op = prog[ip];
      const double v = prog_value<NEST>(nodes, op.node, op.action, op.translate_only != 0, q);
      if ((op.action & 3) == PROG_TOP || (op.action & 3) == PROG_CHILD_FIRST) acc = v;
      else acc = csg(op.op, acc, v, op.k);
    }
    const double d = acc;
    const int32_t t = i + 1;
    const double a = fabs(d);
    if (a < minabs) minabs = a;
    if (d < minv) minv = d;
    const bool neg = mask_le ? (d <= 0.0) : (d < 0.0);
    if (neg && (loc == 0 || d > best)) { best = d; loc = t; }
    if (t == capi) va = d;
    if (t == capj) vb = d;
  }
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) {
    const double m2 = __shfl_xor(minabs, off, 64);
    if (m2 < minabs) minabs = m2;
    const double v2 = __shfl_xor(minv, off, 64);
    if (v2 < minv) minv = v2;
    const double b2 = __shfl_xor(best, off, 64);
    const int32_t l2 = __shfl_xor(loc, off, 64);
    if (l2 != 0 && (loc == 0 || b2 > best || (b2 == best && l2 < loc))) { best = b2; loc = l2; }
  }
  EvalOut r;
  r.minabs = minabs;
  r.minv = minv;
  r.maxloc = loc;
  r.va = capi > 0 ? __shfl(va, (capi - 1) & 63, 64) : 0.0;
  r.vb = capj > 0 ? __shfl(vb, (capj - 1) & 63, 64) : 0.0;
  return r;
}

// ---- cooperative EVAL from an LDS table (COOP instantiation, at most 64 single-primitive
// tops). Lane j keeps top j+1 in column j of a [CTAB_ROWS][64] fp64 table: transform rows
// 0-11, parameters 12-19, kind + 16 * translate_only in row 20. A sparse wave evaluates one
// lane's query point with every lane computing its own top from LDS (no vector memory on the
// path, so nothing waits for the wave's outstanding record stores) and reduces with DPP.
constexpr int CTAB_ROWS = 21;
constexpr int CTAB_DOUBLES = CTAB_ROWS * 64;

__device__ __forceinline__ double readlane_f64(double v, int l) {
  const uint64_t b = (uint64_t)__double_as_longlong(v);
  const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)b, l);
  const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(b >> 32), l);
  return __longlong_as_double((long long)(((uint64_t)hi << 32) | lo));
}
// v of the DPP source lane, or `old` where the control selects none (bound_ctrl off)
template <int CTRL, int ROWS>
__device__ __forceinline__ double dpp_f64(double old, double v) {
  const uint64_t b = (uint64_t)__double_as_longlong(v), o = (uint64_t)__double_as_longlong(old);
  const uint32_t lo = (uint32_t)__builtin_amdgcn_update_dpp((int)(uint32_t)o, (int)(uint32_t)b, CTRL, ROWS, 0xf, false);
  const uint32_t hi =
      (uint32_t)__builtin_amdgcn_update_dpp((int)(uint32_t)(o >> 32), (int)(uint32_t)(b >> 32), CTRL, ROWS, 0xf, false);
  return __longlong_as_double((long long)(((uint64_t)hi << 32) | lo));
}
template <int CTRL, int ROWS>
__device__ __forceinline__ int32_t dpp_i32(int32_t old, int32_t v) {
  return __builtin_amdgcn_update_dpp(old, v, CTRL, ROWS, 0xf, false);
}
struct CoopAcc {
  double minabs, minv, best;
  int32_t loc;
};
// Fold b into a: the serial scan's strict compares, maxloc ties to the lowest top index.
__device__ __forceinline__ void coop_fold(CoopAcc& a, const CoopAcc& b) {
  if (b.minabs < a.minabs) a.minabs = b.minabs;
  if (b.minv < a.minv) a.minv = b.minv;
  if (b.loc != 0 && (a.loc == 0 || b.best > a.best || (b.best == a.best && b.loc < a.loc))) {
    a.best = b.best;
    a.loc = b.loc;
  }
}
template <int CTRL, int ROWS>
__device__ __forceinline__ void coop_step(CoopAcc& a) {
  CoopAcc b;
  b.minabs = dpp_f64<CTRL, ROWS>(__builtin_inf(), a.minabs);
  b.minv = dpp_f64<CTRL, ROWS>(__builtin_inf(), a.minv);
  b.best = dpp_f64<CTRL, ROWS>(-__builtin_inf(), a.best);
  b.loc = dpp_i32<CTRL, ROWS>(0, a.loc);
  coop_fold(a, b);
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

// The whole wave evaluates the SDF array at the wave-uniform point q (all lanes active).
// (lane_d, if given, receives the lane's own ds(lane + 1), 0 past n_top)
__device__ __forceinline__ EvalOut eval_coop_tab(const double* ct, int32_t n_top, V3 q, bool mask_le, int32_t capi,
                                                 int32_t capj, double* lane_d = nullptr) {
  const int lane = (int)(threadIdx.x & 63);
  CoopAcc a;
  a.minabs = __builtin_inf(); a.minv = __builtin_inf(); a.best = -__builtin_inf(); a.loc = 0;
  double d = 0.0;
  if (lane < n_top) {
    const double kc = ct[20 * 64 + lane];
    const int32_t kind = (int32_t)kc & 15;
    d = sdf_prim_s<64>(kind, ct + lane, ct + 12 * 64 + lane, q, kc >= 16.0);
    a.minabs = fabs(d);
    a.minv = d;
    const bool neg = mask_le ? (d <= 0.0) : (d < 0.0);
    if (neg) { a.best = d; a.loc = lane + 1; }
  }
  // inclusive row scans (row_shr 1, 2, 4, 8), then row 0 -> 1 and 2 -> 3 (row_bcast:15),
  // then rows 0-1 -> 2-3 (row_bcast:31): lane 63 holds the wave's fold
  coop_step<0x111, 0xf>(a);
  coop_step<0x112, 0xf>(a);
  coop_step<0x114, 0xf>(a);
  coop_step<0x118, 0xf>(a);
  coop_step<0x142, 0xa>(a);
  coop_step<0x143, 0xc>(a);
  EvalOut r;
  r.minabs = readlane_f64(a.minabs, 63);
  r.minv = readlane_f64(a.minv, 63);
  r.maxloc = __builtin_amdgcn_readlane(a.loc, 63);
  r.va = capi > 0 ? readlane_f64(d, capi - 1) : 0.0;
  r.vb = capj > 0 ? readlane_f64(d, capj - 1) : 0.0;
  if (lane_d) *lane_d = d;
  return r;
}

// The far-field certificate of a full EVAL at p0 (far.h): the nearest top is the primitive
// `node`, every other top has a computed |ds| >= m2 at p0, and neg_other says whether one of
// them is negative there. node < 0: no certificate.
struct FarCert {
  int32_t node, top;  // top: its 1-based index
  double m2;
  bool neg_other;
};

// Culled EVAL (cull.h): the always-evaluated tops wave-uniformly, then each lane walks its
// cell's list of tops with per-lane loads; a lane whose bound test fails (or that needs the
// Fresnel/normal captures, or lies outside the culling grid) takes part in one wave-uniform
// full EVAL instead. The merge keeps eval_sdfs' results exactly: min and abs-min are order
// free, and maxloc ties go to the lowest top index as eval_sdfs' index-order strict compare.
// Call in wave-uniform control flow.
#ifdef SMCRT_DIAG
// diagnostic builds: [0] culled lane-EVALs [1] bound-test fallbacks [2] capture/outside
// fallbacks [3] list entries walked [4] wave-EVALs [5] wave-EVALs with a full fallback
static __device__ unsigned long long g_cull_diag[6];
#endif
#ifndef SMCRT_CULL_PREFETCH
#define SMCRT_CULL_PREFETCH 1
#endif
// (ct: the cooperative EVAL's LDS table when the block staged it (at most 64 single-primitive
// tops): a listed top's kind, transform and parameters then come from LDS by its index, not
// from its node in device memory; sdf_prim_s of the same doubles, so the same value bit for bit)
#ifndef SMCRT_CULL_CTAB
#define SMCRT_CULL_CTAB 1
#endif
// a capture EVAL folds only the captured tops (1, round 6) instead of a full EVAL (0)
#ifndef SMCRT_CULL_CAPTURE
#define SMCRT_CULL_CAPTURE 1
#endif
// a lane stops its list walk at the first entry whose box lies farther than the min|ds| it
// holds (1, round 6: the entries are stored nearest box first with that distance, cull.h)
#ifndef SMCRT_CULL_ELB
#define SMCRT_CULL_ELB 1
#endif
#ifndef SMCRT_CULL_UNROLL
#define SMCRT_CULL_UNROLL 4  // spheres (M2: 17.4-18.2 with 4, 17.1-17.4 with 2, 15.1-17.2 with 1, profiles/r06_s6/ab_m2_cull.txt)
#endif
#ifndef SMCRT_CULL_UNROLL_CAP
#define SMCRT_CULL_UNROLL_CAP 2  // capsules (M4: 13.1-13.2 with 2, 12.7 with 4, 12.5 with 1, profiles/r06_s6/ab_m4_cull.txt)
#endif
template <bool NEST = false>
__device__ __forceinline__ EvalOut eval_culled(const smcrt_sdf_node* __restrict__ nodes,
                                               const ProgOp* __restrict__ prog, int32_t n_prog,
                                               const CullGrid* __restrict__ G, V3 q, bool have, bool mask_le,
                                               int32_t capi, int32_t capj, const double* ct = nullptr) {
  EvalOut r;
  r.minabs = __builtin_inf();
  r.minv = __builtin_inf();
  r.va = 0.0; r.vb = 0.0;
  r.maxloc = 0;
  double best = -__builtin_inf();
  {  // the unboundable tops, wave-uniform (scalar-loaded program)
    const ProgOp* __restrict__ pa = (const ProgOp*)G->prog_always;
    const int32_t na = G->n_prog_always;
    double acc = 0.0;
    for (int32_t ip = 0; ip < na; ++ip) {
      const ProgOp op = pa[ip];
      const int32_t node = __builtin_amdgcn_readfirstlane(op.node);
      const double v = prog_value<NEST>(nodes, node, op.action, op.translate_only != 0, q);
      if ((op.action & 3) == PROG_TOP || (op.action & 3) == PROG_CHILD_FIRST) acc = v;
      else acc = csg(op.op, acc, v, op.k);
      if (op.top > 0) {
        const double d = acc;
        const double a = fabs(d);
        if (a < r.minabs) r.minabs = a;
        if (d < r.minv) r.minv = d;
        const bool neg = mask_le ? (d <= 0.0) : (d < 0.0);
        if (neg && (r.maxloc == 0 || d > best)) { best = d; r.maxloc = op.top; }
      }
    }
  }
#if SMCRT_CULL_CAPTURE
  // A capture (the Fresnel ds lookups, calcNormal's taps: capi or capj set) uses only the
  // captured tops' values, ds(capi) and ds(capj) (kernels.h P3, ST_F0..ST_N4), so such a lane
  // folds those tops' own ops, as eval_sdfs folds them, instead of taking the wave to a full
  // EVAL of every top (round 6; min|ds|, min ds and maxloc are left unset: nothing reads them)
  const bool capture = have && (capi != 0 || capj != 0);
  if (capture) {
    auto top_ds = [&](int32_t i) {  // top i (0-based): its ops of the flattened program
      const int32_t o0 = prog[n_prog + i].node, o1 = prog[n_prog + i + 1].node;
      double acc = 0.0;
      for (int32_t ip = o0; ip < o1; ++ip) {
        const ProgOp op = prog[ip];
        const double v = prog_value<NEST>(nodes, op.node, op.action, op.translate_only != 0, q);
        if ((op.action & 3) == PROG_TOP || (op.action & 3) == PROG_CHILD_FIRST) acc = v;
        else acc = csg(op.op, acc, v, op.k);
      }
      return acc;
    };
    if (capi != 0) r.va = top_ds(capi - 1);
    if (capj != 0) r.vb = top_ds(capj - 1);
  }
  bool full = !have;
#else
  const bool capture = false;
  bool full = !have || capi != 0 || capj != 0;
#endif
  const double fx = (q.x - G->lo[0]) * G->inv_cell, fy = (q.y - G->lo[1]) * G->inv_cell,
               fz = (q.z - G->lo[2]) * G->inv_cell;
  if (!capture && !(fx >= 0.0 && fx < (double)G->n[0] && fy >= 0.0 && fy < (double)G->n[1] && fz >= 0.0 &&
                    fz < (double)G->n[2]))
    full = true;
  if (!full && !capture) {
    const int32_t ix = (int32_t)fx, iy = (int32_t)fy, iz = (int32_t)fz;
    const uint32_t c = (uint32_t)ix + (uint32_t)G->n[0] * ((uint32_t)iy + (uint32_t)G->n[1] * (uint32_t)iz);
    const uint32_t b = G->off[c], e = G->off[c + 1];
    const uint2* __restrict__ ent = (const uint2*)G->list;
    uint32_t k0 = b;
#if SMCRT_CULL_UNROLL > 1
    // Groups of listed tops as straight-line code (sdf_prim_s with the kind a constant: the
    // same operations), so their load and square-root latencies overlap: SMCRT_CULL_UNROLL
    // translation-only spheres from the LDS table, or SMCRT_CULL_UNROLL_CAP translation-only
    // capsules (from the table or their nodes); the first other entry ends the groups and the
    // loop below takes the rest. The fold is order free (min, abs-min; maxloc ties go to the
    // lowest index by its explicit compare).
    for (;;) {
      constexpr int U = SMCRT_CULL_UNROLL, UC = SMCRT_CULL_UNROLL_CAP;
      double du[U];
      int32_t iu[U];
      int n = 0;
      // (the rest of the list is farther than the min|ds| this lane holds: cull.h)
      if (SMCRT_CULL_ELB && k0 < e && (double)G->elb[k0] > r.minabs) { k0 = e; break; }
      if (SMCRT_CULL_CTAB && ct && k0 + (U - 1) < e) {
        uint2 eu[U];
        uint32_t all = ~0u;
#pragma unroll
        for (int u = 0; u < U; ++u) { eu[u] = ent[k0 + u]; all &= eu[u].x; }
        if (all & CULL_SPHERE) {
#pragma unroll
          for (int u = 0; u < U; ++u) {
            iu[u] = (int32_t)(eu[u].x & CULL_TOP_MASK);
            du[u] = sdf_prim_s<64>(SMCRT_SDF_SPHERE, ct + iu[u], ct + 12 * 64 + iu[u], q, true);
          }
          n = U;
        }
      }
      if (n == 0 && UC > 1 && k0 + (UC - 1) < e) {
        uint2 eu[UC];
        uint32_t all = ~0u;
#pragma unroll
        for (int u = 0; u < UC; ++u) { eu[u] = ent[k0 + u]; all &= eu[u].x; }
        if (all & CULL_CAPSULE) {
#pragma unroll
          for (int u = 0; u < UC; ++u) {
            iu[u] = (int32_t)(eu[u].x & CULL_TOP_MASK);
            if (SMCRT_CULL_CTAB && ct) {
              du[u] = sdf_prim_s<64>(SMCRT_SDF_CAPSULE, ct + iu[u], ct + 12 * 64 + iu[u], q, true);
            } else {
              const smcrt_sdf_node* nd = nodes + eu[u].y;
              du[u] = sdf_prim_s<1>(SMCRT_SDF_CAPSULE, nd->transform, nd->param, q, true);
            }
          }
          n = UC;
        }
      }
      if (n == 0) break;  // (the loop below takes the rest)
      k0 += (uint32_t)n;
#pragma unroll
      for (int u = 0; u < U; ++u) {
        if (u >= n) break;
        const double d = du[u];
        const int32_t t = iu[u] + 1;
        const double a = fabs(d);
        if (a < r.minabs) r.minabs = a;
        if (d < r.minv) r.minv = d;
        const bool neg = mask_le ? (d <= 0.0) : (d < 0.0);
        if (neg && (r.maxloc == 0 || d > best || (d == best && t < r.maxloc))) { best = d; r.maxloc = t; }
      }
    }
#endif
#if SMCRT_CULL_PREFETCH
    // the next entry's load is issued before this entry's SDF, so the list walk pays one
    // memory latency per entry (the node's) instead of two
    uint2 nxt = k0 < e ? ent[k0] : make_uint2(0u, 0u);
#endif
    for (uint32_t k = k0; k < e; ++k) {  // per lane: its cell's tops, nearest box first
      if (SMCRT_CULL_ELB && (double)G->elb[k] > r.minabs) break;  // (cull.h)
#if SMCRT_CULL_PREFETCH
      const uint2 en = nxt;
      if (k + 1 < e) nxt = ent[k + 1];
#else
      const uint2 en = ent[k];
#endif
      const int32_t i = (int32_t)(en.x & CULL_TOP_MASK);
      double d;
      if (en.x & CULL_MODEL) {  // a model: its ops in the flattened program
        const int32_t o0 = prog[n_prog + i].node, o1 = prog[n_prog + i + 1].node;
        double acc = 0.0;
        for (int32_t ip = o0; ip < o1; ++ip) {
          const ProgOp op = prog[ip];
          const double v = prog_value<NEST>(nodes, op.node, op.action, op.translate_only != 0, q);
          if ((op.action & 3) == PROG_TOP || (op.action & 3) == PROG_CHILD_FIRST) acc = v;
          else acc = csg(op.op, acc, v, op.k);
        }
        d = acc;
      } else if (SMCRT_CULL_CTAB && ct) {
        const double kc = ct[20 * 64 + i];
        d = sdf_prim_s<64>((int32_t)kc & 15, ct + i, ct + 12 * 64 + i, q, kc >= 16.0);
      } else {
        d = sdf_prim(nodes + en.y, q, (en.x & CULL_TRANSLATE) != 0);
      }
      const int32_t t = i + 1;
      const double a = fabs(d);
      if (a < r.minabs) r.minabs = a;
      if (d < r.minv) r.minv = d;
      const bool neg = mask_le ? (d <= 0.0) : (d < 0.0);
      if (neg && (r.maxloc == 0 || d > best || (d == best && t < r.maxloc))) { best = d; r.maxloc = t; }
    }
    // every unlisted top has ds >= max(distance to the cell's boundary, lb[c])
    const double cx = G->lo[0] + (double)ix * G->cell, cy = G->lo[1] + (double)iy * G->cell,
                 cz = G->lo[2] + (double)iz * G->cell;
    double h = dmin(dmin(dmin(q.x - cx, cx + G->cell - q.x), dmin(q.y - cy, cy + G->cell - q.y)),
                    dmin(q.z - cz, cz + G->cell - q.z));
    h = dmax(h, 0.0);
    const double T = dmax(h, G->lb[c]) * (1.0 - 1e-12);
    if (!(r.minabs < T)) full = true;
#ifdef SMCRT_DIAG
    atomicAdd(&g_cull_diag[0], 1ull);
    atomicAdd(&g_cull_diag[3], (unsigned long long)(e - b));
    if (full) atomicAdd(&g_cull_diag[1], 1ull);
#endif
  }
#ifdef SMCRT_DIAG
  else if (have) atomicAdd(&g_cull_diag[2], 1ull);
  if ((threadIdx.x & 63) == 0) {
    atomicAdd(&g_cull_diag[4], 1ull);
  }
  if ((threadIdx.x & 63) == 0 && __ballot(have && full)) atomicAdd(&g_cull_diag[5], 1ull);
#endif
  if (__ballot(have && full)) {
    const EvalOut f = eval_sdfs<NEST>(nodes, prog, n_prog, q, mask_le, capi, capj);
    if (full) r = f;
  }
  return r;
}

// Culled EVAL for ONE wave-uniform query point q with the whole wave cooperating: the
// always-evaluated tops wave-uniformly, then lane j takes entry b + j (+64, ...) of q's cell
// list and the wave reduces with DPP (eval_coop_tab's fold), so a sparse wave pays one or two
// memory latencies per list instead of one per entry and lane. Results equal eval_culled's
// (and so eval_sdfs'): min and abs-min are order free, maxloc ties go to the lowest index.
// Call with all lanes active; q, mask_le, capi and capj must be wave-uniform.
template <bool NEST = false>
__device__ __forceinline__ EvalOut eval_culled_coop(const smcrt_sdf_node* __restrict__ nodes,
                                                    const ProgOp* __restrict__ prog, int32_t n_prog,
                                                    const CullGrid* __restrict__ G, V3 q, bool mask_le,
                                                    int32_t capi, int32_t capj, FarCert* fc = nullptr) {
  const int lane = (int)(threadIdx.x & 63);
  // (certificate only) the always-evaluated tops' smallest and second smallest |ds|, the node
  // and 1-based index of the smallest when it is a lone primitive (-1: a model), how many are
  // negative and whether the smallest is, and whether any value is NaN or infinite (no
  // certificate then)
  double a_min = __builtin_inf(), a_min2 = __builtin_inf();
  int32_t a_node = -1, a_top = 0;
  uint32_t a_nneg = 0;
  bool a_neg1 = false, a_bad = false;
  if (fc) fc->node = -1;
  EvalOut r;
  r.minabs = __builtin_inf();
  r.minv = __builtin_inf();
  r.va = 0.0; r.vb = 0.0;
  r.maxloc = 0;
  double best = -__builtin_inf();
  {  // the unboundable tops, wave-uniform (as eval_culled)
    const ProgOp* __restrict__ pa = (const ProgOp*)G->prog_always;
    const int32_t na = G->n_prog_always;
    double acc = 0.0;
    for (int32_t ip = 0; ip < na; ++ip) {
      const ProgOp op = pa[ip];
      const int32_t node = __builtin_amdgcn_readfirstlane(op.node);
      const double v = prog_value<NEST>(nodes, node, op.action, op.translate_only != 0, q);
      if ((op.action & 3) == PROG_TOP || (op.action & 3) == PROG_CHILD_FIRST) acc = v;
      else acc = csg(op.op, acc, v, op.k);
      if (op.top > 0) {
        const double d = acc;
        const double a = fabs(d);
        if (a < r.minabs) r.minabs = a;
        if (d < r.minv) r.minv = d;
        const bool neg = mask_le ? (d <= 0.0) : (d < 0.0);
        if (neg && (r.maxloc == 0 || d > best)) { best = d; r.maxloc = op.top; }
        if (fc) {
          if (a < a_min) {
            a_min2 = a_min; a_min = a;
            a_node = op.action == PROG_TOP ? node : -1;
            a_top = op.top;
            a_neg1 = d < 0.0;
          } else if (a < a_min2) {
            a_min2 = a;
          }
          a_nneg += d < 0.0 ? 1u : 0u;
          a_bad = a_bad || !(a <= 0x1.fffffffffffffp+1023);
        }
      }
    }
  }
  bool full = capi != 0 || capj != 0;
  const double fx = (q.x - G->lo[0]) * G->inv_cell, fy = (q.y - G->lo[1]) * G->inv_cell,
               fz = (q.z - G->lo[2]) * G->inv_cell;
  if (!(fx >= 0.0 && fx < (double)G->n[0] && fy >= 0.0 && fy < (double)G->n[1] && fz >= 0.0 &&
        fz < (double)G->n[2]))
    full = true;
  if (!full) {
    const int32_t ix = (int32_t)fx, iy = (int32_t)fy, iz = (int32_t)fz;
    const uint32_t c = (uint32_t)ix + (uint32_t)G->n[0] * ((uint32_t)iy + (uint32_t)G->n[1] * (uint32_t)iz);
    const uint32_t b = G->off[c], e = G->off[c + 1];
    const uint2* __restrict__ ent = (const uint2*)G->list;
    CoopAcc a;
    a.minabs = r.minabs; a.minv = r.minv; a.best = best; a.loc = r.maxloc;  // (every lane: the uniform part)
    // (certificate only) this lane's entries: smallest and second smallest |ds|, the node of
    // the smallest (-1: a model or an LDS record), negatives, and NaN or infinite values
    double l1 = __builtin_inf(), l2 = __builtin_inf();
    int32_t n1 = -1, t1 = 0;
    uint32_t nneg = 0;
    bool neg1 = false, lbad = false;
    for (uint32_t k0 = b; k0 < e; k0 += 64) {
      const uint32_t k = k0 + (uint32_t)lane;
      if (k < e) {
        const uint2 en = ent[k];
        const int32_t i = (int32_t)(en.x & CULL_TOP_MASK);
        double d;
        if (en.x & CULL_MODEL) {
          const int32_t o0 = prog[n_prog + i].node, o1 = prog[n_prog + i + 1].node;
          double acc = 0.0;
          for (int32_t ip = o0; ip < o1; ++ip) {
            const ProgOp op = prog[ip];
            const double v = prog_value<NEST>(nodes, op.node, op.action, op.translate_only != 0, q);
            if ((op.action & 3) == PROG_TOP || (op.action & 3) == PROG_CHILD_FIRST) acc = v;
            else acc = csg(op.op, acc, v, op.k);
          }
          d = acc;
        } else {
          d = sdf_prim(nodes + en.y, q, (en.x & CULL_TRANSLATE) != 0);
        }
        CoopAcc o;
        o.minabs = fabs(d);
        o.minv = d;
        const bool neg = mask_le ? (d <= 0.0) : (d < 0.0);
        o.best = neg ? d : -__builtin_inf();
        o.loc = neg ? i + 1 : 0;
        coop_fold(a, o);
        if (fc) {
          const double ad = o.minabs;
          if (ad < l1) {
            l2 = l1; l1 = ad;
            n1 = (en.x & CULL_MODEL) ? -1 : (int32_t)en.y;
            t1 = i + 1;
            neg1 = d < 0.0;
          } else if (ad < l2) {
            l2 = ad;
          }
          nneg += d < 0.0 ? 1u : 0u;
          lbad = lbad || !(ad <= 0x1.fffffffffffffp+1023);
        }
      }
    }
    coop_step<0x111, 0xf>(a);
    coop_step<0x112, 0xf>(a);
    coop_step<0x114, 0xf>(a);
    coop_step<0x118, 0xf>(a);
    coop_step<0x142, 0xa>(a);
    coop_step<0x143, 0xc>(a);
    r.minabs = readlane_f64(a.minabs, 63);
    r.minv = readlane_f64(a.minv, 63);
    r.maxloc = __builtin_amdgcn_readlane(a.loc, 63);
    // every unlisted top has ds >= max(distance to the cell's boundary, lb[c])
    const double cx = G->lo[0] + (double)ix * G->cell, cy = G->lo[1] + (double)iy * G->cell,
                 cz = G->lo[2] + (double)iz * G->cell;
    double h = dmin(dmin(dmin(q.x - cx, cx + G->cell - q.x), dmin(q.y - cy, cy + G->cell - q.y)),
                    dmin(q.z - cz, cz + G->cell - q.z));
    h = dmax(h, 0.0);
    const double T = dmax(h, G->lb[c]) * (1.0 - 1e-12);
    if (!(r.minabs < T)) {
      full = true;
    } else if (fc) {
      // The far-field certificate (far.h): one top attains min|ds|, either a listed primitive
      // (no always-evaluated top does) or an always-evaluated lone primitive (no listed top
      // does, e.g. a bounding box's wall); every other listed or always-evaluated top has
      // |ds| >= m2, and every unlisted one ds >= T > 0, so m2 also takes T.
      const uint64_t km = __ballot(l1 == r.minabs);
      const bool bad = a_bad || __ballot(lbad) != 0;
      if (__popcll(km) == 1 && !bad && !(a_min <= r.minabs)) {
        const int kl = __builtin_ctzll(km);
        const int32_t node = __builtin_amdgcn_readlane(n1, kl);
        double m2 = wave_min_f64(lane == kl ? l2 : l1);
        m2 = dmin(dmin(m2, a_min), T);
        const bool neg = a_nneg > 0 || __ballot(nneg > ((lane == kl && neg1) ? 1u : 0u)) != 0;
        fc->node = node;
        fc->top = __builtin_amdgcn_readlane(t1, kl);
        fc->m2 = m2;
        fc->neg_other = neg;
      } else if (km == 0 && !bad && a_min == r.minabs && a_min2 > a_min && a_node >= 0) {
        const double m2 = dmin(dmin(wave_min_f64(l1), a_min2), T);
        fc->node = __builtin_amdgcn_readfirstlane(a_node);
        fc->top = __builtin_amdgcn_readfirstlane(a_top);
        fc->m2 = m2;
        fc->neg_other = a_nneg > (a_neg1 ? 1u : 0u) || __ballot(nneg > 0) != 0;
      }
    }
  }
  if (full) r = eval_sdfs<NEST>(nodes, prog, n_prog, q, mask_le, capi, capj);
  return r;
}

}  // namespace smcrt
