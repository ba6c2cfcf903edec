// kernels.h — the transport kernels (transport_kernel here, ws_kernel in ws.h) as templates.
//
// Included only by kinst.hip, which build.py compiles once per (LDS faces, grid mode) pair so
// the instantiations build in parallel; smcrt.hip reaches them through the pointers of
// kernel_ptrs.h. Paths and reference citations: smcrt.hip's header and DESIGN.md §4.3.
#pragma once
#include <hip/hip_runtime.h>

#include "../../include/smcrt.h"
#include "scene_internal.h"
#include "transport.h"
#include "deposit.h"

using namespace smcrt;
// ------------------------------------------------------------------ kernel ---------
__device__ __forceinline__ uint32_t wave_sum_u32(uint32_t v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ double wave_sum_f64(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

#ifdef SMCRT_DIAG
// (one copy per kinst.hip object; kinst_diag_* gathers them)
// Diagnostic build only (-DSMCRT_DIAG): lane-state occupancy per scheduler trip.
// [0..31] lane-trips by state at the trip head (+32 if a segment is active), [64] trips,
// [65] trips running the DDA phase, [66] EVAL, [67] P7 events.
static __device__ unsigned long long g_diag[72];
// wave-time (s_memtime ticks) per phase: [1] fetch [2] EVAL [3] P3 [4] P4 [5] DDA [6] P5-P6
// [7] P7 [8] P8 + loop
static __device__ unsigned long long g_diag_t[9];
#endif

#include "lean.h"
#include "ws.h"
#include "far.h"

// The query point of each EVAL state (the exact expressions of the reference).
__device__ __forceinline__ V3 eval_query(const Lane& L) {
  switch (L.st) {
    case ST_H1: case ST_G0: case ST_F1: return L.ssp;
    case ST_N1: return L.pos + mul(v3(1.0, -1.0, -1.0), 1e-6);   // calcNormal taps,
    case ST_N2: return L.pos + mul(v3(-1.0, -1.0, 1.0), 1e-6);   // sdf_base.f90:176-184
    case ST_N3: return L.pos + mul(v3(-1.0, 1.0, -1.0), 1e-6);
    case ST_N4: return L.pos + mul(v3(1.0, 1.0, 1.0), 1e-6);
    default: return L.pos;
  }
}


// a sparse wave of a culled scene evaluates its lanes' query points one at a time with the
// whole wave (eval_culled_coop) when at most this many lanes need an EVAL
#ifndef SMCRT_COOP_CULL_LANES
#define SMCRT_COOP_CULL_LANES 8
#endif
constexpr uint32_t COOP_CULL_LANES = SMCRT_COOP_CULL_LANES;
// the solo march of a wave's last photon (COOP instantiations; -DSMCRT_SOLO=0 turns it off)
#ifndef SMCRT_SOLO
#define SMCRT_SOLO 1
#endif
#ifndef SMCRT_SOLO_LANES
#define SMCRT_SOLO_LANES 4
#endif

constexpr int SOLO_LANES = SMCRT_SOLO_LANES;

// Waves per SIMD the register allocation aims at: 3 (<= 168 VGPRs) for the plain
// instantiations; the cooperative ones (many tops: LDS table, culling, solo march) hold more
// live state and spill at 168, so they get 2 (M4 +12 %, profiles/r02_s3/NOTE_waves.txt).
#ifndef SMCRT_WAVES_PER_EU
#define SMCRT_WAVES_PER_EU 3
#endif
#ifndef SMCRT_WAVES_PER_EU_COOP
#define SMCRT_WAVES_PER_EU_COOP 2
#endif
#ifndef SMCRT_WAVES_PER_EU_XSRC
#define SMCRT_WAVES_PER_EU_XSRC SMCRT_WAVES_PER_EU
#endif
template <bool LDS_FACES, int GM, bool XSRC, bool COOP>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(COOP ? SMCRT_WAVES_PER_EU_COOP : (XSRC ? SMCRT_WAVES_PER_EU_XSRC : SMCRT_WAVES_PER_EU)))) void transport_kernel(KParams K, const smcrt_sdf_node* __restrict__ nodes,
                                                        const ProgOp* __restrict__ prog,
                                                        const smcrt_detector* __restrict__ dets,
                                                        const int64_t* __restrict__ det_off,
                                                        const KCold* __restrict__ C) {
  __shared__ LaneShared shm;
  LaneShared* sh = &shm;
  const double eps = 1e-8;  // inttau2.f90:56
  const bool test_kernel = (K.flags & SMCRT_FLAG_TEST_KERNEL) != 0;
  const bool survival = (K.flags & SMCRT_FLAG_SURVIVAL_BIAS) != 0;
  const int lane_id = threadIdx.x & 63;

  extern __shared__ double sh_dyn[];  // [props | faces] | [startPos if detectors] | wave tile histograms
  const TopProps* props = K.props;
  const double* xf = K.xface;
  const double* yf = K.yface;
  const double* zf = K.zface;
  int hist_off = 0;  // doubles of sh_dyn before the wave histograms
  if constexpr (LDS_FACES) {
    // per-lane (divergent) lookups go to LDS, never to vector memory: a vector load would
    // make the wave wait for all of its outstanding deposit atomics
    const int np = 4 * K.n_top;
    const double* gp = (const double*)K.props;
    for (int i = threadIdx.x; i < np; i += blockDim.x) sh_dyn[i] = gp[i];
    const int nf = (K.nx + 1) + (K.ny + 1) + (K.nz + 2);
    double* sh_faces = sh_dyn + np;
    for (int i = threadIdx.x; i < nf; i += blockDim.x) sh_faces[i] = K.xface[i];  // faces are contiguous
    props = (const TopProps*)sh_dyn;
    xf = sh_faces;
    yf = sh_faces + (K.nx + 1);
    zf = yf + (K.ny + 1);
    hist_off = np + nf;
  }
  double* const startp = sh_dyn + hist_off + threadIdx.x;  // [3][256] when n_dets > 0
  if (K.n_dets) hist_off += 3 * 256;
  // deposit state: the sorted path's per-wave tile histogram (hist_tiles words) or the
  // bucketed path's per-block word per tile (cur | next | fill: 2 * bucket_tiles words)
  const uint32_t wave_words = K.bucket_tiles ? 0u : K.hist_tiles;
  const uint32_t dep_words = K.bucket_tiles ? 2 * K.bucket_tiles : 4 * K.hist_tiles;  // the block's
  uint32_t* const whist = (uint32_t*)(sh_dyn + hist_off) + (threadIdx.x >> 6) * wave_words;
  // the bucketed path's words are shared by the block's waves (deposit.h); sh_dyn is 8-byte
  // aligned, so they are too
  unsigned long long* const bstate = (unsigned long long*)(sh_dyn + hist_off);
  if (K.bucket_tiles) init_buckets(K, C, bstate);
  else
    for (uint32_t i = threadIdx.x; i < 4 * K.hist_tiles; i += blockDim.x) ((uint32_t*)(sh_dyn + hist_off))[i] = 0;
  // the cooperative EVAL's primitive table (COOP instantiations), after the wave words
  double* const ctab = sh_dyn + hist_off + dep_words / 2;
  if constexpr (COOP) {
    if (K.ctab)
      for (int i = threadIdx.x; i < CTAB_DOUBLES; i += blockDim.x) ctab[i] = K.ctab[i];
  }
#pragma unroll
  for (int c = 0; c < LC_N; ++c) sh->ctr[c][threadIdx.x] = 0;
#pragma unroll
  for (int c = 0; c < LU_N; ++c) sh->u[c][threadIdx.x] = 0;
  __syncthreads();

  Lane L;
  L.st = ST_FETCH; L.pend = false; L.seg = false; L.fault = false; L.tflag = false;
  L.pos = L.dir = L.ssp = L.old = v3(0.0, 0.0, 0.0);
  L.weight = 1.0; L.tau = L.taurun = L.d = L.minabs = 0.0;
  L.xcell = L.ycell = L.zcell = L.layer = L.old_layer = L.new_layer = L.Ls = 0;
  L.hop = L.loopc = L.dda_it = 0;
  L.sd = L.slen = 0.0;
  L.rng.init(0);
  const bool binned = K.rec_pool != nullptr;  // (set only when jmean is tallied)
  RecLog W;
  W.chunk = LOG_NONE; W.fill = 0;
  BucketLog WB;
  WB.next = WB.end = 0;
  uint32_t overflow = 0;
  uint32_t w_dep = 0, w_sdf = 0, w_iters = 0;  // wave totals (scalar registers)
  uint64_t chunk_base = 0;  // wave-uniform photon chunk
  uint32_t chunk_left = 0;

#ifdef SMCRT_DIAG
  unsigned long long t_acc[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0};
  unsigned long long t_last = __builtin_amdgcn_s_memtime();
#define DIAG_T(i)                                                   \
  do {                                                              \
    const unsigned long long t_ = __builtin_amdgcn_s_memtime();     \
    t_acc[(i)] += t_ - t_last;                                      \
    t_last = t_;                                                    \
  } while (0)
#elif defined(SMCRT_ASM_MARKERS)  // analysis builds: phase boundaries visible in the ISA
#define DIAG_T(i) asm volatile("; @@PHASE " #i)
#else
#define DIAG_T(i) do {} while (0)
#endif
  for (;; ++w_iters) {
    DIAG_T(8);
    // ---- photon fetch (wave-aggregated work queue) ------------------------------------
    // A wave takes FETCH_CHUNK photon indices per (returning) queue atomic and hands them
    // to its lanes as they free up: a returning atomic waits for all of the wave's
    // outstanding deposits, so it must be rare.
    {
      uint64_t need = __ballot(L.st == ST_FETCH);
      while (need) {
        if (chunk_left == 0) {
          unsigned long long base = 0;
          if (lane_id == 0) base = atomicAdd(C->queue, (unsigned long long)SMCRT_FETCH_CHUNK);
          chunk_base = __shfl(base, 0, 64);
          const uint64_t n_photons = C->n_photons;
          chunk_left = (chunk_base < n_photons)
                           ? (uint32_t)((n_photons - chunk_base) < SMCRT_FETCH_CHUNK ? (n_photons - chunk_base)
                                                                                       : SMCRT_FETCH_CHUNK)
                           : 0u;
          if (chunk_left == 0) {  // queue exhausted
            if (L.st == ST_FETCH) L.st = ST_IDLE;
            break;
          }
        }
        const uint32_t n = __popcll(need);
        const uint32_t take = n < chunk_left ? n : chunk_left;
        const uint64_t rank = __popcll(need & ((1ull << lane_id) - 1ull));
        if (L.st == ST_FETCH && rank < take) {
          uint64_t g = C->first_photon + chunk_base + rank;
          if constexpr (XSRC) {
            const uint64_t po = C->plan.per_origin;
            if (po) {  // batched point sources: origin g / po, photon first + g % po
              const uint64_t o = g / po;
              LU(LU_ORIGIN) = (uint32_t)o;
              g = C->plan.first + (g - o * po);
            }
          }
          L.rng.init(g);
          L.st = ST_EMIT;
        }
        chunk_base += take;
        chunk_left -= take;
        need = __ballot(L.st == ST_FETCH);
      }
      const uint64_t live = __ballot(L.st != ST_IDLE);
      if (live == 0) break;
    }

#ifdef SMCRT_DIAG_STATES  // (diagnostic builds: lane states per trip into g_diag[0..66])
    {
      const uint32_t cls = (L.seg ? 32u : 0u) + (L.st & 31u);
      for (uint32_t c = 0; c < 64; ++c) {  // wave-uniform loop: count lanes per class
        const uint32_t n = __popcll(__ballot(cls == c));
        if (n && lane_id == 0) atomicAdd(&g_diag[c], (unsigned long long)n);
      }
      if (lane_id == 0) {
        atomicAdd(&g_diag[64], 1ull);
        if (__ballot(L.seg)) atomicAdd(&g_diag[65], 1ull);
        if (__ballot(!L.seg && L.pend)) atomicAdd(&g_diag[66], 1ull);
      }
    }
#endif
    DIAG_T(1);
#if SMCRT_SOLO
    // ---- solo march: a wave left with at most SOLO_LANES photons not waiting for an event -
    // In a launch's tail a lone photon pays the whole trip (every phase's checks, one EVAL
    // and at most SMCRT_DDA_PER_ITER crossings) per march step. When that photon stands at
    // the march loop's EVAL (ST_M1, inttau2.f90:177-191), the wave instead runs the march
    // cycle M1 -> M0 -> segment for it in a tight loop: the cooperative EVAL with every lane,
    // the program points of P3 (ST_M1) and P4 (ST_M0) in the owner lane, and the whole
    // segment's crossings at once. The photon's own sequence of operations is exactly the
    // main loop's, so its trajectory, counters and records are unchanged. The loop ends as
    // soon as the photon leaves the cycle (boundary probe ST_B0, a fault, a new event).
    if constexpr (COOP) {  // (the plain instantiations too: 432 B of spills, M5 -30 %, profiles/r06_s6/ab_solo_plain.txt)
      const bool ev_wait = (L.st == ST_INTERACT || L.st == ST_T2 || L.st == ST_EMIT || L.st == ST_DONE);
      const uint64_t act = __ballot(L.st != ST_IDLE && !ev_wait);
      const uint64_t cand = __ballot(L.st == ST_M1 && L.pend && !L.seg);
      // a glancing loop (ST_G0, inttau2.f90:226-237) that has run a while: tried at its 8th
      // iteration and every 64 after (a try whose certificate fails costs one extra EVAL)
      const uint64_t gcand =
          K.fm_err > 0.0 ? __ballot(L.st == ST_G0 && L.pend && L.loopc >= SMCRT_FAR_MIN_LOOP &&
                                    ((L.loopc - SMCRT_FAR_MIN_LOOP) & 63u) == 0)
                         : 0ull;
      // the full EVAL at q (every lane), and with `want` its far-field certificate (far.h): the
      // near top's kind (SPHERE or BOX; -1: none), where its data are, its 1-based index, a
      // lower bound on every other top's |ds| and whether another top is negative
      int fkind = -1;
      NearTop fnt{nullptr, nullptr, 1};
      int32_t ftop = 0;
      double fm2 = 0.0;
      bool fneg = false;
      auto certified_eval = [&](V3 q, bool want) -> EvalOut {
        EvalOut S;
        double dl = 0.0;  // this lane's ds(lane + 1) (LDS-table EVAL)
        fkind = -1;
        if (K.ctab) {
          S = eval_coop_tab(ctab, K.n_top, q, false, 0, 0, &dl);
          if (want) {
            const bool mine = lane_id < K.n_top;
            const double ad = mine ? fabs(dl) : __builtin_inf();
            const uint64_t km = __ballot(mine && ad == S.minabs);
            const uint64_t bad = __ballot(mine && !(ad <= 0x1.fffffffffffffp+1023));  // NaN, inf
            if (km && !bad) {
              const int k = __builtin_ctzll(km);
              const int kind = (int)ctab[20 * 64 + k] & 15;
              if (kind == SMCRT_SDF_SPHERE || kind == SMCRT_SDF_BOX) {
                fm2 = wave_min_f64(lane_id == k ? __builtin_inf() : ad);
                fneg = __ballot(mine && lane_id != k && dl < 0.0) != 0;
                fnt = NearTop{ctab + k, ctab + 12 * 64 + k, 64};
                ftop = k + 1;
                fkind = kind;
              }
            }
          }
        } else if (K.cull) {
          FarCert fc;
          S = eval_culled_coop<XSRC>(nodes, prog, K.n_prog, K.cull, q, false, 0, 0, want ? &fc : nullptr);
          if (want && fc.node >= 0) {
            const int32_t node = __builtin_amdgcn_readfirstlane(fc.node);
            const int kind = nodes[node].kind;
            if (kind == SMCRT_SDF_SPHERE || kind == SMCRT_SDF_BOX) {
              fm2 = fc.m2;
              fneg = fc.neg_other;
              fnt = NearTop{nodes[node].transform, nodes[node].param, 1};
              ftop = fc.top;
              fkind = kind;
            }
          }
        } else {
          S = eval_sdfs<XSRC>(nodes, prog, K.n_prog, q, false, 0, 0);
        }
        return S;
      };
      if (cand && __popcll(act) <= SOLO_LANES) {  // (a few photons: one after the other)
        const int ow = __builtin_ctzll(cand);
        bool run = true;
        while (run) {
          const V3 q = v3(readlane_f64(L.pos.x, ow), readlane_f64(L.pos.y, ow), readlane_f64(L.pos.z, ow));
          // the far-field certificate of this EVAL, for a march that has run a while
          const bool want = K.fm_err > 0.0 && __builtin_amdgcn_readlane((int)L.loopc, ow) >= SMCRT_FAR_MIN_LOOP;
          const EvalOut S = certified_eval(q, want);
          w_sdf += (uint32_t)K.n_top;  // ST_M1's ds array is counted (packet%cnts)
          if (lane_id == ow) {
            L.pend = false;  // P3, ST_M1: :177-191
            L.minabs = S.minabs;
            L.d = S.minabs;
            if (S.minv > 0.0) { L.tflag = true; L.st = ST_B0; }
            else L.st = ST_M0;
            if (L.st == ST_M0) {  // P4, ST_M0: :155-176
              if (!(L.d >= eps)) {
                L.st = ST_B0;
              } else if (++L.loopc > (uint32_t)MAX_MARCH_ITERS) {
                L.fault = true; L.tflag = true; L.st = ST_B0;
              } else {
                const double kap = props[L.layer - 1].kappa;
                const double t = L.d * kap;
                const V3 oldpos = L.pos;
                if (L.taurun + t < L.tau) {
                  L.taurun = L.taurun + t;
                  L.pos = L.pos + smul(L.d, L.dir);
                  L.st = ST_M1; L.pend = true;
                } else {
                  L.d = (L.tau - L.taurun) / kap;
                  L.taurun = L.tau;
                  L.pos = L.pos + smul(L.d, L.dir);
                  L.st = ST_B0;
                }
                start_segment<GM>(K, L, sh, oldpos, L.d);
              }
            }
          }
          // the segment's crossings (the owner's; wave-uniform so records stay wave-compacted)
          while (__builtin_amdgcn_readlane((int)L.seg, ow)) {
            bool dep = false;
            uint32_t vox = 0;
            double val = 0.0;
            if (lane_id == ow) dda_step<GM>(K, L, L.dir, xf, yf, zf, dep, vox, val, L.weight);
            w_dep += __popcll(__ballot(dep));
            if (binned) {
              if (K.bucket_tiles) emit_bucketed(K, C, WB, dep, vox, val, overflow, bstate);
              else emit_deposits(K, C, W, dep, vox, val, overflow, whist);
            } else if (dep) {
              double* const jm = C->jmean;
              if (jm) atomic_add_nr(jm + vox, val);
            }
          }
          run = __builtin_amdgcn_readlane((int)(L.st == ST_M1 && L.pend && !L.seg), ow) != 0;
          if (run && fkind >= 0) {  // the far-field march from the certificate (far.h)
            uint32_t n = 0, nsdf = 0;
            if (lane_id == ow) {
              double acc = 0.0;
              uint32_t vox = 0;
              const double kap = props[L.layer - 1].kappa;
              n = fkind == SMCRT_SDF_BOX
                      ? far_march<GM, SMCRT_SDF_BOX>(K, L, fnt, fm2, fneg, S.minabs, kap, xf, yf, zf, acc, vox, nsdf)
                      : far_march<GM, SMCRT_SDF_SPHERE>(K, L, fnt, fm2, fneg, S.minabs, kap, xf, yf, zf, acc, vox, nsdf);
              if (n) {
                LCTR(LC_UPD) += n;
                double* const jm = C->jmean;
                if (jm) atomic_add_nr(jm + vox, acc);
                if (C->far_steps) atomicAdd(C->far_steps, (unsigned long long)n);
              }
            }
            n = (uint32_t)__builtin_amdgcn_readlane((int)n, ow);
            nsdf = (uint32_t)__builtin_amdgcn_readlane((int)nsdf, ow);
            w_sdf += nsdf * (uint32_t)K.n_top;
            w_dep += n;
            run = __builtin_amdgcn_readlane((int)(L.st == ST_M1 && L.pend && !L.seg), ow) != 0;
          }
        }
      } else if (gcand && __popcll(act) <= SOLO_LANES) {
        // the glancing loop with the near top only (far.h far_glance); this EVAL is not
        // consumed here: the loop's first iteration re-evaluates the near top at the same point
        const int ow = __builtin_ctzll(gcand);
        const V3 q = v3(readlane_f64(L.ssp.x, ow), readlane_f64(L.ssp.y, ow), readlane_f64(L.ssp.z, ow));
        certified_eval(q, true);
        if (fkind >= 0) {
          uint32_t n = 0;
          if (lane_id == ow)
            n = fkind == SMCRT_SDF_BOX ? far_glance<SMCRT_SDF_BOX>(K, L, fnt, ftop, fm2)
                                       : far_glance<SMCRT_SDF_SPHERE>(K, L, fnt, ftop, fm2);
          n = (uint32_t)__builtin_amdgcn_readlane((int)n, ow);
          w_sdf += n * (uint32_t)K.n_top;  // each iteration consumed a (counted) G0 EVAL
          if (n && lane_id == ow && C->far_steps) atomicAdd(C->far_steps, (unsigned long long)n);
        }
      }
    }
#endif
    // ---- EVAL phase: the SDF array at the lane's query point ----------------------------
    const bool have = !L.seg && L.pend;
    EvalOut R;
    R.minabs = R.minv = R.va = R.vb = 0.0; R.maxloc = 0;
    if (__ballot(have)) {  // wave-uniform: the SDF program stays on the scalar path
      const bool fres = (L.st == ST_F0 || L.st == ST_F1);
      const bool tap = (L.st >= ST_N1 && L.st <= ST_N4);
      const int32_t capi = fres ? L.new_layer : (tap ? L.Ls : 0);
      const int32_t capj = fres ? L.old_layer : 0;
      const bool mask_le = test_kernel && L.st == ST_LAYER;
      const uint64_t evm = __ballot(have);
      if (COOP && K.ctab && (uint32_t)__popcll(evm) <= (uint32_t)K.coop_lanes) {  // sparse wave, LDS table
        const V3 q = eval_query(L);
        uint64_t m = evm;
        while (m) {  // (m and l are scalars: the lane's query reaches the wave by readlane)
          const int l = __builtin_ctzll(m);
          m &= m - 1;
          const V3 ql = v3(readlane_f64(q.x, l), readlane_f64(q.y, l), readlane_f64(q.z, l));
          const EvalOut o = eval_coop_tab(ctab, K.n_top, ql, __builtin_amdgcn_readlane((int)mask_le, l) != 0,
                                          __builtin_amdgcn_readlane(capi, l), __builtin_amdgcn_readlane(capj, l));
          if (lane_id == l) R = o;
        }
      } else if (COOP && !K.cull && (uint32_t)__popcll(evm) <= (uint32_t)K.coop_lanes) {  // sparse, one lane at a time
        const V3 q = eval_query(L);
        uint64_t m = evm;
        while (m) {
          const int l = __builtin_ctzll(m);
          m &= m - 1;
          const V3 ql = v3(__shfl(q.x, l, 64), __shfl(q.y, l, 64), __shfl(q.z, l, 64));
          const EvalOut o = eval_sdfs_coop<XSRC>(nodes, prog, K.n_prog, K.n_top, ql, __shfl((int)mask_le, l, 64) != 0,
                                           __shfl(capi, l, 64), __shfl(capj, l, 64));
          if (lane_id == l) R = o;
        }
      } else if (COOP && K.cull && (uint32_t)__popcll(evm) <= COOP_CULL_LANES) {  // sparse wave, culled
        const V3 q = eval_query(L);
        uint64_t m = evm;
        while (m) {
          const int l = __builtin_ctzll(m);
          m &= m - 1;
          const V3 ql = v3(readlane_f64(q.x, l), readlane_f64(q.y, l), readlane_f64(q.z, l));
          const EvalOut o = eval_culled_coop<XSRC>(nodes, prog, K.n_prog, K.cull, ql,
                                             __builtin_amdgcn_readlane((int)mask_le, l) != 0,
                                             __builtin_amdgcn_readlane(capi, l), __builtin_amdgcn_readlane(capj, l));
          if (lane_id == l) R = o;
        }
      } else if (COOP && K.cull) {  // many tops: exact culling (cull.h)
        R = eval_culled<XSRC>(nodes, prog, K.n_prog, K.cull, eval_query(L), have, mask_le, capi, capj,
                              K.ctab ? ctab : nullptr);
      } else {
        R = eval_sdfs<XSRC, true>(nodes, prog, K.n_prog, eval_query(L), mask_le, capi, capj);
      }
      // packet%cnts counts the evaluations of tauint2's ds/dsNew arrays only (inttau2.f90:67,83,
      // 138,183,219,232): not the initial layer search, the Fresnel ds lookups or calcNormal.
      const bool counted = L.st == ST_H0 || L.st == ST_H1 || L.st == ST_H3 || L.st == ST_M1 || L.st == ST_G0;
      w_sdf += __popcll(__ballot(have && counted)) * (uint32_t)K.n_top;
      if (have) L.pend = false;
    }

    DIAG_T(2);
    // ---- P3: consume the EVAL result ----------------------------------------------------
    if (have) {
      switch (L.st) {
        case ST_LAYER:  // kernelsMod.f90:1948-1952 (test_kernel: mask ds<=0, :2136)
          L.layer = R.maxloc;
          if (L.layer == 0) { L.fault = true; L.st = ST_DONE; }
          else L.st = ST_T2;
          break;
        case ST_H0:  // inttau2.f90:63-84, 149-152
          L.minabs = R.minabs;
          L.d = R.minabs;
          L.loopc = 0;  // march guard
          if (L.d < eps) {  // on a surface: micro-step
            L.d = R.minabs + 2.0 * eps;
            L.ssp = L.pos + smul(L.d, L.dir);
            L.st = ST_H1; L.pend = true;
          } else {
            L.st = (L.taurun >= L.tau || L.tflag) ? ST_T2END : ST_M0;
          }
          break;
        case ST_H1: {  // forward / backward micro-step, :86-123
          const double kap = props[L.layer - 1].kappa;
          const V3 oldpos = L.pos;
          const double t = L.d * kap;
          if (R.maxloc == L.layer) {
            if (L.taurun + t < L.tau) { L.pos = L.pos + smul(L.d, L.dir); L.taurun = L.taurun + t; }
            else { L.d = (L.tau - L.taurun) / kap; L.taurun = L.taurun + t; }
          } else {
            if (L.taurun + t < L.tau) { L.pos = L.pos - smul(L.d, L.dir); L.taurun = L.taurun + t; }
            else { L.d = (L.tau - L.taurun) / kap; L.pos = L.pos - smul(L.d, L.dir); }
          }
          L.st = ST_H2;
          start_segment<GM>(K, L, sh, oldpos, L.d);
          break;
        }
        case ST_H3:  // :133-152
          L.minabs = R.minabs;
          L.d = R.minabs;
          if (R.minv > 0.0) L.tflag = true;
          L.st = (L.taurun >= L.tau || L.tflag) ? ST_T2END : ST_M0;
          break;
        case ST_M1:  // :177-191
          L.minabs = R.minabs;
          L.d = R.minabs;
          if (R.minv > 0.0) { L.tflag = true; L.st = ST_B0; }
          else L.st = ST_M0;
          break;
        case ST_G0: {  // new layer and the glancing loop, :220-245
          L.new_layer = R.maxloc;
          if (L.new_layer == L.old_layer && R.minabs < eps) {
            if (++L.loopc > (uint32_t)MAX_GLANCE_ITERS) { L.fault = true; L.tflag = true; L.st = ST_T2END; break; }
            L.d = L.d + eps;
            L.ssp = L.pos + smul(L.d, L.dir);
            L.pend = true;  // evaluate G0 again
            break;
          }
          if (L.new_layer == 0) { L.tflag = true; L.st = ST_T2END; break; }
          const double n1 = props[L.layer - 1].n, n2 = props[L.new_layer - 1].n;
          if (n1 != n2) { L.st = ST_F0; L.pend = true; break; }
          L.layer = L.new_layer;  // equal n: cross, :318-328
          L.st = ST_X1;
          start_segment<GM>(K, L, sh, L.pos, L.d);
          break;
        }
        case ST_F0:  // ds(new), ds(old) at pos (kept in sd/slen: no segment is active)
          L.sd = R.va; L.slen = R.vb;
          L.st = ST_F1; L.pend = true;
          break;
        case ST_F1: {  // which SDF's normal, :250-277
          const double ds_new = L.sd, ds_old = L.slen, dn_new = R.va, dn_old = R.vb;
          if (dn_new < 0.0 && ds_new >= 0.0) L.Ls = L.new_layer;
          else if (dn_old >= 0.0 && ds_old < 0.0) L.Ls = L.old_layer;
          else if (dn_new < 0.0 && dn_old < 0.0) L.Ls = L.new_layer;
          else if (ds_old >= 0.0 && dn_old >= 0.0) L.Ls = L.old_layer;
          else { L.fault = true; L.tflag = true; L.st = ST_T2END; break; }  // error stop :264-277
          L.st = ST_N1; L.pend = true;
          break;
        }
        case ST_N1: L.old.x = R.va; L.st = ST_N2; L.pend = true; break;  // calcNormal taps in old.xyz
        case ST_N2: L.old.y = R.va; L.st = ST_N3; L.pend = true; break;
        case ST_N3: L.old.z = R.va; L.st = ST_N4; L.pend = true; break;
        case ST_N4: {  // calcNormal (sdf_base.f90:166-190) + reflect_refract (surfaces.f90:14-84)
          const double e4 = R.va;
          const V3 xyy = v3(1.0, -1.0, -1.0), yyx = v3(-1.0, -1.0, 1.0), yxy = v3(-1.0, 1.0, -1.0),
                   xxx = v3(1.0, 1.0, 1.0);
          const V3 nn = ((mul(xyy, L.old.x) + mul(yyx, L.old.y)) + mul(yxy, L.old.z)) + mul(xxx, e4);
          const double ln = len(nn);
          const V3 N = v3(nn.x / ln, nn.y / ln, nn.z / ln);
          const double n1 = props[L.layer - 1].n, n2 = props[L.new_layer - 1].n;
          LCTR(LC_FRES)++;
          const double Rf = fresnel(L.dir, N, n1, n2);
          if (L.rng.next(K.key0, K.key1) <= Rf) {  // reflect :42-55, :304-316
            const double s2 = 2.0 * dot(N, L.dir);
            L.dir = L.dir - smul(s2, N);
            LCTR(LC_REFL)++;
            if (K.n_dets) { startp[0] = L.pos.x; startp[256] = L.pos.y; startp[512] = L.pos.z; }
            if (++LU(LU_BOUNCES) > 1000) {  // :313-315: return without write-back
              LCTR(LC_BABORT)++;
              L.pos = v3(sh->entry[0][threadIdx.x], sh->entry[1][threadIdx.x], sh->entry[2][threadIdx.x]);
              L.dir = v3(sh->entry[3][threadIdx.x], sh->entry[4][threadIdx.x], sh->entry[5][threadIdx.x]);
              L.st = ST_INTERACT;
            } else {
              L.st = ST_H0;  // arrives in P8
            }
          } else {  // refract :57-84, transmit :284-303
            const double eta = n1 / n2;
            V3 Nt = N;
            double c1 = dot(Nt, L.dir);
            if (c1 < 0.0) c1 = -c1;
            else Nt = smul(-1.0, N);
            const double c2 = sqrt(1.0 - (eta * eta) * (1.0 - c1 * c1));
            L.dir = smul(eta, L.dir) + smul(eta * c1 - c2, Nt);
            L.layer = L.new_layer;
            L.st = ST_X1;
            start_segment<GM>(K, L, sh, L.pos, L.d);
          }
          break;
        }
        default:
          break;
      }
    }

    DIAG_T(3);
    // ---- P4: a march step starts its deposit segment, :155-176 -------------------------
    if (!L.seg && L.st == ST_M0) {
      if (!(L.d >= eps)) {
        L.st = ST_B0;
      } else if (++L.loopc > (uint32_t)MAX_MARCH_ITERS) {
        L.fault = true; L.tflag = true; L.st = ST_B0;
      } else {
        const double kap = props[L.layer - 1].kappa;
        const double t = L.d * kap;
        const V3 oldpos = L.pos;
        if (L.taurun + t < L.tau) {
          L.taurun = L.taurun + t;
          L.pos = L.pos + smul(L.d, L.dir);
          L.st = ST_M1; L.pend = true;
        } else {
          L.d = (L.tau - L.taurun) / kap;
          L.taurun = L.tau;
          L.pos = L.pos + smul(L.d, L.dir);
          L.st = ST_B0;
        }
        start_segment<GM>(K, L, sh, oldpos, L.d);
      }
    }

    DIAG_T(4);
    // ---- DDA phase: voxel crossings of pending deposit segments ------------------------
    // Placed after the program points that start segments (P3, P4) and before the ones that
    // consume them (P5), so a short segment is started, walked and finished in one trip.
    if (__ballot(L.seg)) {  // wave-uniform, so deposit records can be wave-compacted
#pragma unroll
      for (int k = 0; k < SMCRT_DDA_PER_ITER; ++k) {
        bool dep = false;
        uint32_t vox = 0;
        double val = 0.0;
        if (L.seg) dda_step<GM>(K, L, L.dir, xf, yf, zf, dep, vox, val, L.weight);
        w_dep += __popcll(__ballot(dep));
        if (binned) {
          if (K.bucket_tiles) emit_bucketed(K, C, WB, dep, vox, val, overflow, bstate);
          else emit_deposits(K, C, W, dep, vox, val, overflow, whist);
        }
        else if (dep) {
          double* const jm = C->jmean;
          if (jm) atomic_add_nr(jm + vox, val);
        }
      }
    }

    DIAG_T(5);
    // ---- P5: after a deposit segment: detectors and the next program point -------------
    bool rec = false;
    V3 rec_start = v3(0.0, 0.0, 0.0);
    double rec_sep = 0.0;
    if (!L.seg && (L.st == ST_H2 || L.st == ST_B0 || L.st == ST_X1)) {
      if (L.st == ST_X1) {  // :294-303 / :326-335
        L.taurun = L.taurun + L.d * props[L.layer - 1].kappa;
        L.pos = L.ssp;
      }
      rec = true;  // :125-131, 195-201
      if (K.n_dets) {
        rec_start = v3(startp[0], startp[256], startp[512]);
        rec_sep = pointsep(L.pos, rec_start);
        startp[0] = L.pos.x; startp[256] = L.pos.y; startp[512] = L.pos.z;
      }
      if (L.st == ST_H2) {
        L.st = ST_H3; L.pend = true;
      } else if (L.st == ST_X1) {
        L.st = L.tflag ? ST_T2END : ST_H0;
      } else if (L.taurun >= L.tau || L.tflag) {  // B0, :204-207
        L.st = ST_T2END;
      } else {  // boundary probe, :213-222
        L.d = L.minabs + 2.0 * eps;
        L.ssp = L.pos + smul(L.d, L.dir);
        L.old_layer = L.layer;
        L.loopc = 0;  // glancing guard
        L.st = ST_G0; L.pend = true;
      }
    }
    if (K.n_dets && rec) {
      double* tot = nullptr;
      if constexpr (XSRC) {
        if (C->plan.det_totals) tot = C->plan.det_totals + (uint64_t)LU(LU_ORIGIN) * (uint64_t)K.n_dets;
      }
      LCTR(LC_HITS) += record_hits(K, C->det_bins, dets, det_off, rec_start, L.dir, rec_sep, L.layer, L.weight, tot);
    }

    // ---- P6: tauint2 write-back checks, :341-362 -----------------------------------------
    if (!L.seg && L.st == ST_T2END) {
      if (fabs(L.pos.x) > K.xmax) L.tflag = true;
      if (fabs(L.pos.y) > K.ymax) L.tflag = true;
      if (fabs(L.pos.z) > K.zmax) L.tflag = true;
      L.st = ST_INTERACT;
    }

    DIAG_T(6);
    // ---- P7: photon events (interaction, tauint2 entry, emission, completion) ----------
    // These are the expensive, rare program points; a wave runs them together once enough
    // lanes wait for one (or nothing else is left), instead of paying for them every trip.
    {
      const bool ev = (L.st == ST_INTERACT || L.st == ST_T2 || L.st == ST_EMIT || L.st == ST_DONE);
      const uint64_t evm = __ballot(ev);
      const uint64_t busy = __ballot(L.st != ST_IDLE && L.st != ST_FETCH);
      const uint32_t nev = __popcll(evm);
      if (nev && (nev >= SMCRT_EVENT_LANES || evm == busy)) {
#ifdef SMCRT_DIAG
        if (lane_id == 0) atomicAdd(&g_diag[67], 1ull);
#endif
        if (L.st == ST_INTERACT) {  // kernelsMod.f90:1958-1975 / 2036-2065 / 2126-2170
          if (L.tflag || L.fault) {
            L.st = ST_DONE;
          } else if (++LU(LU_INTER) > (uint32_t)MAX_INTERACTIONS) {
            L.fault = true; L.st = ST_DONE;
          } else {
            const double ran = L.rng.next(K.key0, K.key1);
            const TopProps pr = props[L.layer - 1];
            bool sc = false;
            if (survival) {
              const double w_abs = L.weight * (1.0 - pr.albedo);
              L.weight = L.weight - w_abs;
              add_cell(K, C->absorb, L, w_abs);
              sc = true;
              if (L.weight < 0.01) {
                if (ran < 0.1) L.weight = L.weight / 0.1;
                else { L.tflag = true; LU(LU_STATUS) = 1; LCTR(LC_ABSORBED)++; sc = false; }
              }
            } else if (ran < pr.albedo) {
              sc = true;
            } else {
              L.tflag = true; LU(LU_STATUS) = 1; LCTR(LC_ABSORBED)++;
              if (!test_kernel) add_cell(K, C->absorb, L, 1.0);  // recordWeight(packet, 1.0)
            }
            if (sc) {
              scatter(K, L, pr.hgg);
              const uint32_t st = ++LU(LU_NSCATT);
              LCTR(LC_SCATTERS)++;
              if (test_kernel && !survival) {
                if (st >= 1 && st <= 4) {
                  double* const moments = C->moments;
                  if (moments) {
                    double* m = moments + 3 * (st - 1);
                    double* m2 = moments + 12 + 3 * (st - 1);
                    atomic_add_nr(m + 0, L.pos.x); atomic_add_nr(m + 1, L.pos.y); atomic_add_nr(m + 2, L.pos.z);
                    atomic_add_nr(m2 + 0, L.pos.x * L.pos.x);
                    atomic_add_nr(m2 + 1, L.pos.y * L.pos.y);
                    atomic_add_nr(m2 + 2, L.pos.z * L.pos.z);
                  }
                } else if (K.flags & SMCRT_FLAG_END_EARLY) {
                  L.tflag = true;
                  LU(LU_STATUS) = 4;
                }
              }
              L.st = ST_T2;
            } else {
              L.st = ST_DONE;
            }
          }
        }
        if (L.st == ST_T2) {  // tauint2 entry, inttau2.f90:48-60
          if (K.n_dets) { startp[0] = L.pos.x; startp[256] = L.pos.y; startp[512] = L.pos.z; }
          sh->entry[0][threadIdx.x] = L.pos.x; sh->entry[1][threadIdx.x] = L.pos.y;
          sh->entry[2][threadIdx.x] = L.pos.z; sh->entry[3][threadIdx.x] = L.dir.x;
          sh->entry[4][threadIdx.x] = L.dir.y; sh->entry[5][threadIdx.x] = L.dir.z;
          LCTR(LC_TAU)++;
          L.tau = -det_log(L.rng.next(K.key0, K.key1));
          L.taurun = 0.0;
          L.hop = 0;
          L.st = ST_H0;  // arrives in P8
        }
        if (L.st == ST_EMIT) {  // kernelsMod.f90:1937-1945
          L.fault = false; L.layer = 0;
          LU(LU_STATUS) = 0; LU(LU_NSCATT) = 0; LU(LU_INTER) = 0; LU(LU_BOUNCES) = 0;
          L.xcell = L.ycell = L.zcell = 0;
          emit<GM, XSRC>(K, C, L, XSRC ? LU(LU_ORIGIN) : 0u);
          if (!test_kernel) {
            int64_t tries = 0;
            while (cell_out(K, L)) {
              if (++tries > MAX_EMIT_TRIES) { L.fault = true; break; }
              LCTR(LC_RETRIES)++;
              emit<GM, XSRC>(K, C, L, XSRC ? LU(LU_ORIGIN) : 0u);
            }
            if (!L.fault && (K.flags & SMCRT_FLAG_RENDER_SOURCE)) add_cell(K, C->emission, L, 1.0);
          }
          if (L.fault) L.st = ST_DONE;
          else { L.st = ST_LAYER; L.pend = true; }
        }
        if (L.st == ST_DONE) {  // photon finished
          if (L.fault) { LU(LU_STATUS) = 3; LCTR(LC_FAULTS)++; }
          else if (LU(LU_STATUS) == 0) { LU(LU_STATUS) = 2; LCTR(LC_ESCAPED)++; }
          LCTR(LC_PHOTONS)++;
          LCTR(LC_DRAWS) += L.rng.draws;
#ifdef SMCRT_DIAG
          if (C->done_time)
            C->done_time[(((uint64_t)L.rng.pid_hi << 32) | L.rng.pid_lo) - C->done_base] = __builtin_amdgcn_s_memrealtime();
#endif
          smcrt_photon_record* const records = C->records;
          if ((K.flags & SMCRT_FLAG_RECORD_PHOTONS) && records) {
            const uint64_t pid = ((uint64_t)L.rng.pid_hi << 32) | L.rng.pid_lo;
            smcrt_photon_record* r = records + (pid - C->first_photon);
            r->pos[0] = L.pos.x; r->pos[1] = L.pos.y; r->pos[2] = L.pos.z;
            r->dir[0] = L.dir.x; r->dir[1] = L.dir.y; r->dir[2] = L.dir.z;
            r->weight = L.weight;
            r->cell[0] = L.xcell; r->cell[1] = L.ycell; r->cell[2] = L.zcell;
            r->layer = L.layer;
            r->nscatt = LU(LU_NSCATT);
            r->bounces = LU(LU_BOUNCES);
            r->draws = L.rng.draws;
            r->status = LU(LU_STATUS);
          }
          L.tflag = false; L.fault = false;
          L.st = ST_FETCH;
        }
      }
    }

    DIAG_T(7);
    // ---- P8: arrive at the hop-loop head, :61 ---------------------------------------------
    if (!L.seg && L.st == ST_H0 && !L.pend) {
      if (!(L.taurun <= L.tau)) L.st = ST_T2END;
      else if (++L.hop > (uint32_t)MAX_HOP_ITERS) { L.fault = true; L.tflag = true; L.st = ST_T2END; }
      else L.pend = true;
    }
  }

  if (binned) {
    if (K.bucket_tiles) {
      close_buckets(K, C, WB, w_dep - overflow, overflow);
      __syncthreads();  // every wave of the block is done depositing
      close_block_buckets(K, C, bstate);
    } else {
      close_log(K, C, W, overflow, whist);
    }
  }

#ifdef SMCRT_DIAG
  if (lane_id == 0) {
    for (int i = 0; i < 9; ++i) atomicAdd(&g_diag_t[i], t_acc[i]);
    unsigned long long tw = 0;
    for (int i = 0; i < 9; ++i) tw += t_acc[i];
    atomicMax(&g_diag[68], (unsigned long long)w_iters);  // the longest wave: iterations, ticks
    atomicMax(&g_diag[69], tw);
    atomicAdd(&g_diag[70], 1ull);  // waves
  }
#endif
  // ---- per-wave counter reduction ------------------------------------------------------
  if (binned && K.bucket_tiles) {  // segments of this launch (the host's lean-kernel choice)
    const uint32_t u = wave_sum_u32(LCTR(LC_UPD));
    if (lane_id == 0 && u) atomicAdd(C->dep_ctl + 6, u);
  }
  unsigned long long* const counters = C->counters;
  if (counters) {
    uint32_t c[SMCRT_NCOUNTERS];
    c[SMCRT_CTR_PHOTONS] = LCTR(LC_PHOTONS);
    c[SMCRT_CTR_EMIT_RETRIES] = LCTR(LC_RETRIES);
    c[SMCRT_CTR_SCATTERS] = LCTR(LC_SCATTERS);
    c[SMCRT_CTR_ABSORBED] = LCTR(LC_ABSORBED);
    c[SMCRT_CTR_SDF_EVALS] = lane_id == 0 ? w_sdf : 0u;
    c[SMCRT_CTR_DEPOSITS] = lane_id == 0 ? w_dep : 0u;
    c[SMCRT_CTR_GRID_UPDATES] = LCTR(LC_UPD);
    c[SMCRT_CTR_TAUINT] = LCTR(LC_TAU);
    c[SMCRT_CTR_FRESNEL] = LCTR(LC_FRES);
    c[SMCRT_CTR_REFLECTIONS] = LCTR(LC_REFL);
    c[SMCRT_CTR_BOUNCE_ABORTS] = LCTR(LC_BABORT);
    c[SMCRT_CTR_FAULTS] = LCTR(LC_FAULTS);
    c[SMCRT_CTR_RNG_DRAWS] = LCTR(LC_DRAWS);
    c[SMCRT_CTR_DETECTOR_HITS] = LCTR(LC_HITS);
    c[SMCRT_CTR_ESCAPED] = LCTR(LC_ESCAPED);
    c[SMCRT_CTR_WAVE_ITERS] = lane_id == 0 ? w_iters : 0u;
#pragma unroll
    for (int i = 0; i < SMCRT_NCOUNTERS; ++i) {
      const uint32_t s = wave_sum_u32(c[i]);
      if (lane_id == 0 && s) atomicAdd(counters + i, (unsigned long long)s);
    }
  }
  double* const nscatt = C->nscatt;
  if (nscatt) {  // nscatt = number of scatters (kernelsMod.f90:1966)
    const uint32_t s = wave_sum_u32(LCTR(LC_SCATTERS));
    if (lane_id == 0 && s) atomic_add_nr(nscatt, (double)s);
  }
}
