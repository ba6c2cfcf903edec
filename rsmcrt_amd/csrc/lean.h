// lean.h — the transport kernel of simple scenes, with the voxel walk decoupled from the photon.
//
// Same path as transport_kernel (noBiasPropagation kernelsMod.f90:1901-1976 -> tauint2
// inttau2.f90:15-364 -> update_grids :367-465), same arithmetic, same results bit for bit,
// for the scenes the north-star workload is made of: every top-level SDF has the same
// refractive index (no Fresnel events: reflect_refract is never reached, :248), no detectors,
// no survival bias, path-length deposition into buckets (deposit.h), the three plain sources.
//
// Why a second kernel. In transport_kernel a photon that starts a deposit segment
// (update_grids) walks it before it may take its next step, and every lane of a wave walks its
// own segment: a lane with a one-crossing segment idles while its neighbour walks five, and a
// march step whose segment is longer than one trip's crossings costs another trip (M1: 57
// segments of 3.5 crossings per photon; the walk was 65 % of the wave's time with 42.5 of 64
// lanes busy). Here the photon does not wait for the walk:
//   * a segment is a pure function of (start, direction, length, start cell): update_grids
//     reads pos, dir and d_sdf and writes only jmean and the packet's cells (:401-445);
//   * the only results the photon consumes are tflag (the walk left the grid, :437-440), the
//     error stops (:510-516, :570-573) and the final cells (read by recordWeight at an
//     absorption, kernelsMod.f90:2202-2220, and by the photon record).
// So the photon hands the segment to its wave's ring of segments (LDS) and goes on. The
// wave's lanes then walk segments from the ring, any lane any segment, refilled after every
// crossing, so the walk runs on nearly full waves and a march step costs one trip.
//   * A segment that provably stays inside the grid (both ends at least lean_margin from every
//     grid face, see below) cannot set tflag, so the photon continues at once ("deferred").
//   * Any other segment is "synchronous": the photon waits for it exactly as before and takes
//     its tflag, error flags and cells when a walker finishes it.
//   * The final cells of a deferred segment land in the photon's slot (pcell); a photon that
//     must record an absorption (or its record) waits until its segments are done and reads
//     them. Its RNG draw is taken back first, so the draw sequence is unchanged.
//
// Why a deferred segment cannot leave the grid: dda_step moves each coordinate either by
// dir_a * dcell (exact up to rounding) or, on the crossing axis, to face +- delta (1e-8,
// inttau2.f90:393). A snap puts the walk delta ahead of the straight line along that axis, so
// after k snaps on axis a the walk is at most k * delta (+ rounding) beyond the line at the
// same path length, and k <= n_a (the walk is monotonic along each axis). The line between
// the segment's ends stays inside the box shrunk by lean_margin (convexity), so with
// lean_margin_a = 2 * delta * (n_a + 2) no snap can reach a boundary face. The remaining
// error stops need NaNs or an overshoot of one ulp at an exact tie of two wall distances
// (probability ~1e-16 per crossing); a deferred segment that nevertheless ends in one (a
// "hazard": its photon has gone on as if the walk had stayed inside) is counted in
// SMCRT_CTR_FAULTS and in smcrt_kernel_times.lean_hazards, never silently dropped. The debug
// knob SMCRT_DEBUG_LEAN_MARGIN=0/all provokes hazards to test that accounting.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "transport.h"
#include "deposit.h"

// (diagnostic builds: g_diag, g_diag_t are defined in kernels.h before this header)

namespace smcrt {

#ifndef SMCRT_WAVES_PER_EU_LEAN
#define SMCRT_WAVES_PER_EU_LEAN 3
#endif
// crossing steps per trip of the walk phase (each refills idle walkers from the ring first)
#ifndef SMCRT_LEAN_STEPS
#define SMCRT_LEAN_STEPS 3
#endif
// crossing steps past SMCRT_LEAN_STEPS while at least SMCRT_LEAN_BUSY walkers are busy
#ifndef SMCRT_LEAN_EXTRA
#define SMCRT_LEAN_EXTRA 0
#endif
#ifndef SMCRT_LEAN_BUSY
#define SMCRT_LEAN_BUSY 48
#endif
// after the first crossing step of a walk phase, idle walkers refill only once this many are
// idle (1: every step)
#ifndef SMCRT_LEAN_REFILL_IDLE
#define SMCRT_LEAN_REFILL_IDLE 1
#endif
// walkers keep their segment's direction reciprocals (formed at the refill) instead of
// forming them at every crossing
#ifndef SMCRT_LEAN_RCP
#define SMCRT_LEAN_RCP 0
#endif
// photon events run once this many lanes wait for one (or nothing else is left). The lean
// kernel's other phases keep the waiting lanes' walkers busy, so it batches more than
// transport_kernel's SMCRT_EVENT_LANES = 16: 20 measured +3.5 % on M1 (same box, two rounds,
// profiles/r03_s3/lean_tune_ab.txt)
#ifndef SMCRT_LEAN_EVENT_LANES
#define SMCRT_LEAN_EVENT_LANES 20
#endif
constexpr uint32_t ST_ABSORB = 40;  // absorbed; recordWeight waits for the photon's cells
// The block's event pool (see "Event pool" below; off by default): interactions of every wave
// of the block are queued in LDS and run by whichever wave has SMCRT_LEAN_POOL_MIN of them (or
// nothing else to do), so the event code runs on fuller waves than one wave's own events fill.
// Measured on M1 (same box, round 4, profiles/r04_s2/ab_pool.txt): 196-204 M photons/s
// against 207-213 M without it (bit-exact either way): the pooled events' extra LDS traffic,
// the two segment slots its LDS forces and the separate runs of the remaining local events
// cost more than the fuller event waves save.
#ifndef SMCRT_LEAN_POOL
#define SMCRT_LEAN_POOL 0
#endif
#ifndef SMCRT_LEAN_POOL_MIN
#define SMCRT_LEAN_POOL_MIN 48
#endif
// With the pool, the events a wave still runs itself (completion, emission, the tauint2 entry
// after an emission, interactions that end the photon) are one or two per photon, and a
// finished photon's lane takes no new photon until they have run: run them once this many
// wait (the interactions' batch size, SMCRT_LEAN_EVENT_LANES, would leave lanes empty;
// 4 measured best of 1 and 4).
#ifndef SMCRT_LEAN_LOCAL_EVENT_LANES
#define SMCRT_LEAN_LOCAL_EVENT_LANES 4
#endif
#ifndef SMCRT_LEAN_SLOTS
#if SMCRT_LEAN_POOL
#define SMCRT_LEAN_SLOTS 2  // (the pool's LDS: two slots keep three blocks per CU)
#else
#define SMCRT_LEAN_SLOTS 3
#endif
#endif
constexpr uint32_t LEAN_SLOTS = SMCRT_LEAN_SLOTS;  // segments a photon may have in flight (<= 4)
// Ring entries per wave. Idle walkers refill from the ring at the end of every walk phase, so
// when segments are handed out, either the ring is empty or all 64 walkers hold one: the ring
// then holds at most 64 * LEAN_SLOTS - 64 segments (every slot of every lane, minus those the
// walkers hold), and never more than 64 right after an empty ring.
constexpr uint32_t LEAN_RING = 64 * (LEAN_SLOTS - 1);
static_assert(LEAN_SLOTS >= 2 && LEAN_SLOTS <= 4 && (LEAN_RING & (LEAN_RING - 1)) == 0,
              "the ring index wraps with a mask");
constexpr int LEAN_CELL_BITS = 20;               // per axis in a packed cell word (cell + 1)
constexpr uint64_t LEAN_CELL_MASK = (1ull << LEAN_CELL_BITS) - 1;
constexpr uint64_t LEAN_TFLAG = 1ull << 60, LEAN_FAULT = 1ull << 61;

// Per-block LDS of the lean kernel: the four waves' segment rings (SoA, so consecutive tickets
// hit consecutive banks), the photons' end-cell slots and busy bits, per-photon fields, and
// per-wave counters.
struct LeanShared {
  double ox[4][LEAN_RING], oy[4][LEAN_RING], oz[4][LEAN_RING];  // start, corner coordinates
  double dx[4][LEAN_RING], dy[4][LEAN_RING], dz[4][LEAN_RING];  // direction
  double sl[4][LEAN_RING];                                      // length
  unsigned long long cw[4][LEAN_RING];                          // start cells (packed)
  uint32_t meta[4][LEAN_RING];  // owner lane | slot << 6 | synchronous << 8
  unsigned long long pcell[256][LEAN_SLOTS];  // a finished segment: cells | tflag | fault
  uint32_t busy[256];                         // bit s: slot s holds a segment in flight
  uint32_t lu[3][256];                        // interactions, nscatt, status of the photon (LL_*)
  uint32_t wctr[4][LC_N];                     // per-wave counters
#if SMCRT_LEAN_POOL
  // the event pool: per photon (thread) an in/out slot, and a ring of queued owners
  double ev_dir[3][256];     // in: direction; out: the scattered direction
  double ev_cached[256];     // in/out: the RNG's cached half block
  double ev_tau[256];        // out: the new optical depth
  uint32_t ev_pid[2][256];   // in: photon index words
  uint32_t ev_draws[256];    // in/out: draws taken
  uint32_t ev_code[256];     // in: layer; out: EV_DONE | result bits (written last)
  uint32_t eq[256];          // ticket << 8 | owner thread, written after the owner's slot
  uint32_t eq_head, eq_tail; // tickets: claimed by processors / reserved by producers
#endif
};

__device__ __forceinline__ unsigned long long lean_pack(int32_t x, int32_t y, int32_t z) {
  return (unsigned long long)(uint32_t)(x + 1) | ((unsigned long long)(uint32_t)(y + 1) << LEAN_CELL_BITS) |
         ((unsigned long long)(uint32_t)(z + 1) << (2 * LEAN_CELL_BITS));
}
__device__ __forceinline__ int32_t lean_cell(unsigned long long w, int a) {
  return (int32_t)((w >> (a * LEAN_CELL_BITS)) & LEAN_CELL_MASK) - 1;
}

// A walker's segment (the fields dda_step uses).
struct WalkSeg {
  V3 old;
  double sd, slen;
  int32_t xcell, ycell, zcell;
  uint32_t dda_it;
  bool seg, tflag, fault;
};

// The photon (registers). Counters and rare per-photon fields are in LeanShared.
// A segment request (update_grids entry) is the photon's pos and d at the request, plus the
// move tauint2 makes right after it (pos + d*dir, pos - d*dir or none): the move is applied
// when the segment is handed to the ring, so the request costs no registers.
enum : uint32_t {
  LF_PEND = 1u,    // an EVAL was requested for the current state
  LF_TFLAG = 2u,
  LF_FAULT = 4u,
  LF_REQ = 8u,     // a segment waits to be handed to the ring
  LF_WAIT = 16u,   // waiting for a synchronous segment
  LF_CELLS = 32u,  // xcell/ycell/zcell are the photon's cells
  LF_MOVE_FWD = 64u, LF_MOVE_BACK = 128u,  // the move after the request
  LF_EVQ = 256u,   // the photon's interaction is queued in the block's event pool
};
enum : uint32_t { EV_DONE = 1u << 31, EV_ABSORB = 1u, EV_RUNAWAY = 2u };  // LeanShared::ev_code results
struct LeanPhoton {
  V3 pos, dir;
  Rng rng;
  double tau, taurun, d, minabs;
  int32_t layer;
  int32_t xcell, ycell, zcell;  // valid with LF_CELLS
  uint32_t hop, loopc, st, seq;  // seq: the slot of the next segment (0 .. LEAN_SLOTS-1)
  uint32_t f;                    // LF_* flags
  __device__ __forceinline__ bool has(uint32_t b) const { return (f & b) != 0; }
  __device__ __forceinline__ void set(uint32_t b) { f |= b; }
  __device__ __forceinline__ void clr(uint32_t b) { f &= ~b; }
};

enum : int { LL_INTER = 0, LL_NSCATT, LL_STATUS };  // per-photon fields (LeanShared::lu)
#define LLU(f) (sh->lu[(f)][threadIdx.x])

// count one event per active lane into the wave's counter c (divergent code is fine)
__device__ __forceinline__ void lean_count(LeanShared* sh, int c) {
  const uint64_t m = __ballot(1);
  if ((int)(threadIdx.x & 63) == __builtin_ctzll(m)) atomicAdd(&sh->wctr[threadIdx.x >> 6][c], (uint32_t)__popcll(m));
}

#ifdef SMCRT_DIAG
// Diagnostic builds (-DSMCRT_DIAG): wave-uniform tallies of the lean kernel's schedule, added to
// g_diag[0..15] at the end of each wave (the host prints them per launch), and the s_memtime
// share of each phase in g_diag_t[1..8].
enum : int { LD_TRIPS = 0, LD_WSTEPS, LD_WLANES, LD_PUSH, LD_SYNC, LD_BLOCKED, LD_EVALS, LD_ELANES, LD_P7,
             LD_REVERT, LD_WAITING, LD_IDLE, LD_RING, LD_EVWAIT, LD_BUSY, LD_POOL, LD_POOLN, LD_P7LANES, LD_N };
#define LDIAG(i, v) (ld[(i)] += (uint64_t)(v))
#define LDIAG_T(i)                                                  \
  do {                                                              \
    const unsigned long long t_ = __builtin_amdgcn_s_memtime();     \
    lt[(i)] += t_ - lt_last;                                        \
    lt_last = t_;                                                   \
  } while (0)
#elif defined(SMCRT_ASM_MARKERS)  // analysis builds: phase boundaries visible in the ISA
#define LDIAG(i, v) do {} while (0)
#define LDIAG_T(i) asm volatile("; @@LPHASE " #i)
#else
#define LDIAG(i, v) do {} while (0)
#define LDIAG_T(i) do {} while (0)
#endif

// analysis builds: a hard VGPR budget (the waves-per-EU hint alone is not enforced)
#ifdef SMCRT_LEAN_NUM_VGPR
#define SMCRT_LEAN_VGPR_ATTR __attribute__((amdgpu_num_vgpr(SMCRT_LEAN_NUM_VGPR)))
#else
#define SMCRT_LEAN_VGPR_ATTR
#endif
template <bool LDS_FACES, int GM>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(SMCRT_WAVES_PER_EU_LEAN))) SMCRT_LEAN_VGPR_ATTR void lean_kernel(
    KParams K, const smcrt_sdf_node* __restrict__ nodes, const ProgOp* __restrict__ prog,
    const KCold* __restrict__ C) {
  __shared__ LeanShared shm;
  LeanShared* sh = &shm;
  const double eps = 1e-8;  // inttau2.f90:56
  const bool test_kernel = (K.flags & SMCRT_FLAG_TEST_KERNEL) != 0;
  const bool records_on = (K.flags & SMCRT_FLAG_RECORD_PHOTONS) != 0 && C->records != nullptr;
  const int lane_id = threadIdx.x & 63;
  const int wv = threadIdx.x >> 6;

  extern __shared__ double sh_dyn[];  // [props | faces] | the block's bucket words
  const TopProps* props = K.props;
  const double* xf = K.xface;
  const double* yf = K.yface;
  const double* zf = K.zface;
  int dyn_off = 0;
  if constexpr (LDS_FACES) {
    const int np = 4 * K.n_top;
    const double* gp = (const double*)K.props;
    for (int i = threadIdx.x; i < np; i += blockDim.x) sh_dyn[i] = gp[i];
    const int nf = (K.nx + 1) + (K.ny + 1) + (K.nz + 2);
    double* sh_faces = sh_dyn + np;
    for (int i = threadIdx.x; i < nf; i += blockDim.x) sh_faces[i] = K.xface[i];
    props = (const TopProps*)sh_dyn;
    xf = sh_faces;
    yf = sh_faces + (K.nx + 1);
    zf = yf + (K.ny + 1);
    dyn_off = np + nf;
  }
  unsigned long long* const bstate = (unsigned long long*)(sh_dyn + dyn_off);
  init_buckets(K, C, bstate);
  for (int c = lane_id; c < LC_N; c += 64) sh->wctr[wv][c] = 0;
  for (int f = 0; f < 3; ++f) sh->lu[f][threadIdx.x] = 0;
  sh->busy[threadIdx.x] = 0;
#if SMCRT_LEAN_POOL
  sh->eq[threadIdx.x] = ((threadIdx.x - 256u) & 0xFFFFFFu) << 8;  // (no ticket matches before it is written)
  if (threadIdx.x == 0) sh->eq_head = sh->eq_tail = 0;
#endif
  __syncthreads();

  // lean_margin (see the header comment), per axis, corner coordinates. The debug knob
  // SMCRT_DEBUG_LEAN_MARGIN (K.lean_debug, tests only) drops the margin (1) or defers every
  // segment that starts in the grid (2): the hazards that then occur must be counted.
  const double mf = K.lean_debug ? 0.0 : 2.0 * eps;
  const double mx = mf * (double)(K.nx + 2), my = mf * (double)(K.ny + 2), mz = mf * (double)(K.nz + 2);
  const double ex = 2.0 * K.xmax - mx, ey = 2.0 * K.ymax - my, ez = 2.0 * K.zmax - mz;
  const bool defer_all = K.lean_debug == 2u;

  LeanPhoton P;
  P.st = ST_FETCH; P.f = LF_CELLS;
  P.pos = P.dir = v3(0.0, 0.0, 0.0);
  P.tau = P.taurun = P.d = P.minabs = 0.0;
  P.layer = P.xcell = P.ycell = P.zcell = 0;
  P.hop = P.loopc = P.seq = 0;
  P.rng.init(0);
  WalkSeg W;
  W.old = v3(0.0, 0.0, 0.0);
  W.sd = W.slen = 0.0;
  W.xcell = W.ycell = W.zcell = 0;
  W.dda_it = 0;
  W.seg = W.tflag = W.fault = false;
  V3 wdir = v3(0.0, 0.0, 0.0);
#if SMCRT_LEAN_RCP
  V3 wrcp = v3(0.0, 0.0, 0.0);  // ieee_rcp_f64 of wdir, formed once per segment at the refill
#endif
  uint32_t wmeta = 0;
  uint32_t head = 0, tail = 0;  // the wave's ring tickets (scalar registers)
  BucketLog WB;
  WB.next = WB.end = 0;
  uint32_t overflow = 0, hazards = 0;
  uint32_t w_dep = 0, w_sdf = 0, w_iters = 0;
  uint64_t chunk_base = 0;
  uint32_t chunk_left = 0;
  bool more = true;  // photons may still come from the queue

#ifdef SMCRT_DIAG
  uint64_t ld[LD_N] = {};
  unsigned long long lt[9] = {};
  unsigned long long lt_last = __builtin_amdgcn_s_memtime();
#endif
#if SMCRT_LEAN_POOL
  // a pooled interaction's results (written by whichever wave ran it), see "Event pool"
  auto pickup = [&]() {
    if (P.has(LF_EVQ)) {
      const uint32_t code = __hip_atomic_load(&sh->ev_code[threadIdx.x], __ATOMIC_ACQUIRE,
                                              __HIP_MEMORY_SCOPE_WORKGROUP);
      if (code & EV_DONE) {
        P.clr(LF_EVQ);
        P.rng.draws = sh->ev_draws[threadIdx.x];
        P.rng.cached = sh->ev_cached[threadIdx.x];
        if (code & EV_ABSORB) {  // absorbed: recordWeight once the cells are in
          P.set(LF_TFLAG);
          P.st = ST_ABSORB;
        } else {  // scattered, then the next tauint2 entry
          if (code & EV_RUNAWAY) P.set(LF_FAULT | LF_TFLAG);
          P.dir = v3(sh->ev_dir[0][threadIdx.x], sh->ev_dir[1][threadIdx.x], sh->ev_dir[2][threadIdx.x]);
          P.tau = sh->ev_tau[threadIdx.x];
          P.taurun = 0.0;
          P.hop = 0;
          P.st = ST_H0;
        }
      }
    }
  };
#endif
  // P8: arrive at the hop-loop head, inttau2.f90:61
  auto p8 = [&]() {
    if (!(P.f & (LF_REQ | LF_WAIT | LF_PEND)) && P.st == ST_H0) {
      if (!(P.taurun <= P.tau)) P.st = ST_T2END;
      else if (++P.hop > (uint32_t)MAX_HOP_ITERS) { P.set(LF_FAULT | LF_TFLAG); P.st = ST_T2END; }
      else P.set(LF_PEND);
    }
  };
  for (;; ++w_iters) {
    LDIAG_T(8);
    LDIAG(LD_TRIPS, 1);
    // ---- photon fetch (wave-aggregated work queue), as transport_kernel ----------------
    {
      uint64_t need = __ballot(P.st == ST_FETCH);
      while (need && more) {
        if (chunk_left == 0) {
          unsigned long long base = 0;
          if (lane_id == 0) base = atomicAdd(C->queue, (unsigned long long)SMCRT_FETCH_CHUNK);
          chunk_base = __shfl(base, 0, 64);
          const uint64_t n_photons = C->n_photons;
          chunk_left = (chunk_base < n_photons)
                           ? (uint32_t)((n_photons - chunk_base) < SMCRT_FETCH_CHUNK ? (n_photons - chunk_base)
                                                                                       : SMCRT_FETCH_CHUNK)
                           : 0u;
          if (chunk_left == 0) { more = false; break; }
        }
        const uint32_t n = __popcll(need);
        const uint32_t take = n < chunk_left ? n : chunk_left;
        const uint64_t rank = __popcll(need & ((1ull << lane_id) - 1ull));
        if (P.st == ST_FETCH && rank < take) {
          P.rng.init(C->first_photon + chunk_base + rank);
          P.st = ST_EMIT;
        }
        chunk_base += take;
        chunk_left -= take;
        need = __ballot(P.st == ST_FETCH);
      }
      if (!more && P.st == ST_FETCH) P.st = ST_IDLE;
      // done: no photon, no walk in progress, nothing in the ring
      if (__ballot(P.st != ST_IDLE || W.seg) == 0 && head == tail) break;
    }

#if SMCRT_LEAN_POOL
    // results other waves wrote since this wave's last P7: the photon evaluates this trip
    if (__ballot(P.has(LF_EVQ))) {
      pickup();
      p8();
    }
#endif
    LDIAG(LD_WAITING, __popcll(__ballot(P.has(LF_WAIT))));
    LDIAG(LD_IDLE, __popcll(__ballot(P.st == ST_IDLE)));
    LDIAG(LD_BUSY, __popcll(__ballot(P.st != ST_IDLE)));
    LDIAG_T(1);
    // ---- EVAL: the SDF array at the photon's query point ---------------------------------
    const bool have = (P.f & (LF_PEND | LF_REQ | LF_WAIT)) == LF_PEND;
    EvalOut R;
    R.minabs = R.minv = R.va = R.vb = 0.0; R.maxloc = 0;
    if (__ballot(have)) {
      const bool mask_le = test_kernel && P.st == ST_LAYER;
      // smallStepPos = pos + d*dir (H1, G0): recomputed, since pos, d and dir are unchanged
      // since it was formed (no Fresnel in these scenes, so no refraction in between)
      const V3 q = (P.st == ST_H1 || P.st == ST_G0) ? P.pos + smul(P.d, P.dir) : P.pos;
      R = eval_sdfs(nodes, prog, K.n_prog, q, mask_le, 0, 0);
      const bool counted = P.st == ST_H0 || P.st == ST_H1 || P.st == ST_H3 || P.st == ST_M1 || P.st == ST_G0;
      w_sdf += __popcll(__ballot(have && counted)) * (uint32_t)K.n_top;
      if (have) P.clr(LF_PEND);
    }

    LDIAG(LD_EVALS, __ballot(have) ? 1 : 0);
    LDIAG(LD_ELANES, __popcll(__ballot(have)));
    LDIAG_T(2);
    // ---- P3: consume the EVAL result (transport_kernel's P3 without Fresnel) -------------
    // The three "d = minval(abs(ds))" program points, the bulk of the EVALs, as one block of
    // selects (fewer divergent paths): H0 :63-84/149-152, H3 :133-152, M1 :177-191.
    if (have && (P.st == ST_H0 || P.st == ST_H3 || P.st == ST_M1)) {
      const uint32_t st0 = P.st;
      P.minabs = R.minabs;
      const bool small = st0 == ST_H0 && R.minabs < eps;  // on a surface: micro-step
      const bool out = st0 != ST_H0 && R.minv > 0.0;
      if (out) P.set(LF_TFLAG);
      if (st0 == ST_H0) P.loopc = 0;
      const bool done = P.taurun >= P.tau || P.has(LF_TFLAG);
      P.d = small ? R.minabs + 2.0 * eps : R.minabs;
      uint32_t ns = st0 == ST_M1 ? (out ? (uint32_t)ST_B0 : (uint32_t)ST_M0) : (done ? (uint32_t)ST_T2END : (uint32_t)ST_M0);
      if (small) { ns = ST_H1; P.set(LF_PEND); }
      P.st = ns;
    } else if (have) {
      switch (P.st) {
        case ST_LAYER:  // kernelsMod.f90:1948-1952 (test_kernel: mask ds<=0, :2136)
          P.layer = R.maxloc;
          if (P.layer == 0) { P.set(LF_FAULT); P.st = ST_DONE; }
          else P.st = ST_T2;
          break;
        case ST_H1: {  // :86-123 (the segment starts at the pre-move pos)
          const double kap = props[P.layer - 1].kappa;
          const double t = P.d * kap;
          if (R.maxloc == P.layer) {
            if (P.taurun + t < P.tau) { P.set(LF_MOVE_FWD); P.taurun = P.taurun + t; }
            else { P.d = (P.tau - P.taurun) / kap; P.taurun = P.taurun + t; }
          } else {
            if (P.taurun + t < P.tau) { P.set(LF_MOVE_BACK); P.taurun = P.taurun + t; }
            else { P.d = (P.tau - P.taurun) / kap; P.set(LF_MOVE_BACK); }
          }
          P.st = ST_H2;
          P.set(LF_REQ);
          break;
        }
        case ST_G0: {  // new layer and the glancing loop, :220-245; equal n: cross, :318-328
          const int32_t new_layer = R.maxloc;
          if (new_layer == P.layer && R.minabs < eps) {  // (old_layer == layer here)
            if (++P.loopc > (uint32_t)MAX_GLANCE_ITERS) { P.set(LF_FAULT | LF_TFLAG); P.st = ST_T2END; break; }
            P.d = P.d + eps;
            P.set(LF_PEND);
            break;
          }
          if (new_layer == 0) { P.set(LF_TFLAG); P.st = ST_T2END; break; }
          P.layer = new_layer;
          P.st = ST_X1;
          P.set(LF_REQ);
          break;
        }
        default:
          break;
      }
    }

    // ---- P4: a march step, :155-176 ------------------------------------------------------
    if (!(P.f & (LF_REQ | LF_WAIT)) && P.st == ST_M0) {
      if (!(P.d >= eps)) {
        P.st = ST_B0;
      } else if (++P.loopc > (uint32_t)MAX_MARCH_ITERS) {
        P.set(LF_FAULT | LF_TFLAG); P.st = ST_B0;
      } else {
        const double kap = props[P.layer - 1].kappa;
        const double t = P.d * kap;
        if (P.taurun + t < P.tau) {
          P.taurun = P.taurun + t;
          P.st = ST_M1; P.set(LF_PEND);
        } else {
          P.d = (P.tau - P.taurun) / kap;
          P.taurun = P.tau;
          P.st = ST_B0;
        }
        P.set(LF_REQ | LF_MOVE_FWD);  // pos += d*dir once the segment from pos is handed out
      }
    }

    LDIAG_T(3);
    // ---- hand the new segments to the ring (update_grids entry, :401-415) -----------------
    if (__ballot(P.has(LF_REQ))) {
      bool push = false, sync = false;
      unsigned long long cw = 0;
      V3 old = v3(0.0, 0.0, 0.0);
      const uint32_t slot = P.seq;
      if (P.has(LF_REQ) && !(sh->busy[threadIdx.x] & (1u << slot))) {  // (else: retry next trip)
        lean_count(sh, LC_UPD);
        old = v3(P.pos.x + K.xmax, P.pos.y + K.ymax, P.pos.z + K.zmax);
        const int32_t ci = cell_of<GM>(old.x, K.nx, K.xmax, K.inv2x, K.fex),
                      cj = cell_of<GM>(old.y, K.ny, K.ymax, K.inv2y, K.fey),
                      ck = cell_of<GM>(old.z, K.nz, K.zmax, K.inv2z, K.fez);
        // tauint2's move after update_grids (inttau2.f90:98-122, 163-173)
        if (P.has(LF_MOVE_FWD)) P.pos = P.pos + smul(P.d, P.dir);
        else if (P.has(LF_MOVE_BACK)) P.pos = P.pos - smul(P.d, P.dir);
        P.clr(LF_REQ | LF_MOVE_FWD | LF_MOVE_BACK);
        if (ci == -1 || cj == -1 || ck == -1) {  // outside the grid: tflag, no walk
          P.set(LF_TFLAG | LF_CELLS);
          P.xcell = ci; P.ycell = cj; P.zcell = ck;
        } else {
          const double len = P.d;
          const V3 e = v3(old.x + P.dir.x * len, old.y + P.dir.y * len, old.z + P.dir.z * len);
          const bool inside = old.x >= mx && old.x <= ex && old.y >= my && old.y <= ey && old.z >= mz &&
                              old.z <= ez && e.x >= mx && e.x <= ex && e.y >= my && e.y <= ey && e.z >= mz &&
                              e.z <= ez;
          push = true;
          sync = !inside && !defer_all;
          cw = lean_pack(ci, cj, ck);
        }
      }
      const uint64_t pm = __ballot(push);
      LDIAG(LD_PUSH, __popcll(pm));
      LDIAG(LD_SYNC, __popcll(__ballot(push && sync)));
      LDIAG(LD_BLOCKED, __popcll(__ballot(P.has(LF_REQ))));
      if (pm) {
        const uint32_t rank = __builtin_amdgcn_mbcnt_hi((uint32_t)(pm >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)pm, 0u));
        if (push) {
          const uint32_t ix = (tail + rank) & (LEAN_RING - 1);
          sh->ox[wv][ix] = old.x; sh->oy[wv][ix] = old.y; sh->oz[wv][ix] = old.z;
          sh->dx[wv][ix] = P.dir.x; sh->dy[wv][ix] = P.dir.y; sh->dz[wv][ix] = P.dir.z;
          sh->sl[wv][ix] = P.d;
          sh->cw[wv][ix] = cw;
          sh->meta[wv][ix] = (uint32_t)lane_id | (slot << 6) | (sync ? 256u : 0u);
          atomicOr(&sh->busy[threadIdx.x], 1u << slot);
          P.seq = P.seq + 1 == LEAN_SLOTS ? 0u : P.seq + 1;
          P.clr(LF_CELLS);
          if (sync) P.set(LF_WAIT);
        }
        tail += (uint32_t)__popcll(pm);
      }
    }

    LDIAG(LD_RING, tail - head);
    LDIAG_T(4);
    // idle walkers take the oldest segments of the ring (wave-uniform call)
    auto refill = [&](uint32_t min_idle) {
      const uint64_t im = __ballot(!W.seg);
      const uint32_t avail = tail - head;
      const uint32_t ni = (uint32_t)__popcll(im);
      const uint32_t take = ni < avail ? ni : avail;
      if (take && ni >= min_idle) {
        const uint32_t rank = __builtin_amdgcn_mbcnt_hi((uint32_t)(im >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)im, 0u));
        if (!W.seg && rank < take) {
          const uint32_t ix = (head + rank) & (LEAN_RING - 1);
          W.old = v3(sh->ox[wv][ix], sh->oy[wv][ix], sh->oz[wv][ix]);
          wdir = v3(sh->dx[wv][ix], sh->dy[wv][ix], sh->dz[wv][ix]);
#if SMCRT_LEAN_RCP
          wrcp = v3(ieee_rcp_f64(wdir.x), ieee_rcp_f64(wdir.y), ieee_rcp_f64(wdir.z));
#endif
          W.slen = sh->sl[wv][ix];
          const unsigned long long cw = sh->cw[wv][ix];
          W.xcell = lean_cell(cw, 0); W.ycell = lean_cell(cw, 1); W.zcell = lean_cell(cw, 2);
          wmeta = sh->meta[wv][ix];
          W.sd = 0.0; W.dda_it = 0;
          W.seg = true; W.tflag = false; W.fault = false;
        }
        head += take;
      }
    };
    // ---- walk phase: crossings of ring segments on every lane ------------------------------
#pragma unroll 1  // one copy of the crossing: the unrolled steps' live ranges cost occupancy
    for (int k = 0; k < SMCRT_LEAN_STEPS + SMCRT_LEAN_EXTRA; ++k) {
      refill(k == 0 ? 1u : (uint32_t)SMCRT_LEAN_REFILL_IDLE);
      const uint64_t am = __ballot(W.seg);
      if (!am) break;
      if (k >= SMCRT_LEAN_STEPS && __popcll(am) < SMCRT_LEAN_BUSY) break;
      LDIAG(LD_WSTEPS, 1);
      LDIAG(LD_WLANES, __popcll(am));
      bool dep = false;
      uint32_t vox = 0;
      double val = 0.0;
#ifdef SMCRT_LEAN_ABL_NO_WALK  // register-pressure analysis builds only
      W.seg = false;
#else
#if SMCRT_LEAN_RCP
      if (W.seg) dda_step_r<GM>(K, W, wdir, wrcp, xf, yf, zf, dep, vox, val, 1.0);
#else
      if (W.seg) dda_step<GM>(K, W, wdir, xf, yf, zf, dep, vox, val, 1.0);
#endif
#endif
      w_dep += __popcll(__ballot(dep));
#ifndef SMCRT_LEAN_ABL_NO_EMIT  // register-pressure analysis builds only
      emit_bucketed(K, C, WB, dep, vox, val, overflow, bstate);
#else
      if (__ballot(dep) == 0x123ull) atomic_add_nr(C->jmean + vox, val);
#endif
      // a finished segment: its cells and flags to the owner's slot, then the slot is free
      if ((am >> lane_id & 1ull) && !W.seg) {
        const uint32_t owner = (uint32_t)(wv * 64) + (wmeta & 63u), slot = (wmeta >> 6) & 3u;
        const bool sync = (wmeta & 256u) != 0;
        if (!sync && (W.tflag || W.fault)) ++hazards;  // cannot happen (header comment); counted as a fault
        sh->pcell[owner][slot] = lean_pack(W.xcell, W.ycell, W.zcell) | (W.tflag ? LEAN_TFLAG : 0ull) |
                                 (W.fault ? LEAN_FAULT : 0ull);
        atomicAnd(&sh->busy[owner], ~(1u << slot));
      }
    }

    refill(1);  // (the ring bound above: every walker busy, or the ring empty)
#ifdef SMCRT_LEAN_ABL_DROP_WALK  // register-pressure analysis builds only (not exact)
    W.seg = false; W.old = wdir = v3(0.0, 0.0, 0.0); W.sd = W.slen = 0.0; wmeta = 0;
    W.xcell = W.ycell = W.zcell = 0; W.dda_it = 0;
#endif
    LDIAG_T(5);
    // ---- P5: a synchronous segment finished; after a segment: next program point ---------
    if (P.has(LF_WAIT) && !(sh->busy[threadIdx.x] & (1u << ((P.seq + LEAN_SLOTS - 1) % LEAN_SLOTS)))) {
      const unsigned long long w = sh->pcell[threadIdx.x][(P.seq + LEAN_SLOTS - 1) % LEAN_SLOTS];
      P.xcell = lean_cell(w, 0); P.ycell = lean_cell(w, 1); P.zcell = lean_cell(w, 2);
      P.set(LF_CELLS);
      if (w & LEAN_TFLAG) P.set(LF_TFLAG);
      if (w & LEAN_FAULT) P.set(LF_FAULT);
      P.clr(LF_WAIT);
    }
    const bool free_ = !(P.f & (LF_REQ | LF_WAIT));
    if (free_ && (P.st == ST_H2 || P.st == ST_B0 || P.st == ST_X1)) {
      if (P.st == ST_X1) {  // :326-335 (pos = smallStepPos)
        P.taurun = P.taurun + P.d * props[P.layer - 1].kappa;
        P.pos = P.pos + smul(P.d, P.dir);
      }
      if (P.st == ST_H2) {
        P.st = ST_H3; P.set(LF_PEND);
      } else if (P.st == ST_X1) {
        P.st = P.has(LF_TFLAG) ? ST_T2END : ST_H0;
      } else if (P.taurun >= P.tau || P.has(LF_TFLAG)) {  // B0, :204-207
        P.st = ST_T2END;
      } else {  // boundary probe, :213-222 (smallStepPos = pos + d*dir, formed at the EVAL)
        P.d = P.minabs + 2.0 * eps;
        P.loopc = 0;
        P.st = ST_G0; P.set(LF_PEND);
      }
    }

    // ---- P6: tauint2 write-back checks, :341-362 -----------------------------------------
    if (free_ && P.st == ST_T2END) {
      if (fabs(P.pos.x) > K.xmax) P.set(LF_TFLAG);
      if (fabs(P.pos.y) > K.ymax) P.set(LF_TFLAG);
      if (fabs(P.pos.z) > K.zmax) P.set(LF_TFLAG);
      P.st = ST_INTERACT;
    }
    // the final cells of the photon's deferred segments, once they are all done (read only
    // where they are used: recordWeight of an absorption, the photon record)
    if (!P.has(LF_CELLS) && (P.st == ST_ABSORB || (records_on && P.st == ST_DONE)) && sh->busy[threadIdx.x] == 0) {
      const unsigned long long w = sh->pcell[threadIdx.x][(P.seq + LEAN_SLOTS - 1) % LEAN_SLOTS];
      P.xcell = lean_cell(w, 0); P.ycell = lean_cell(w, 1); P.zcell = lean_cell(w, 2);
      P.set(LF_CELLS);
    }

    LDIAG_T(6);
    // recordWeight of an absorbed photon (kernelsMod.f90:2202-2220) once its cells are in
    if (P.st == ST_ABSORB && P.has(LF_CELLS)) {
      if (P.xcell < 1 || P.xcell > K.nx || P.ycell < 1 || P.ycell > K.ny || P.zcell < 1 || P.zcell > K.nz)
        P.set(LF_FAULT);
      else if (C->absorb) atomic_add_nr(C->absorb + lin(K, P.xcell, P.ycell, P.zcell), 1.0);
      P.st = ST_DONE;
    }
    // ---- P7: photon events, batched as in transport_kernel ---------------------------------
#if SMCRT_LEAN_POOL
    // Event pool. An interaction that will draw (albedo roulette, then scatter and the next
    // tauint2 entry, kernelsMod.f90:1958-1975 + inttau2.f90:48-60) is not run by its own wave:
    // the photon writes its direction, RNG state and layer to its slot in LDS and queues its
    // thread index in the block's ring; any wave of the block that finds SMCRT_LEAN_POOL_MIN
    // queued (or has nothing else to do) claims up to 64 of them and runs them on its lanes,
    // writing the results back to the owners' slots, which the owners pick up. A photon's draws
    // come from its own Philox stream, so which lane runs its event changes no bit.
    // Ordering: LDS operations of one wave complete in order; slot data precede the release
    // store of the ring entry (or of the result code), which the reader acquires.
    {
      pickup();
      // queue this wave's interactions that draw (test_kernel runs its events locally: moments)
      const bool qev = free_ && !test_kernel && P.st == ST_INTERACT && !(P.f & (LF_TFLAG | LF_FAULT | LF_EVQ)) &&
                       LLU(LL_INTER) + 1u <= (uint32_t)MAX_INTERACTIONS;
      const uint64_t qm = __ballot(qev);
      if (qm) {
        const int first = __builtin_ctzll(qm);
        uint32_t base = 0;
        if (lane_id == first) base = atomicAdd(&sh->eq_tail, (uint32_t)__popcll(qm));
        base = __builtin_amdgcn_readlane(base, first);
        if (qev) {
          const uint32_t rank = __builtin_amdgcn_mbcnt_hi((uint32_t)(qm >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)qm, 0u));
          sh->ev_dir[0][threadIdx.x] = P.dir.x; sh->ev_dir[1][threadIdx.x] = P.dir.y; sh->ev_dir[2][threadIdx.x] = P.dir.z;
          sh->ev_cached[threadIdx.x] = P.rng.cached;
          sh->ev_pid[0][threadIdx.x] = P.rng.pid_lo; sh->ev_pid[1][threadIdx.x] = P.rng.pid_hi;
          sh->ev_draws[threadIdx.x] = P.rng.draws;
          sh->ev_code[threadIdx.x] = (uint32_t)P.layer;
          const uint32_t t = base + rank;
          __hip_atomic_store(&sh->eq[t & 255u], ((t & 0xFFFFFFu) << 8) | threadIdx.x, __ATOMIC_RELEASE,
                             __HIP_MEMORY_SCOPE_WORKGROUP);
          P.set(LF_EVQ);
        }
      }
      // run queued events: SMCRT_LEAN_POOL_MIN of them, or any when every busy lane of this wave
      // waits for one (the wave has nothing else to do; this also drains the pool at the end)
      const uint64_t qbusy = __ballot(P.st != ST_IDLE && P.st != ST_FETCH);
      const uint64_t qwait = __ballot(P.has(LF_EVQ));
      uint32_t claim_h = 0, claim_n = 0;
      if (lane_id == 0) {
        const uint32_t want = (qbusy != 0 && qwait == qbusy) ? 1u : (uint32_t)SMCRT_LEAN_POOL_MIN;
        for (;;) {
          const uint32_t h = __hip_atomic_load(&sh->eq_head, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
          const uint32_t tl = __hip_atomic_load(&sh->eq_tail, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
          const uint32_t av = tl - h;
          if (av < want) break;
          const uint32_t n = av < 64u ? av : 64u;
          uint32_t exp = h;
          if (__hip_atomic_compare_exchange_strong(&sh->eq_head, &exp, h + n, __ATOMIC_RELAXED, __ATOMIC_RELAXED,
                                                   __HIP_MEMORY_SCOPE_WORKGROUP)) {
            claim_h = h; claim_n = n;
            break;
          }
        }
      }
      claim_n = __builtin_amdgcn_readfirstlane(claim_n);
      claim_h = __builtin_amdgcn_readfirstlane(claim_h);
      LDIAG(LD_POOL, claim_n ? 1 : 0);
      LDIAG(LD_POOLN, claim_n);
      if (claim_n) {
        if ((uint32_t)lane_id < claim_n) {
          const uint32_t t = claim_h + (uint32_t)lane_id;
          uint32_t e;
          // the producer reserved the ticket before writing its entry: wait for it (a few cycles)
          while (((e = __hip_atomic_load(&sh->eq[t & 255u], __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP)) >> 8) !=
                 (t & 0xFFFFFFu))
            __builtin_amdgcn_s_sleep(1);
          const uint32_t o = e & 255u;
          Rng rg;
          rg.pid_lo = sh->ev_pid[0][o]; rg.pid_hi = sh->ev_pid[1][o];
          rg.draws = sh->ev_draws[o]; rg.cached = sh->ev_cached[o];
          const int32_t layer = (int32_t)sh->ev_code[o];
          const TopProps pr = props[layer - 1];
          // kernelsMod.f90:1958-1975 (the local path below, for another photon)
          const double ran = rg.next(K.key0, K.key1);
          ++sh->lu[LL_INTER][o];
          uint32_t res = 0;
          if (!(ran < pr.albedo)) {
            sh->lu[LL_STATUS][o] = 1;
            lean_count(sh, LC_ABSORBED);
            res = EV_ABSORB;
          } else {
            Lane L;
            L.dir = v3(sh->ev_dir[0][o], sh->ev_dir[1][o], sh->ev_dir[2][o]);
            L.rng = rg; L.fault = false; L.tflag = false;
            scatter(K, L, pr.hgg);  // photon.f90:1045-1103
            rg = L.rng;
            if (L.fault) res = EV_RUNAWAY;
            ++sh->lu[LL_NSCATT][o];
            lean_count(sh, LC_SCATTERS);
            lean_count(sh, LC_TAU);  // tauint2 entry, inttau2.f90:48-60
            sh->ev_tau[o] = -det_log(rg.next(K.key0, K.key1));
            sh->ev_dir[0][o] = L.dir.x; sh->ev_dir[1][o] = L.dir.y; sh->ev_dir[2][o] = L.dir.z;
          }
          sh->ev_draws[o] = rg.draws;
          sh->ev_cached[o] = rg.cached;
          __hip_atomic_store(&sh->ev_code[o], res | EV_DONE, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
        }
        pickup();  // (this wave's own events among them)
      }
    }
#endif
    {
      const bool ev = free_ && !P.has(LF_EVQ) && (P.st == ST_INTERACT || P.st == ST_T2 || P.st == ST_EMIT || P.st == ST_DONE);
      const uint64_t evm = __ballot(ev);
      const uint64_t busy = __ballot(P.st != ST_IDLE && P.st != ST_FETCH && !P.has(LF_EVQ));
      const uint32_t nev = __popcll(evm);
#if SMCRT_LEAN_POOL
      const bool run_ev = nev && (nev >= SMCRT_LEAN_LOCAL_EVENT_LANES || evm == busy);
#else
      const bool run_ev = nev && (nev >= SMCRT_LEAN_EVENT_LANES || evm == busy);
#endif
      LDIAG(LD_P7, run_ev ? 1 : 0);
      LDIAG(LD_EVWAIT, run_ev ? 0 : nev);
      LDIAG(LD_P7LANES, run_ev ? nev : 0);
#ifdef SMCRT_LEAN_ABL_NO_P7  // register-pressure analysis builds only (tools/regs.sh)
      if (run_ev && __ballot(P.st == 12345)) {
#else
      if (run_ev) {
#endif
        if (ev && P.st == ST_INTERACT) {  // kernelsMod.f90:1958-1975 / 2126-2170
          if (P.f & (LF_TFLAG | LF_FAULT)) {
            P.st = ST_DONE;
          } else if (LLU(LL_INTER) + 1u > (uint32_t)MAX_INTERACTIONS) {
            ++LLU(LL_INTER);
            P.set(LF_FAULT); P.st = ST_DONE;
          } else {
            const double ran = P.rng.next(K.key0, K.key1);
            const TopProps pr = props[P.layer - 1];
            const bool sc = ran < pr.albedo;
            {
              ++LLU(LL_INTER);
              if (!sc) {
                P.set(LF_TFLAG); LLU(LL_STATUS) = 1; lean_count(sh, LC_ABSORBED);
                // recordWeight(packet, 1.0) at the photon's cells: those of its last segment,
                // which may still be walked (ST_ABSORB adds it once they are in)
                P.st = test_kernel ? ST_DONE : ST_ABSORB;
#ifdef SMCRT_DIAG
                if (!P.has(LF_CELLS)) atomicAdd(&::g_diag[LD_REVERT], 1ull);
#endif
              } else {
                // scatter, photon.f90:1045-1103
                Lane L;
                L.dir = P.dir; L.rng = P.rng; L.fault = false; L.tflag = false;
                scatter(K, L, pr.hgg);
                P.dir = L.dir; P.rng = L.rng;
                if (L.fault) P.set(LF_FAULT | LF_TFLAG);  // (renormalisation runaway)
                const uint32_t st = ++LLU(LL_NSCATT);
                lean_count(sh, LC_SCATTERS);
                if (test_kernel) {
                  if (st >= 1 && st <= 4) {
                    double* const moments = C->moments;
                    if (moments) {
                      double* m = moments + 3 * (st - 1);
                      double* m2 = moments + 12 + 3 * (st - 1);
                      atomic_add_nr(m + 0, P.pos.x); atomic_add_nr(m + 1, P.pos.y); atomic_add_nr(m + 2, P.pos.z);
                      atomic_add_nr(m2 + 0, P.pos.x * P.pos.x);
                      atomic_add_nr(m2 + 1, P.pos.y * P.pos.y);
                      atomic_add_nr(m2 + 2, P.pos.z * P.pos.z);
                    }
                  } else if (K.flags & SMCRT_FLAG_END_EARLY) {
                    P.set(LF_TFLAG);
                    LLU(LL_STATUS) = 4;
                  }
                }
                P.st = ST_T2;
              }
            }
          }
        }
        if (ev && P.st == ST_T2) {  // tauint2 entry, inttau2.f90:48-60
          lean_count(sh, LC_TAU);
          P.tau = -det_log(P.rng.next(K.key0, K.key1));
          P.taurun = 0.0;
          P.hop = 0;
          P.st = ST_H0;  // arrives in P8
        }
        if (ev && P.st == ST_EMIT) {  // kernelsMod.f90:1937-1945
          P.clr(LF_FAULT); P.layer = 0;
          LLU(LL_STATUS) = 0; LLU(LL_NSCATT) = 0; LLU(LL_INTER) = 0;
          Lane L;
          L.rng = P.rng; L.xcell = L.ycell = L.zcell = 0; L.layer = 0; L.tflag = false;
          emit<GM, false>(K, C, L, 0u);
          if (!test_kernel) {
            int64_t tries = 0;
            while (cell_out(K, L)) {
              if (++tries > MAX_EMIT_TRIES) { P.set(LF_FAULT); break; }
              lean_count(sh, LC_RETRIES);
              emit<GM, false>(K, C, L, 0u);
            }
          }
          P.pos = L.pos; P.dir = L.dir; P.rng = L.rng; P.clr(LF_TFLAG);
          P.layer = L.layer;
          P.xcell = L.xcell; P.ycell = L.ycell; P.zcell = L.zcell;
          P.set(LF_CELLS);
          if (!test_kernel && !P.has(LF_FAULT) && (K.flags & SMCRT_FLAG_RENDER_SOURCE) && C->emission)
            atomic_add_nr(C->emission + lin(K, P.xcell, P.ycell, P.zcell), 1.0);
          if (P.has(LF_FAULT)) P.st = ST_DONE;
          else { P.st = ST_LAYER; P.set(LF_PEND); }
        }
        if (ev && P.st == ST_DONE && (P.has(LF_CELLS) || !records_on)) {  // photon finished
          if (P.has(LF_FAULT)) { LLU(LL_STATUS) = 3; lean_count(sh, LC_FAULTS); }
          else if (LLU(LL_STATUS) == 0) { LLU(LL_STATUS) = 2; lean_count(sh, LC_ESCAPED); }
          lean_count(sh, LC_PHOTONS);
          atomicAdd(&sh->wctr[wv][LC_DRAWS], P.rng.draws);
          if (records_on) {
            const uint64_t pid = ((uint64_t)P.rng.pid_hi << 32) | P.rng.pid_lo;
            smcrt_photon_record* r = C->records + (pid - C->first_photon);
            r->pos[0] = P.pos.x; r->pos[1] = P.pos.y; r->pos[2] = P.pos.z;
            r->dir[0] = P.dir.x; r->dir[1] = P.dir.y; r->dir[2] = P.dir.z;
            r->weight = 1.0;
            r->cell[0] = P.xcell; r->cell[1] = P.ycell; r->cell[2] = P.zcell;
            r->layer = P.layer;
            r->nscatt = LLU(LL_NSCATT);
            r->bounces = 0;
            r->draws = P.rng.draws;
            r->status = LLU(LL_STATUS);
          }
          P.clr(LF_TFLAG | LF_FAULT);
          P.st = ST_FETCH;
        }
      }
    }

    LDIAG_T(7);
    // ---- P8: arrive at the hop-loop head, :61 --------------------------------------------
    p8();
  }

#ifdef SMCRT_DIAG
  if (lane_id == 0) {
    for (int i = 0; i < LD_N; ++i)
      if (i != LD_REVERT && ld[i]) atomicAdd(&::g_diag[i], (unsigned long long)ld[i]);
    for (int i = 1; i < 9; ++i) atomicAdd(&::g_diag_t[i], lt[i]);
  }
#endif
  close_buckets(K, C, WB, w_dep - overflow, overflow);
  __syncthreads();  // every wave of the block is done depositing
  close_block_buckets(K, C, bstate);

  // ---- per-wave counters ---------------------------------------------------------------
  unsigned long long* const counters = C->counters;
  const uint32_t hz = wave_sum_u32(hazards);
  if (lane_id == 0) {
    if (hz) {  // reported: smcrt_kernel_times.lean_hazards, and SMCRT_CTR_FAULTS below
      atomicAdd(C->dep_ctl + 5, hz);
      atomicAdd(C->lean_hazards, (unsigned long long)hz);
    }
    if (C->dep_ctl && sh->wctr[wv][LC_UPD]) atomicAdd(C->dep_ctl + 6, sh->wctr[wv][LC_UPD]);  // segments
    if (counters) {
      const uint32_t* c = sh->wctr[wv];
      const uint32_t v[SMCRT_NCOUNTERS] = {c[LC_PHOTONS], c[LC_RETRIES], c[LC_SCATTERS], c[LC_ABSORBED], w_sdf,
                                           w_dep,         c[LC_UPD],     c[LC_TAU],      0u,             0u,
                                           0u,            c[LC_FAULTS] + hz, c[LC_DRAWS], 0u,             c[LC_ESCAPED],
                                           w_iters};
      for (int i = 0; i < SMCRT_NCOUNTERS; ++i)
        if (v[i]) atomicAdd(counters + i, (unsigned long long)v[i]);
    }
    double* const nscatt = C->nscatt;
    if (nscatt && sh->wctr[wv][LC_SCATTERS]) atomic_add_nr(nscatt, (double)sh->wctr[wv][LC_SCATTERS]);
  }
}

#undef LLU

}  // namespace smcrt
