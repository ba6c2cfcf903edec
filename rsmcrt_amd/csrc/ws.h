// ws.h — the lean path's transport kernel: wave-specialised blocks (photon, event and walker waves).
//
// The path is noBiasPropagation kernelsMod.f90:1901-1976 -> tauint2 inttau2.f90:15-364 ->
// update_grids :367-465, restated with transport_kernel's arithmetic (kernels.h), with the same
// results bit for bit, for scenes of few tops with no survival bias, a plain source and bucketed
// path-length deposition (smcrt.hip: lean_ok; the XF instantiation adds Fresnel interfaces and
// detectors).
//
// Why. A photon and its voxel walk want different code and different registers: the walk (a
// crossing and the bucket emit) holds no photon state, the photon's code holds no walk. Round 4
// ran both in every wave (lean_kernel, 167 VGPRs, three waves a SIMD); here a block of
// WS_WAVES = 16 waves splits them, each role within 128 VGPRs (four waves a SIMD):
//   * photon waves (WS_PW = 8) run fetch, EVAL, P3/P4, the segment hand-out, P5/P6 and P8 on
//     their 64 photons; a segment (update_grids entry) goes into one of the photon's slots and a
//     token for it into the block's ring in LDS;
//   * walker waves (7) take the oldest tokens of the ring into idle lanes, walk the segments
//     SMCRT_WS_DDA crossings per iteration with dda_step_r (transport.h), file the records into
//     the block's buckets (deposit.h) and, at a segment's end, write its final cells and flags
//     into the owner photon's slot;
//   * event waves (WS_EW = 1, at issue priority 3) run the photons' interactions: the albedo
//     roulette, scatter and the next tauint2 entry (kernelsMod.f90:1958-1975, photon.f90:
//     1045-1103, inttau2.f90:48-60), the tauint2 entry after an emission, the emission itself
//     (kernelsMod.f90:1937-1945 with the source's draws, photon.f90:311-710) and, in the XF
//     instantiation, reflect_refract (inttau2.f90:248-328, surfaces.f90:14-84). A photon with
//     such an event writes its direction, RNG state and layer into its event slot, queues its
//     lane in the block's event queue and waits; an event lane takes the queued owner, runs the
//     event on the owner's values with the owner's own Philox stream and writes the results
//     back, so the event code runs on full waves. Completion, the rare terminal interactions
//     and every event of test_kernel runs (moments) stay in the photon waves, batched once
//     SMCRT_LEAN_EVENT_LANES lanes wait.
// A segment's walk is a pure function of (start, direction, length) (the start cell is
// recomputed from the start with the same cell_of) and the deferred/synchronous rule and the
// hazard accounting are lean.h's, so the records, counters and tallies are transport_kernel's;
// only the order of the fp64 jmean sums differs.
//
// Segments and the block ring. A photon's segment lives in one of its WS_SLOTS slots (`seg`,
// structure of arrays over the photon lanes), which its busy bit guards: the photon writes a
// slot only while the bit is clear and sets it, the walker clears it when the walk is done. The
// ring (multi-producer, multi-consumer, LDS) carries only tokens: owner, slot, synchronous flag.
// Tickets are matched one to one: photon waves take them from `tail` (one reserved per
// segment), walker lanes from `head` (one held per idle lane; head may run ahead of tail).
// Ticket t uses ring word t mod WS_RING, a sequence lock ordering the word's laps:
//     written(t) -> consumed(t) -> written(t + WS_RING) -> consumed(t + WS_RING) -> ...
//   * a photon wave reserves n tickets with one LDS add on `tail`; for each ticket t the lane
//     writes its slot, sets its busy bit, waits until the word shows consumed(t - WS_RING) (the
//     initial 0 for t < WS_RING) and stores written(t) with release (the slot before the token);
//   * a walker lane that holds ticket t checks its word once per iteration (no wait); when it
//     shows written(t) (acquire) the lane stores consumed(t), reads the owner's slot and walks;
//   * every wait is a producer's, for the consumption of a strictly smaller ticket whose holder
//     checks it every iteration, so the waits cannot form a cycle. In practice a producer never
//     waits: a photon has at most WS_SLOTS segments in flight (its busy bits), WS_RING >=
//     WS_NPL * WS_SLOTS, and held tickets are taken as soon as they are written;
//   * termination: each photon wave decrements `alive` after its last photon (its last push
//     precedes that in its LDS order), which fixes the final tail; walker lanes drop tickets at
//     or past it, and a walker wave ends when it holds no segment and no earlier ticket.
// Otherwise no wave waits for another except a photon for its synchronous segment (and the
// bucket claims of deposit.h among the walker waves, whose bound is unchanged: only walkers
// deposit). An emission's position comes back in the start fields of the photon's next slot,
// which must be free when the emission is queued.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "lean.h"

namespace smcrt {

#ifndef SMCRT_WS_PHOTON_WAVES
#define SMCRT_WS_PHOTON_WAVES 8
#endif
#ifndef SMCRT_WS_EVENT_WAVES
#define SMCRT_WS_EVENT_WAVES 1
#endif
#ifndef SMCRT_WS_DDA
#define SMCRT_WS_DDA 2  // crossing steps per walker iteration (1: -2.5 %, profiles/r05_ws/ab_walker.txt)
#endif
#ifndef SMCRT_WS_WAVES
#define SMCRT_WS_WAVES 16
#endif
// the photon hands a segment's start cell to its walker in the slot's cell word (1) instead of
// the walker recomputing it from the start (0); the same cell_of on the same start either way
// the plain instantiation reads the deferral box from KParams too (1) or keeps it in VGPRs (0)
#ifndef SMCRT_WS_KBOUNDS_PLAIN
#define SMCRT_WS_KBOUNDS_PLAIN 0
#endif
#ifndef SMCRT_WS_START_CELLS
#define SMCRT_WS_START_CELLS 1
#endif
constexpr int WS_WAVES = SMCRT_WS_WAVES;  // waves per block (8: two blocks per CU, 16: one)
constexpr int WS_THREADS = 64 * WS_WAVES;
constexpr int WS_PW = SMCRT_WS_PHOTON_WAVES;  // photon waves per block (waves 0 .. WS_PW-1)
constexpr int WS_EW = SMCRT_WS_EVENT_WAVES;   // event waves (next), the rest walk
static_assert(WS_PW >= 1 && WS_EW >= 1 && WS_PW + WS_EW < WS_WAVES, "a block needs all three roles");
constexpr uint32_t WS_NPL = 64u * WS_PW;  // photon lanes per block (<= 512: 9 owner bits)
constexpr uint32_t ws_pow2(uint32_t v) { return v <= 1 ? 1 : 2 * ws_pow2((v + 1) / 2); }
constexpr uint32_t WS_EQ = ws_pow2(WS_NPL);  // event queue entries (a photon has at most one event queued)
// meta word: owner (9 bits) | slot << 9 (2 bits) | synchronous << 11 | consumed << 12 |
// ((ticket + 1) mod 2^19) << 13; 0 = never written
constexpr uint32_t WS_CONSUMED = 1u << 12;
constexpr uint32_t WS_SEQ_MASK = 0xFFFFF000u;  // ticket and consumed bit
__device__ __forceinline__ uint32_t ws_tick(uint32_t t) { return ((t + 1u) & 0x7FFFFu) << 13; }

enum : int { SG_OX = 0, SG_OY, SG_OZ, SG_DX, SG_DY, SG_DZ, SG_LEN, SG_N };  // segment fields
// SL: segments a photon may have in flight (its slots). Three measured +2 % over two on M1
// (profiles/r05_ws/ab_slots.txt); they need 146 KiB of LDS, so grids whose tile words and faces
// do not fit beside them run the two-slot instantiation (109 KiB).
template <uint32_t SL>
struct WsSharedT {
  static constexpr uint32_t SLOTS = SL;
  static constexpr uint32_t RING = ws_pow2(WS_NPL * SL);  // ring words
  static_assert(SL >= 1 && SL <= 4, "two slot bits in a meta word");
  static_assert(RING >= WS_NPL * SL && RING < (1u << 18), "ring bound");
  // a photon's segments in flight, one per slot (its busy bit guards the slot): start (corner
  // coordinates), direction, length; the emitted position (EMIT, in a free slot's start)
  double seg[SL][SG_N][WS_NPL];
  uint32_t meta[RING];                           // the ring: owner, slot, flags, sequence lock
  unsigned long long pcell[WS_NPL][SL];          // a finished segment: cells | tflag | fault
  uint32_t busy[WS_NPL];                         // bit s: slot s holds a segment in flight
  uint32_t lu[3][WS_NPL];                        // interactions, nscatt, status (LL_*)
  uint32_t wctr[WS_WAVES][LC_N];                 // per-wave counters
  // the event queue (see "Event waves" above): per photon lane an in/out slot, and a queue of
  // owner lanes with the ring's sequence lock
  double ev_dir[3][WS_NPL];   // in: direction; out: the scattered (or emitted) direction
  double ev_cached[WS_NPL];   // in/out: the RNG's cached half block
  double ev_tau[WS_NPL];      // out: the new optical depth
  uint32_t ev_pid[2][WS_NPL]; // in: photon index words
  uint32_t ev_draws[WS_NPL];  // in/out: draws taken
  uint32_t ev_code[WS_NPL];   // in: layer | kind << 16 | slot << 19; out: EV_DONE | result bits (stored last)
  uint32_t evq[WS_EQ];        // owner | consumed | ticket, as the ring's meta
  uint32_t head, tail;        // ring tickets: handed to walker lanes / reserved by photon waves
  uint32_t ev_head, ev_tail;  // event tickets: held by event lanes / reserved by photon waves
  uint32_t alive;
  uint32_t abort_;            // the watchdog fired in this block: every wave leaves its loop
};
// event kinds (ev_code bits 16-18; the photon's free slot in bits 19-20)
constexpr uint32_t WS_EV_INTERACT = 1u, WS_EV_TAU = 2u, WS_EV_EMIT = 3u, WS_EV_FRESNEL = 4u;

// The lane scratch (global memory, KCold::lane_scratch, scenes with Fresnel interfaces or
// detectors): per photon lane the state of the rare program points that the photon's
// registers do not hold, structure of arrays over the launch's photon lanes
// (blockIdx.x * WS_NPL + pl). Doubles: the tauint2 entry's pos and dir (the bounce abort
// returns to them, inttau2.f90:313-315), the detector start point (startp, :125-131), the
// refraction's smallStepPos; then 32-bit words: the new layer and the bounce count. Only the
// photon's own lane touches its scratch (what reflect_refract's event lane needs and returns
// travels through LDS: the photon's free slot and its event slot).
enum : int { WX_ENTRY = 0, WX_START = 6, WX_SSP = 9, WX_ND = 12 };
enum : int { WXI_NEWL = 0, WXI_BOUNCES, WXI_N };
__host__ __device__ constexpr size_t ws_scratch_bytes(size_t lanes) {
  return lanes * (WX_ND * sizeof(double) + WXI_N * sizeof(uint32_t));
}

template <class S>
__device__ __forceinline__ void ws_count(S* sh, int c) {
  const uint64_t m = __ballot(1);
  if ((int)(threadIdx.x & 63) == __builtin_ctzll(m)) atomicAdd(&sh->wctr[threadIdx.x >> 6][c], (uint32_t)__popcll(m));
}

// the owner's view of its busy bits (another wave's walker clears them)
template <class S>
__device__ __forceinline__ uint32_t ws_busy(S* sh, uint32_t pl) {
  return __hip_atomic_load(&sh->busy[pl], __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP);
}

__device__ __forceinline__ uint32_t ws_load(uint32_t* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}


#ifdef SMCRT_ASM_MARKERS  // analysis builds (tools/isa_phases.py --kernel ws): region boundaries in the ISA
#define WS_MARK(i) asm volatile("; @@LPHASE " #i)
#else
#define WS_MARK(i) do {} while (0)
#endif
#ifdef SMCRT_DIAG
// Diagnostic builds (-DSMCRT_DIAG): wave-uniform tallies of the schedule in g_diag[20..39]
// (kernels.h), printed per launch by the host ([diag-ws]).
enum : int { WD_WITERS = 20, WD_WIDLE, WD_WBUSY, WD_WPEND, WD_PTRIPS, WD_PSLEEP, WD_PBLOCKED, WD_PWAIT, WD_P7,
             WD_P7LANES, WD_PIDLE, WD_ELANES, WD_PUSH, WD_PRODWAIT, WD_EITERS, WD_ELANESRUN, WD_PEVQ,
             // s_memtime ticks per region (WST): photon waves, walker waves, event waves
             WD_TP_FETCH, WD_TP_POLL, WD_TP_EVAL, WD_TP_P34, WD_TP_HAND, WD_TP_P56, WD_TP_P7, WD_TP_P8,
             WD_TW_CLAIM, WD_TW_IDLE, WD_TW_WALK, WD_TW_FIN, WD_TE_RUN, WD_TE_IDLE, WD_N };
static_assert(WD_N <= 64, "g_diag[64..] belongs to transport_kernel");
#define WSDIAG(i, v) (wd[(i) - WD_WITERS] += (uint64_t)(v))
#define WST(i)                                                \
  do {                                                        \
    const uint64_t now_ = __builtin_amdgcn_s_memtime();       \
    wd[(i) - WD_WITERS] += now_ - tprev;                      \
    tprev = now_;                                             \
  } while (0)
#else
#define WSDIAG(i, v) do {} while (0)
#define WST(i) do {} while (0)
#endif

// XF: scenes with Fresnel interfaces or detectors (their program points cost the photon waves
// registers, so the other scenes run an instantiation without them)
template <bool LDS_FACES, int GM, bool XF, uint32_t SL>
__global__ __launch_bounds__(WS_THREADS) __attribute__((amdgpu_waves_per_eu(4))) void ws_kernel(
    KParams K, const smcrt_sdf_node* __restrict__ nodes, const ProgOp* __restrict__ prog,
    const KCold* __restrict__ C) {
  using WsShared = WsSharedT<SL>;
  constexpr uint32_t WS_SLOTS = SL, WS_RING = WsShared::RING;
  __shared__ WsShared shm;
  WsShared* sh = &shm;
  const double eps = 1e-8;  // inttau2.f90:56
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
  for (uint32_t i = threadIdx.x; i < WS_NPL; i += WS_THREADS) {
    sh->busy[i] = 0;
    sh->lu[0][i] = sh->lu[1][i] = sh->lu[2][i] = 0;
  }
  for (uint32_t i = threadIdx.x; i < WS_RING; i += WS_THREADS) sh->meta[i] = 0;
  for (uint32_t i = threadIdx.x; i < WS_EQ; i += WS_THREADS) sh->evq[i] = 0;
  if (threadIdx.x == 0) {
    sh->head = sh->tail = 0;
    sh->ev_head = sh->ev_tail = 0;
    sh->alive = WS_PW;
    sh->abort_ = 0;
  }
  __syncthreads();

  uint32_t w_iters = 0, w_sdf = 0, w_dep = 0, hazards = 0;
  // per-lane tallies of the frequent counters, summed over the wave at the end (the rare ones
  // go through ws_count into the wave's LDS counters)
  uint32_t r_upd = 0, r_scat = 0, r_tau = 0, r_abs = 0;
#ifdef SMCRT_DIAG
  uint64_t wd[WD_N - WD_WITERS] = {};
  uint64_t tprev = __builtin_amdgcn_s_memtime();
#endif
  if (wv < WS_PW) {
    WS_MARK(1);
    // =================================================================== photon waves ======
    const bool test_kernel = (K.flags & SMCRT_FLAG_TEST_KERNEL) != 0;
    const bool records_on = (K.flags & SMCRT_FLAG_RECORD_PHOTONS) != 0 && C->records != nullptr;
    const uint32_t pl = threadIdx.x;  // photon lane (the photon waves come first)
#define WLU(f) (sh->lu[(f)][pl])
    // lean_margin (lean.h), per axis, corner coordinates; SMCRT_DEBUG_LEAN_MARGIN (tests only)
    // (the XF instantiation reads the box from KParams at the hand-out instead, see there)
    const double mf = (K.lean_debug & 3u) ? 0.0 : 2.0 * eps;
    const double mx0 = mf * (double)(K.nx + 2), my0 = mf * (double)(K.ny + 2), mz0 = mf * (double)(K.nz + 2);
    const double ex0 = 2.0 * K.xmax - mx0, ey0 = 2.0 * K.ymax - my0, ez0 = 2.0 * K.zmax - mz0;
    const bool defer_all = (K.lean_debug & 3u) == 2u;
    // SMCRT_DEBUG_DROP_EVENT (tests only): this lane's first event is marked queued, never queued
    bool drop_event = (K.lean_debug & 4u) && blockIdx.x == 0 && pl == 0;
    uint64_t wait_t0 = 0;  // (the watchdog: since when every live lane of this wave has waited)
    // the lane scratch (see WX_*): field f of this lane at X[f * xs]
    const size_t xs = (size_t)gridDim.x * WS_NPL;
    double* const X = XF ? C->lane_scratch + (size_t)blockIdx.x * WS_NPL + pl : nullptr;
    uint32_t* const XI = XF ? (uint32_t*)(C->lane_scratch + WX_ND * xs) + (size_t)blockIdx.x * WS_NPL + pl
                                         : nullptr;
    LeanPhoton P;
    P.st = ST_FETCH; P.f = LF_CELLS;
    P.pos = P.dir = v3(0.0, 0.0, 0.0);
    P.tau = P.taurun = P.d = P.minabs = 0.0;
    P.layer = P.xcell = P.ycell = P.zcell = 0;
    P.hop = P.loopc = P.seq = 0;
    P.rng.init(0);
    uint64_t chunk_base = 0;
    uint32_t chunk_left = 0;
    bool more = true;
    // tauint2 entry (inttau2.f90:48-60): the bounce abort's return point and the detector start
    auto t2_entry = [&]() {
      if constexpr (XF) {
        X[(WX_ENTRY + 0) * xs] = P.pos.x; X[(WX_ENTRY + 1) * xs] = P.pos.y; X[(WX_ENTRY + 2) * xs] = P.pos.z;
        X[(WX_ENTRY + 3) * xs] = P.dir.x; X[(WX_ENTRY + 4) * xs] = P.dir.y; X[(WX_ENTRY + 5) * xs] = P.dir.z;
        X[(WX_START + 0) * xs] = P.pos.x; X[(WX_START + 1) * xs] = P.pos.y; X[(WX_START + 2) * xs] = P.pos.z;
      }
    };

    // P8: arrive at the hop-loop head, inttau2.f90:61
    auto p8 = [&]() {
      if (!(P.f & (LF_REQ | LF_WAIT | LF_PEND)) && P.st == ST_H0) {
        if (!(P.taurun <= P.tau)) P.st = ST_T2END;
        else if (++P.hop > (uint32_t)MAX_HOP_ITERS) { P.set(LF_FAULT | LF_TFLAG); P.st = ST_T2END; }
        else P.set(LF_PEND);
      }
    };
    for (;; ++w_iters) {
      // ---- photon fetch (wave-aggregated work queue) ------------------------------------------
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
            sh->ev_pid[0][pl] = P.rng.pid_lo; sh->ev_pid[1][pl] = P.rng.pid_hi;  // (the event lanes' key)
            P.st = ST_EMIT;
          }
          chunk_base += take;
          chunk_left -= take;
          need = __ballot(P.st == ST_FETCH);
        }
        if (!more && P.st == ST_FETCH) P.st = ST_IDLE;
        const uint64_t live = __ballot(P.st != ST_IDLE);
        if (live == 0) break;  // (walkers finish this wave's segments)
      }
      WST(WD_TP_FETCH);
      // an event lane's results (see "Event waves"): the photon evaluates this trip
      if (P.has(LF_EVQ)) {
        const uint32_t code = __hip_atomic_load(&sh->ev_code[pl], __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP);
        if (code & EV_DONE) {
          P.clr(LF_EVQ);
          P.rng.draws = sh->ev_draws[pl];
          P.rng.cached = sh->ev_cached[pl];
          if (P.st == ST_EMIT) {  // the emitted photon (its tauint2 entry follows the layer search)
            P.pos = v3(sh->seg[P.seq][SG_OX][pl], sh->seg[P.seq][SG_OY][pl], sh->seg[P.seq][SG_OZ][pl]);
            P.dir = v3(sh->ev_dir[0][pl], sh->ev_dir[1][pl], sh->ev_dir[2][pl]);
            P.clr(LF_TFLAG);
            P.layer = (int32_t)(code & 0xFFFFu);
            // (emit's own cells: vox_of of the emitted position, transport.h emit)
            P.xcell = vox_of<GM>(P.pos.x, K.nx, K.xmax, K.inv2x, K.fex);
            P.ycell = vox_of<GM>(P.pos.y, K.ny, K.ymax, K.inv2y, K.fey);
            P.zcell = vox_of<GM>(P.pos.z, K.nz, K.zmax, K.inv2z, K.fez);
            P.set(LF_CELLS);
            if (code & EV_RUNAWAY) { P.set(LF_FAULT); P.st = ST_DONE; }  // (emission retries exhausted)
            else { P.st = ST_LAYER; P.set(LF_PEND); }
          } else if (XF && P.st == ST_F0) {  // reflect_refract's outcome (surfaces.f90:14-84)
            if (code & EV_RUNAWAY) {  // error stop :264-277
              P.set(LF_FAULT | LF_TFLAG); P.st = ST_T2END;
            } else if (code & EV_FR_REFLECT) {  // :304-316
              X[WX_START * xs] = P.pos.x; X[(WX_START + 1) * xs] = P.pos.y; X[(WX_START + 2) * xs] = P.pos.z;
              const uint32_t nb = XI[WXI_BOUNCES * xs] + 1u;
              XI[WXI_BOUNCES * xs] = nb;
              if (nb > 1000u) {  // :313-315: return without write-back, back to the tauint2 entry
                ws_count(sh, LC_BABORT);
                P.pos = v3(X[WX_ENTRY * xs], X[(WX_ENTRY + 1) * xs], X[(WX_ENTRY + 2) * xs]);
                P.dir = v3(X[(WX_ENTRY + 3) * xs], X[(WX_ENTRY + 4) * xs], X[(WX_ENTRY + 5) * xs]);
                P.st = ST_INTERACT;
              } else {
                P.dir = v3(sh->ev_dir[0][pl], sh->ev_dir[1][pl], sh->ev_dir[2][pl]);
                P.st = ST_H0;
                p8();
              }
            } else {  // refracted: cross with the new direction from smallStepPos, :284-303
              X[WX_SSP * xs] = sh->seg[P.seq][SG_DX][pl];
              X[(WX_SSP + 1) * xs] = sh->seg[P.seq][SG_DY][pl];
              X[(WX_SSP + 2) * xs] = sh->seg[P.seq][SG_DZ][pl];
              P.dir = v3(sh->ev_dir[0][pl], sh->ev_dir[1][pl], sh->ev_dir[2][pl]);
              P.layer = (int32_t)XI[WXI_NEWL * xs];
              P.st = ST_X1;
              P.set(LF_REQ | LF_SSP);
            }
          } else if (code & EV_ABSORB) {  // absorbed: recordWeight once the cells are in
            P.set(LF_TFLAG);
            P.st = ST_ABSORB;
          } else {  // scattered (or after an emission), then the tauint2 entry
            if (code & EV_RUNAWAY) P.set(LF_FAULT | LF_TFLAG);
            P.dir = v3(sh->ev_dir[0][pl], sh->ev_dir[1][pl], sh->ev_dir[2][pl]);
            P.tau = sh->ev_tau[pl];
            P.taurun = 0.0;
            P.hop = 0;
            P.st = ST_H0;
            t2_entry();
            p8();
          }
        }
      }
      WSDIAG(WD_PTRIPS, 1);
      WSDIAG(WD_PIDLE, __popcll(__ballot(P.st == ST_IDLE)));
      WSDIAG(WD_PWAIT, __popcll(__ballot(P.has(LF_WAIT))));
      WSDIAG(WD_PEVQ, __popcll(__ballot(P.has(LF_EVQ))));

      WST(WD_TP_POLL);
      // ---- EVAL: the SDF array at the photon's query point ------------------------------------
      const bool have = (P.f & (LF_PEND | LF_REQ | LF_WAIT)) == LF_PEND;
      EvalOut R;
      R.minabs = R.minv = R.va = R.vb = 0.0; R.maxloc = 0;
      if (__ballot(have)) {
        const bool mask_le = test_kernel && P.st == ST_LAYER;
        const V3 q = (P.st == ST_H1 || P.st == ST_G0) ? P.pos + smul(P.d, P.dir) : P.pos;
        R = eval_sdfs(nodes, prog, K.n_prog, q, mask_le, 0, 0);
        const bool counted = P.st == ST_H0 || P.st == ST_H1 || P.st == ST_H3 || P.st == ST_M1 || P.st == ST_G0;
        w_sdf += __popcll(__ballot(have && counted)) * (uint32_t)K.n_top;
        WSDIAG(WD_ELANES, __popcll(__ballot(have)));
        if (have) P.clr(LF_PEND);
      }

      WST(WD_TP_EVAL);
      // ---- P3: consume the EVAL result -----------------------------------------------------
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
            if (new_layer == P.layer && R.minabs < eps) {
              if (++P.loopc > (uint32_t)MAX_GLANCE_ITERS) { P.set(LF_FAULT | LF_TFLAG); P.st = ST_T2END; break; }
              P.d = P.d + eps;
              P.set(LF_PEND);
              break;
            }
            if (new_layer == 0) { P.set(LF_TFLAG); P.st = ST_T2END; break; }
            if (XF && props[P.layer - 1].n != props[new_layer - 1].n) {  // reflect_refract, :248
              // (to the event waves: F0/F1, the calcNormal taps and the surface, see below)
              XI[WXI_NEWL * xs] = (uint32_t)new_layer;
              P.st = ST_F0;
              break;
            }
            P.layer = new_layer;
            P.st = ST_X1;
            P.set(LF_REQ);
            break;
          }
          default:
            break;
        }
      }

      // ---- P4: a march step, :155-176 -------------------------------------------------------
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

      WST(WD_TP_P34);
      // ---- hand the new segments to the block's ring (update_grids entry, :401-415) ------------
      if (__ballot(P.has(LF_REQ))) {
        bool push = false, sync = false;
        V3 old = v3(0.0, 0.0, 0.0);
        const uint32_t slot = P.seq;
        if (P.has(LF_REQ) && !(ws_busy(sh, pl) & (1u << slot))) {  // (else: retry next trip)
          ++r_upd;
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
            // The XF instantiation takes the deferral box from KParams (scalar loads; in VGPRs it
            // spilled to scratch and was reloaded here): M3 181.0/181.6 vs 172.9/173.1 M photons/s.
            // The other one keeps it in VGPRs, where its register allocation is faster: M1 with
            // KParams 252.3 vs 257.5 M (profiles/r06_s7/ab_kparams_bounds.txt).
            constexpr bool KB = XF || SMCRT_WS_KBOUNDS_PLAIN;
            const double mx = KB ? K.lean_lo[0] : mx0, my = KB ? K.lean_lo[1] : my0, mz = KB ? K.lean_lo[2] : mz0;
            const double ex = KB ? K.lean_hi[0] : ex0, ey = KB ? K.lean_hi[1] : ey0, ez = KB ? K.lean_hi[2] : ez0;
            const bool inside = old.x >= mx && old.x <= ex && old.y >= my && old.y <= ey && old.z >= mz &&
                                old.z <= ez && e.x >= mx && e.x <= ex && e.y >= my && e.y <= ey && e.z >= mz &&
                                e.z <= ez;
            push = true;
            sync = !inside && !defer_all;
#if SMCRT_WS_START_CELLS
            sh->pcell[pl][slot] = lean_pack(ci, cj, ck);  // the start cell for the walker (slot free)
#endif
            if constexpr (GM != 2) {
              // faces k*2max/n and the cell of a point are rounded separately, so a start
              // within an ulp of a face may lie outside its own cell: the walk's first wall
              // distance is then negative, an error stop (:510-516) the photon must see. (GM 2:
              // both exact, never.) Such a start is synchronous.
              const bool in_cell = face<GM>(xf, ci - 1, K.fex) <= old.x && old.x <= face<GM>(xf, ci, K.fex) &&
                                   face<GM>(yf, cj - 1, K.fey) <= old.y && old.y <= face<GM>(yf, cj, K.fey) &&
                                   face<GM>(zf, ck - 1, K.fez) <= old.z && old.z <= face<GM>(zf, ck, K.fez);
              if (!in_cell) sync = true;
            }
          }
        }
        const uint64_t pm = __ballot(push);
        WSDIAG(WD_PUSH, __popcll(pm));
        WSDIAG(WD_PBLOCKED, __popcll(__ballot(P.has(LF_REQ))));
        if (pm) {
          const int first = __builtin_ctzll(pm);
          uint32_t base = 0;
          if (lane_id == first) base = atomicAdd(&sh->tail, (uint32_t)__popcll(pm));
          base = __builtin_amdgcn_readlane(base, first);
          if (push) {
            const uint32_t rank = __builtin_amdgcn_mbcnt_hi((uint32_t)(pm >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)pm, 0u));
            const uint32_t t = base + rank;
            const uint32_t ix = t & (WS_RING - 1);
            // the segment into its slot (free: its busy bit is clear), then the ring token
            double* const sg = &sh->seg[slot][0][pl];
            sg[SG_OX * WS_NPL] = old.x; sg[SG_OY * WS_NPL] = old.y; sg[SG_OZ * WS_NPL] = old.z;
            sg[SG_DX * WS_NPL] = P.dir.x; sg[SG_DY * WS_NPL] = P.dir.y; sg[SG_DZ * WS_NPL] = P.dir.z;
            sg[SG_LEN * WS_NPL] = P.d;
            atomicOr(&sh->busy[pl], 1u << slot);
            // the token's previous lap must have been consumed (see the header; no wait in practice)
            const uint32_t prev = t < WS_RING ? 0u : (ws_tick(t - WS_RING) | WS_CONSUMED);
            uint64_t t0 = 0;
            while (__hip_atomic_load(&sh->meta[ix], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) != prev) {
              WSDIAG(WD_PRODWAIT, 1);
              __builtin_amdgcn_s_sleep(1);
              if (!t0) t0 = __builtin_amdgcn_s_memrealtime();
              else if (watchdog_expired(C, t0, WDOG_RING)) break;  // (the run fails; the grid drains)
            }
            __hip_atomic_store(&sh->meta[ix], pl | (slot << 9) | (sync ? (1u << 11) : 0u) | ws_tick(t),
                               __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
            P.seq = P.seq + 1 == WS_SLOTS ? 0u : P.seq + 1;
            P.clr(LF_CELLS);
            if (sync) P.set(LF_WAIT);
          }
        }
      }

      WST(WD_TP_HAND);
      // ---- P5: a synchronous segment finished; after a segment: next program point ---------
      if (P.has(LF_WAIT) && !(ws_busy(sh, pl) & (1u << ((P.seq + WS_SLOTS - 1) % WS_SLOTS)))) {
        const unsigned long long w = sh->pcell[pl][(P.seq + WS_SLOTS - 1) % WS_SLOTS];
        P.xcell = lean_cell(w, 0); P.ycell = lean_cell(w, 1); P.zcell = lean_cell(w, 2);
        P.set(LF_CELLS);
        if (w & LEAN_TFLAG) P.set(LF_TFLAG);
        if (w & LEAN_FAULT) P.set(LF_FAULT);
        P.clr(LF_WAIT);
      }
      const bool free_ = !(P.f & (LF_REQ | LF_WAIT));
      if (free_ && (P.st == ST_H2 || P.st == ST_B0 || P.st == ST_X1)) {
        if (P.st == ST_X1) {  // :326-335 / :294-303 (pos = smallStepPos)
          P.taurun = P.taurun + P.d * props[P.layer - 1].kappa;
          if (XF && P.has(LF_SSP)) P.pos = v3(X[WX_SSP * xs], X[(WX_SSP + 1) * xs], X[(WX_SSP + 2) * xs]);
          else P.pos = P.pos + smul(P.d, P.dir);
          P.clr(LF_SSP);
        }
        if (XF && K.n_dets) {  // detectors, :125-131 / 195-201 (from startp to pos along dir)
          const V3 st = v3(X[WX_START * xs], X[(WX_START + 1) * xs], X[(WX_START + 2) * xs]);
          const double sep = pointsep(P.pos, st);
          X[WX_START * xs] = P.pos.x; X[(WX_START + 1) * xs] = P.pos.y; X[(WX_START + 2) * xs] = P.pos.z;
          const uint32_t hits = record_hits(K, C->det_bins, K.dets, K.det_off, st, P.dir, sep, P.layer, 1.0);
          if (hits) atomicAdd(&sh->wctr[wv][LC_HITS], hits);
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

      // ---- P6: tauint2 write-back checks, :341-362 ------------------------------------------
      if (free_ && P.st == ST_T2END) {
        if (fabs(P.pos.x) > K.xmax) P.set(LF_TFLAG);
        if (fabs(P.pos.y) > K.ymax) P.set(LF_TFLAG);
        if (fabs(P.pos.z) > K.zmax) P.set(LF_TFLAG);
        P.st = ST_INTERACT;
      }
      // the final cells of the photon's deferred segments, once they are all done
      if (!P.has(LF_CELLS) && (P.st == ST_ABSORB || (records_on && P.st == ST_DONE)) && ws_busy(sh, pl) == 0) {
        const unsigned long long w = sh->pcell[pl][(P.seq + WS_SLOTS - 1) % WS_SLOTS];
        P.xcell = lean_cell(w, 0); P.ycell = lean_cell(w, 1); P.zcell = lean_cell(w, 2);
        P.set(LF_CELLS);
      }
      // recordWeight of an absorbed photon (kernelsMod.f90:2202-2220) once its cells are in
      if (P.st == ST_ABSORB && P.has(LF_CELLS)) {
        if (P.xcell < 1 || P.xcell > K.nx || P.ycell < 1 || P.ycell > K.ny || P.zcell < 1 || P.zcell > K.nz)
          P.set(LF_FAULT);
        else if (C->absorb) atomic_add_nr(C->absorb + lin(K, P.xcell, P.ycell, P.zcell), 1.0);
        P.st = ST_DONE;
      }

      WST(WD_TP_P56);
      // ---- P7: the interactions and tauint2 entries go to the event waves -------------------
      {
        // (test_kernel runs keep the interactions, tauint2 entries and emissions in the photon
        // waves; a Fresnel event always goes to the event waves. Keeping them in the photon waves
        // for detector scenes too measured M5 34.3-34.9 vs 30.8-30.9 M photons/s, still short of
        // transport_kernel's 42.7-43.5, profiles/r05_ws/ab_m5_inline.txt)
        bool qev = free_ && !P.has(LF_EVQ) &&
                   ((!test_kernel && ((P.st == ST_INTERACT && !(P.f & (LF_TFLAG | LF_FAULT)) &&
                                     WLU(LL_INTER) + 1u <= (uint32_t)MAX_INTERACTIONS) ||
                                    P.st == ST_T2 || (P.st == ST_EMIT && !(ws_busy(sh, pl) & (1u << P.seq))))) ||
                    (XF && P.st == ST_F0 && !(ws_busy(sh, pl) & (1u << P.seq))));
        if (drop_event && qev) {  // (debug knob: a missed enqueue; the photon waits for nothing)
          drop_event = qev = false;
          __hip_atomic_store(&sh->ev_code[pl], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
          P.set(LF_EVQ);
        }
        const uint64_t qm = __ballot(qev);
        if (qm) {
          const int first = __builtin_ctzll(qm);
          uint32_t base = 0;
          if (lane_id == first) base = atomicAdd(&sh->ev_tail, (uint32_t)__popcll(qm));
          base = __builtin_amdgcn_readlane(base, first);
          if (qev) {
            const uint32_t t = base + __builtin_amdgcn_mbcnt_hi((uint32_t)(qm >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)qm, 0u));
            const uint32_t ix = t & (WS_EQ - 1);
            const uint32_t prev = t < WS_EQ ? 0u : (ws_tick(t - WS_EQ) | WS_CONSUMED);
            uint64_t t0 = 0;
            while (__hip_atomic_load(&sh->evq[ix], __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) != prev) {
              __builtin_amdgcn_s_sleep(1);  // (never in practice: one queued event per photon)
              if (!t0) t0 = __builtin_amdgcn_s_memrealtime();
              else if (watchdog_expired(C, t0, WDOG_EVENT_QUEUE)) break;
            }
            sh->ev_dir[0][pl] = P.dir.x; sh->ev_dir[1][pl] = P.dir.y; sh->ev_dir[2][pl] = P.dir.z;
            sh->ev_cached[pl] = P.rng.cached;
            sh->ev_draws[pl] = P.rng.draws;
            if (XF && P.st == ST_F0) {  // reflect_refract's inputs: pos and step in the free slot, the new layer
              sh->seg[P.seq][SG_OX][pl] = P.pos.x; sh->seg[P.seq][SG_OY][pl] = P.pos.y;
              sh->seg[P.seq][SG_OZ][pl] = P.pos.z; sh->seg[P.seq][SG_LEN][pl] = P.d;
              sh->ev_tau[pl] = (double)XI[WXI_NEWL * xs];
            }
            if (P.st == ST_EMIT) {  // kernelsMod.f90:1937-1945: a fresh packet
              P.clr(LF_FAULT); P.layer = 0;
              WLU(LL_STATUS) = 0; WLU(LL_NSCATT) = 0; WLU(LL_INTER) = 0;
              if constexpr (XF) XI[WXI_BOUNCES * xs] = 0;
            }
            sh->ev_code[pl] = (uint32_t)P.layer |
                              ((P.st == ST_INTERACT ? WS_EV_INTERACT
                                : (P.st == ST_T2 ? WS_EV_TAU : (P.st == ST_EMIT ? WS_EV_EMIT : WS_EV_FRESNEL))) << 16) |
                              (P.seq << 19);
            __hip_atomic_store(&sh->evq[ix], pl | ws_tick(t), __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
            P.set(LF_EVQ);
          }
        }
      }
      // ---- P7: the photon's other events, batched ---------------------------------------------
      {
        const bool ev = free_ && !P.has(LF_EVQ) &&
                        (P.st == ST_INTERACT || P.st == ST_T2 || P.st == ST_EMIT || P.st == ST_DONE);
        const uint64_t evm = __ballot(ev);
        const uint64_t busy = __ballot(P.st != ST_IDLE && P.st != ST_FETCH && !P.has(LF_EVQ));
        const uint32_t nev = __popcll(evm);
        // (test_kernel runs every event here; otherwise only emission, completion and the rare
        // terminal interactions are left, one or two per photon: run them once a few wait)
        const uint32_t batch = test_kernel ? (uint32_t)SMCRT_LEAN_EVENT_LANES : 4u;
        const bool run_ev = nev && (nev >= batch || evm == busy);
        WSDIAG(WD_P7, run_ev ? 1 : 0);
        WSDIAG(WD_P7LANES, run_ev ? nev : 0);
        if (run_ev) {
          if (ev && P.st == ST_INTERACT) {  // kernelsMod.f90:1958-1975 / 2126-2170
            if (P.f & (LF_TFLAG | LF_FAULT)) {
              P.st = ST_DONE;
            } else if (WLU(LL_INTER) + 1u > (uint32_t)MAX_INTERACTIONS) {
              ++WLU(LL_INTER);
              P.set(LF_FAULT); P.st = ST_DONE;
            } else {
              const double ran = P.rng.next(K.key0, K.key1);
              const TopProps pr = props[P.layer - 1];
              const bool sc = ran < pr.albedo;
              ++WLU(LL_INTER);
              if (!sc) {
                P.set(LF_TFLAG); WLU(LL_STATUS) = 1; ++r_abs;
                // recordWeight(packet, 1.0) at the photon's cells once they are in (ST_ABSORB)
                P.st = test_kernel ? ST_DONE : ST_ABSORB;
              } else {
                Lane L;  // scatter, photon.f90:1045-1103
                L.dir = P.dir; L.rng = P.rng; L.fault = false; L.tflag = false;
                scatter(K, L, pr.hgg);
                P.dir = L.dir; P.rng = L.rng;
                if (L.fault) P.set(LF_FAULT | LF_TFLAG);  // (renormalisation runaway)
                const uint32_t st = ++WLU(LL_NSCATT);
                ++r_scat;
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
                    WLU(LL_STATUS) = 4;
                  }
                }
                P.st = ST_T2;
              }
            }
          }
          if (ev && P.st == ST_T2) {  // tauint2 entry, inttau2.f90:48-60
            ++r_tau;
            t2_entry();
            P.tau = -det_log(P.rng.next(K.key0, K.key1));
            P.taurun = 0.0;
            P.hop = 0;
            P.st = ST_H0;  // arrives in P8
          }
          if (ev && P.st == ST_EMIT) {  // kernelsMod.f90:1937-1945
            P.clr(LF_FAULT); P.layer = 0;
            WLU(LL_STATUS) = 0; WLU(LL_NSCATT) = 0; WLU(LL_INTER) = 0;
            if constexpr (XF) XI[WXI_BOUNCES * xs] = 0;
            Lane L;
            L.rng = P.rng; L.xcell = L.ycell = L.zcell = 0; L.layer = 0; L.tflag = false;
            emit<GM, false>(K, C, L, 0u);
            if (!test_kernel) {
              int64_t tries = 0;
              while (cell_out(K, L)) {
                if (++tries > MAX_EMIT_TRIES) { P.set(LF_FAULT); break; }
                ws_count(sh, LC_RETRIES);
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
            if (P.has(LF_FAULT)) { WLU(LL_STATUS) = 3; ws_count(sh, LC_FAULTS); }
            else if (WLU(LL_STATUS) == 0) { WLU(LL_STATUS) = 2; ws_count(sh, LC_ESCAPED); }
            ws_count(sh, LC_PHOTONS);
            atomicAdd(&sh->wctr[wv][LC_DRAWS], P.rng.draws);
#ifdef SMCRT_DIAG
            if (C->done_time)
              C->done_time[(((uint64_t)P.rng.pid_hi << 32) | P.rng.pid_lo) - C->done_base] = __builtin_amdgcn_s_memrealtime();
#endif
            if (records_on) {
              const uint64_t pid = ((uint64_t)P.rng.pid_hi << 32) | P.rng.pid_lo;
              smcrt_photon_record* r = C->records + (pid - C->first_photon);
              r->pos[0] = P.pos.x; r->pos[1] = P.pos.y; r->pos[2] = P.pos.z;
              r->dir[0] = P.dir.x; r->dir[1] = P.dir.y; r->dir[2] = P.dir.z;
              r->weight = 1.0;
              r->cell[0] = P.xcell; r->cell[1] = P.ycell; r->cell[2] = P.zcell;
              r->layer = P.layer;
              r->nscatt = WLU(LL_NSCATT);
              r->bounces = XF ? XI[WXI_BOUNCES * xs] : 0u;
              r->draws = P.rng.draws;
              r->status = WLU(LL_STATUS);
            }
            P.clr(LF_TFLAG | LF_FAULT);
            P.st = ST_FETCH;
          }
        }
      }

      WST(WD_TP_P7);
      // ---- P8: arrive at the hop-loop head, :61 ---------------------------------------------
      p8();
      // every photon of the wave waits for a walker (a synchronous segment or a free slot):
      // yield the issue slots to the walkers
      if (__ballot(P.st != ST_IDLE && !(P.has(LF_WAIT) || P.has(LF_REQ) || P.has(LF_EVQ) ||
                                        (P.st == ST_ABSORB && !P.has(LF_CELLS)))) == 0) {
        WSDIAG(WD_PSLEEP, 1);
        __builtin_amdgcn_s_sleep(1);  // (0, 3: within noise)
        // the watchdog: an event, segment or slot that never comes (a lost enqueue) would hold
        // the wave here forever; past the budget the wave fails the run and leaves, and so does
        // every wave of the block (abort_)
        if (!wait_t0) {
          wait_t0 = __builtin_amdgcn_s_memrealtime();
        } else if (ws_load(&sh->abort_) || watchdog_expired(C, wait_t0, WDOG_PHOTON_WAVE)) {
          if (lane_id == 0) __hip_atomic_store(&sh->abort_, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
          break;
        }
      } else {
        wait_t0 = 0;
      }
      WST(WD_TP_P8);
    }
#undef WLU
    if (lane_id == 0) atomicSub(&sh->alive, 1u);  // (after this wave's last push, in its LDS order)
  } else if (wv < WS_PW + WS_EW) {
    WS_MARK(2);
    // The event wave issues first on its SIMD (s_setprio 3): one event wave serves the block's
    // 512 photons, and a photon waiting for its event waits for that wave's turn behind three
    // other waves. +4.5-5 % on M1 (243-246 -> 256-258 M photons/s); the photon waves at 1 or 2
    // changed nothing, the walkers at 1 lost 35 % (profiles/r05_ws/ab_prio.txt).
    __builtin_amdgcn_s_setprio(3);
    // =================================================================== event waves =======
    // An event lane holds a ticket of the event queue (as a walker lane holds a ring ticket),
    // and when the queue entry shows written(ticket) it runs the owner's event: the code of
    // P7 on the owner's direction, layer and Philox stream (kernelsMod.f90:1958-1975,
    // photon.f90:1045-1103, inttau2.f90:48-60), so the draws and results are the owner's own.
    bool pend = false;
    uint32_t tk = 0;
    for (;; ++w_iters) {
      const uint64_t cm = __ballot(!pend);
      if (cm) {
        const int first = __builtin_ctzll(cm);
        uint32_t base = 0;
        if (lane_id == first) base = atomicAdd(&sh->ev_head, (uint32_t)__popcll(cm));
        base = __builtin_amdgcn_readlane(base, first);
        if (!pend) {
          tk = base + __builtin_amdgcn_mbcnt_hi((uint32_t)(cm >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)cm, 0u));
          pend = true;
        }
      }
      bool run = false;
      uint32_t o = 0;
      if (pend) {
        const uint32_t ix = tk & (WS_EQ - 1);
        const uint32_t m = __hip_atomic_load(&sh->evq[ix], __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP);
        if ((m & WS_SEQ_MASK) == ws_tick(tk)) {
          o = m & 511u;
          __hip_atomic_store(&sh->evq[ix], ws_tick(tk) | WS_CONSUMED, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
          run = true;
          pend = false;
        }
      }
      if (!__ballot(run)) {
        // nothing queued: done once every photon wave has finished (the final tail is known), or
        // at once when the watchdog fired in this block
        if (ws_load(&sh->abort_)) break;
        if (ws_load(&sh->alive) == 0) {
          const uint32_t T = ws_load(&sh->ev_tail);
          if (pend && (int32_t)(tk - T) >= 0) pend = false;  // (a ticket nobody will write)
          if (!__ballot(pend) && (int32_t)(ws_load(&sh->ev_head) - T) >= 0) break;
        }
        __builtin_amdgcn_s_sleep(2);
        WST(WD_TE_IDLE);
        continue;
      }
      WSDIAG(WD_EITERS, 1);
      WSDIAG(WD_ELANESRUN, __popcll(__ballot(run)));
      if (run) {
        Rng rg;
        rg.pid_lo = sh->ev_pid[0][o]; rg.pid_hi = sh->ev_pid[1][o];
        rg.draws = sh->ev_draws[o]; rg.cached = sh->ev_cached[o];
        const uint32_t code = sh->ev_code[o];
        const int32_t layer = (int32_t)(code & 0xFFFFu);
        uint32_t res = 0;
        const uint32_t kind = (code >> 16) & 7u;
        bool tau_entry = kind == WS_EV_TAU;
        if (kind == WS_EV_EMIT) {  // kernelsMod.f90:1937-1945 (emit until the cell is in the grid)
          Lane L;
          L.rng = rg; L.xcell = L.ycell = L.zcell = 0; L.layer = 0; L.tflag = false;
          emit<GM, false>(K, C, L, 0u);
          int64_t tries = 0;
          bool fault = false;
          while (cell_out(K, L)) {
            if (++tries > MAX_EMIT_TRIES) { fault = true; break; }
            ws_count(sh, LC_RETRIES);
            emit<GM, false>(K, C, L, 0u);
          }
          rg = L.rng;
          const uint32_t es = (code >> 19) & 3u;  // the owner's free slot carries the position
          sh->seg[es][SG_OX][o] = L.pos.x; sh->seg[es][SG_OY][o] = L.pos.y; sh->seg[es][SG_OZ][o] = L.pos.z;
          sh->ev_dir[0][o] = L.dir.x; sh->ev_dir[1][o] = L.dir.y; sh->ev_dir[2][o] = L.dir.z;
          if (!fault && (K.flags & SMCRT_FLAG_RENDER_SOURCE) && C->emission)
            atomic_add_nr(C->emission + lin(K, L.xcell, L.ycell, L.zcell), 1.0);
          res = (fault ? EV_RUNAWAY : 0u) | ((uint32_t)L.layer & 0xFFFFu);
        } else if (XF && kind == WS_EV_FRESNEL) {
          // reflect_refract (inttau2.f90:248-328, surfaces.f90:14-84) for the owner: the ds pair
          // at pos and at smallStepPos, which SDF's normal, calcNormal's four taps (sdf_base.f90:
          // 166-190), the Fresnel draw, then the reflection (with the bounce count) or the
          // refraction's direction; the owner's pos and step come in its free slot (es), the new
          // layer in ev_tau; the bounce count and its abort are the owner's (photon waves)
          const uint32_t es = (code >> 19) & 3u;
          const V3 pos = v3(sh->seg[es][SG_OX][o], sh->seg[es][SG_OY][o], sh->seg[es][SG_OZ][o]);
          const V3 dir0 = v3(sh->ev_dir[0][o], sh->ev_dir[1][o], sh->ev_dir[2][o]);
          const int32_t new_layer = (int32_t)sh->ev_tau[o];
          const V3 ssp = pos + smul(sh->seg[es][SG_LEN][o], dir0);
          const EvalOut R0 = eval_sdfs(nodes, prog, K.n_prog, pos, false, new_layer, layer);
          const EvalOut R1 = eval_sdfs(nodes, prog, K.n_prog, ssp, false, new_layer, layer);
          const double ds_new = R0.va, ds_old = R0.vb, dn_new = R1.va, dn_old = R1.vb;
          int32_t ls = 0;
          if (dn_new < 0.0 && ds_new >= 0.0) ls = new_layer;
          else if (dn_old >= 0.0 && ds_old < 0.0) ls = layer;
          else if (dn_new < 0.0 && dn_old < 0.0) ls = new_layer;
          else if (ds_old >= 0.0 && dn_old >= 0.0) ls = layer;
          if (ls == 0) {
            res = EV_RUNAWAY;  // error stop :264-277
          } else {
            const double t = 1e-6;
            const double e1 = eval_sdfs(nodes, prog, K.n_prog, pos + mul(v3(1.0, -1.0, -1.0), t), false, ls, 0).va;
            const double e2 = eval_sdfs(nodes, prog, K.n_prog, pos + mul(v3(-1.0, -1.0, 1.0), t), false, ls, 0).va;
            const double e3 = eval_sdfs(nodes, prog, K.n_prog, pos + mul(v3(-1.0, 1.0, -1.0), t), false, ls, 0).va;
            const double e4 = eval_sdfs(nodes, prog, K.n_prog, pos + mul(v3(1.0, 1.0, 1.0), t), false, ls, 0).va;
            const V3 xyy = v3(1.0, -1.0, -1.0), yyx = v3(-1.0, -1.0, 1.0), yxy = v3(-1.0, 1.0, -1.0),
                     xxx = v3(1.0, 1.0, 1.0);
            const V3 nn = ((mul(xyy, e1) + mul(yyx, e2)) + mul(yxy, e3)) + mul(xxx, e4);
            const double ln = len(nn);
            const V3 N = v3(nn.x / ln, nn.y / ln, nn.z / ln);
            const double n1 = props[layer - 1].n, n2 = props[new_layer - 1].n;
            ws_count(sh, LC_FRES);
            const double Rf = fresnel(dir0, N, n1, n2);
            V3 dn;
            if (rg.next(K.key0, K.key1) <= Rf) {  // reflect :42-55, :304-316
              const double s2 = 2.0 * dot(N, dir0);
              dn = dir0 - smul(s2, N);
              ws_count(sh, LC_REFL);
              res = EV_FR_REFLECT;
            } else {  // refract :57-84 (pos = smallStepPos on the incoming direction, in the slot)
              sh->seg[es][SG_DX][o] = ssp.x; sh->seg[es][SG_DY][o] = ssp.y; sh->seg[es][SG_DZ][o] = ssp.z;
              const double eta = n1 / n2;
              V3 Nt = N;
              double c1 = dot(Nt, dir0);
              if (c1 < 0.0) c1 = -c1;
              else Nt = smul(-1.0, N);
              const double c2 = sqrt(1.0 - (eta * eta) * (1.0 - c1 * c1));
              dn = smul(eta, dir0) + smul(eta * c1 - c2, Nt);
            }
            sh->ev_dir[0][o] = dn.x; sh->ev_dir[1][o] = dn.y; sh->ev_dir[2][o] = dn.z;
          }
        } else if (kind == WS_EV_INTERACT) {  // kernelsMod.f90:1958-1975
          const TopProps pr = props[layer - 1];
          const double ran = rg.next(K.key0, K.key1);
          ++sh->lu[LL_INTER][o];
          if (!(ran < pr.albedo)) {
            sh->lu[LL_STATUS][o] = 1;
            ++r_abs;
            res = EV_ABSORB;
          } else {
            Lane L;  // scatter, photon.f90:1045-1103
            L.dir = v3(sh->ev_dir[0][o], sh->ev_dir[1][o], sh->ev_dir[2][o]);
            L.rng = rg; L.fault = false; L.tflag = false;
            scatter(K, L, pr.hgg);
            rg = L.rng;
            if (L.fault) res = EV_RUNAWAY;  // (renormalisation runaway: tflag and a fault)
            ++sh->lu[LL_NSCATT][o];
            ++r_scat;
            sh->ev_dir[0][o] = L.dir.x; sh->ev_dir[1][o] = L.dir.y; sh->ev_dir[2][o] = L.dir.z;
            tau_entry = true;
          }
        }
        if (tau_entry) {  // tauint2 entry, inttau2.f90:48-60
          ++r_tau;
          sh->ev_tau[o] = -det_log(rg.next(K.key0, K.key1));
        }
        sh->ev_draws[o] = rg.draws;
        sh->ev_cached[o] = rg.cached;
        __hip_atomic_store(&sh->ev_code[o], res | EV_DONE, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
      }
      WST(WD_TE_RUN);
    }
  } else {
    WS_MARK(10);
    // =================================================================== walker waves ======
    WalkSeg W;
    W.old = v3(0.0, 0.0, 0.0);
    W.sd = W.slen = 0.0;
    W.xcell = W.ycell = W.zcell = 0;
    W.dda_it = 0;
    W.seg = W.tflag = W.fault = false;
    V3 wdir = v3(0.0, 0.0, 0.0);
    // the direction's refined reciprocals (ieee_rcp_f64, the first half of the IEEE division
    // sequence, detmath.h), formed once per segment when it is taken instead of at every crossing
    V3 wrcp = v3(0.0, 0.0, 0.0);
    uint32_t wmeta = 0;
    BucketLog WB;
    WB.next = WB.end = 0;
    uint32_t overflow = 0;
    // A walker lane without a segment holds a ticket of its own (`tk`, taken with one
    // wave-aggregated LDS add on `head`, which may run ahead of `tail`) and checks its entry
    // once per iteration without waiting: when its meta word shows written(tk) (acquire: the
    // producer stores meta last, with release) the lane loads the fields and takes the segment.
    // (Loading the fields with the meta word, before the check, measured the same; a lane
    // holding the ticket of its next segment while it walks, -15 %: the segment waits behind the
    // lane's current one instead of going to an idle lane.) Each iteration walks SMCRT_WS_DDA
    // crossings of every held segment. A ticket no photon will
    // reserve (past the final tail once every photon wave has finished) is dropped.
    bool pend = false;
    uint32_t tk = 0;
    for (;; ++w_iters) {
      WS_MARK(11);
      const uint64_t cm = __ballot(!W.seg && !pend);
      if (cm) {
        const int first = __builtin_ctzll(cm);
        uint32_t base = 0;
        if (lane_id == first) base = atomicAdd(&sh->head, (uint32_t)__popcll(cm));
        base = __builtin_amdgcn_readlane(base, first);
        if (!W.seg && !pend) {
          tk = base + __builtin_amdgcn_mbcnt_hi((uint32_t)(cm >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)cm, 0u));
          pend = true;
        }
      }
      if (pend) {
        const uint32_t ix = tk & (WS_RING - 1);
        const uint32_t m = __hip_atomic_load(&sh->meta[ix], __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP);
        if ((m & WS_SEQ_MASK) == ws_tick(tk)) {
          __hip_atomic_store(&sh->meta[ix], ws_tick(tk) | WS_CONSUMED, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
          const double* const sg = &sh->seg[(m >> 9) & 3u][0][m & 511u];
          const V3 o = v3(sg[SG_OX * WS_NPL], sg[SG_OY * WS_NPL], sg[SG_OZ * WS_NPL]);
          const V3 dd = v3(sg[SG_DX * WS_NPL], sg[SG_DY * WS_NPL], sg[SG_DZ * WS_NPL]);
          const double l = sg[SG_LEN * WS_NPL];
          W.old = o;
          wdir = dd;
          wrcp = v3(ieee_rcp_f64(dd.x), ieee_rcp_f64(dd.y), ieee_rcp_f64(dd.z));
          W.slen = l;
          wmeta = m;
          // the start cell, as the photon computed it from the same start (update_grids :401-415)
#if SMCRT_WS_START_CELLS
          {  // (written by the photon into the slot's cell word before the token)
            const unsigned long long cw = sh->pcell[m & 511u][(m >> 9) & 3u];
            W.xcell = lean_cell(cw, 0); W.ycell = lean_cell(cw, 1); W.zcell = lean_cell(cw, 2);
          }
#else
          W.xcell = cell_of<GM>(W.old.x, K.nx, K.xmax, K.inv2x, K.fex);
          W.ycell = cell_of<GM>(W.old.y, K.ny, K.ymax, K.inv2y, K.fey);
          W.zcell = cell_of<GM>(W.old.z, K.nz, K.zmax, K.inv2z, K.fez);
#endif
          W.sd = 0.0; W.dda_it = 0;
          W.seg = true; W.tflag = false; W.fault = false;
          pend = false;
        }
      }
      const uint64_t am = __ballot(W.seg);
      WSDIAG(WD_WITERS, 1);
      WSDIAG(WD_WIDLE, am ? 0 : 1);
      WSDIAG(WD_WBUSY, __popcll(am));
      WSDIAG(WD_WPEND, __popcll(__ballot(pend)));
      WST(WD_TW_CLAIM);
      if (!am) {
        // nothing to walk: once every photon wave has finished, the final tail is known and the
        // tickets past it are never reserved; done when no lane holds an earlier one (or at once
        // when the watchdog fired in this block)
        if (ws_load(&sh->abort_)) break;
        if (ws_load(&sh->alive) == 0) {
          const uint32_t T = ws_load(&sh->tail);
          if (pend && (int32_t)(tk - T) >= 0) pend = false;  // (a ticket nobody will write)
          if (!__ballot(pend) && (int32_t)(ws_load(&sh->head) - T) >= 0) break;
        }
        __builtin_amdgcn_s_sleep(2);
        WST(WD_TW_IDLE);
        continue;
      }
      // ---- one crossing of every held segment (dda_step: wall_dist, deposit, update_pos) ----
      WS_MARK(12);
#pragma unroll
      for (int k = 0; k < SMCRT_WS_DDA; ++k) {
        if (k > 0 && !__ballot(W.seg)) break;
        bool dep = false;
        uint32_t vox = 0;
        double val = 0.0;
        if (W.seg) dda_step_r<GM>(K, W, wdir, wrcp, xf, yf, zf, dep, vox, val, 1.0);
        w_dep += __popcll(__ballot(dep));
        WS_MARK(13);
        emit_bucketed(K, C, WB, dep, vox, val, overflow, bstate);
      }
      WS_MARK(14);
      WST(WD_TW_WALK);
      // a finished segment: its cells and flags to the owner's slot, then the slot is free
      if ((am >> lane_id & 1ull) && !W.seg) {
        const uint32_t owner = wmeta & 511u, slot = (wmeta >> 9) & 3u;
        const bool sync = (wmeta & (1u << 11)) != 0;
        if (!sync && (W.tflag || W.fault)) ++hazards;  // cannot happen (lean.h); counted as a fault
        sh->pcell[owner][slot] = lean_pack(W.xcell, W.ycell, W.zcell) | (W.tflag ? LEAN_TFLAG : 0ull) |
                                 (W.fault ? LEAN_FAULT : 0ull);
        // (release: the slot's cells before the bit; the owner reads the bit with acquire)
        __hip_atomic_fetch_and(&sh->busy[owner], ~(1u << slot), __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
      }
      WST(WD_TW_FIN);
    }
    WS_MARK(15);
    close_buckets(K, C, WB, w_dep - overflow, overflow);
  }
  WS_MARK(16);
  // ---- per-wave counters (each role adds its own) ------------------------------------------
  {
    unsigned long long* const counters = C->counters;
    const uint32_t hz = wave_sum_u32(hazards);
    const uint32_t n_upd = wave_sum_u32(r_upd), n_scat = wave_sum_u32(r_scat), n_tau = wave_sum_u32(r_tau),
                   n_abs = wave_sum_u32(r_abs);
    if (lane_id == 0) {
      if (hz) {  // reported: smcrt_kernel_times.lean_hazards, and SMCRT_CTR_FAULTS
        atomicAdd(C->dep_ctl + 5, hz);
        atomicAdd(C->lean_hazards, (unsigned long long)hz);
      }
      if (C->dep_ctl && n_upd) atomicAdd(C->dep_ctl + 6, n_upd);  // segments
      if (counters) {
        const uint32_t* c = sh->wctr[wv];
        const uint32_t v[SMCRT_NCOUNTERS] = {c[LC_PHOTONS], c[LC_RETRIES], n_scat,        n_abs,          w_sdf,
                                             w_dep,         n_upd,         n_tau,          c[LC_FRES],     c[LC_REFL],
                                             c[LC_BABORT],  c[LC_FAULTS] + hz, c[LC_DRAWS], c[LC_HITS],   c[LC_ESCAPED],
                                             w_iters};
        for (int i = 0; i < SMCRT_NCOUNTERS; ++i)
          if (v[i]) atomicAdd(counters + i, (unsigned long long)v[i]);
      }
      double* const nscatt = C->nscatt;
      if (nscatt && n_scat) atomic_add_nr(nscatt, (double)n_scat);
    }
  }
#ifdef SMCRT_DIAG
  if (lane_id == 0)
    for (int i = 0; i < WD_N - WD_WITERS; ++i)
      if (wd[i]) atomicAdd(&::g_diag[WD_WITERS + i], (unsigned long long)wd[i]);
#endif
  __syncthreads();  // every wave of the block is done depositing
  close_block_buckets(K, C, bstate);
}

}  // namespace smcrt
