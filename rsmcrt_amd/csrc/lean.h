// lean.h — the lean path: the transport of simple scenes with the voxel walk decoupled from the
// photon. This header holds its shared definitions (the photon and walker state, the flags, the
// segment-safety margin below, computed per axis at the top of ws_kernel, or on the host into
// KParams::lean_lo/hi for the XF instantiation); the kernel is ws_kernel (ws.h), which runs the photons, their
// events and the walks in separate waves of a block. (Rounds 3-4 ran it as lean_kernel, whose
// waves were both photons and walkers; ws_kernel replaced it in round 5.)
//
// Same path as transport_kernel (noBiasPropagation kernelsMod.f90:1901-1976 -> tauint2
// inttau2.f90:15-364 -> update_grids :367-465), same arithmetic, same results bit for bit,
// for scenes of few tops with no survival bias, path-length deposition into buckets
// (deposit.h) and the three plain sources. Scenes with Fresnel interfaces (reflect_refract,
// :248-328, in the event waves) take it by default through ws_kernel's XF instantiation (round
// 5); scenes with detectors run the XF instantiation only with SMCRT_LEAN=1 (record_hits at
// every segment end in the photon waves: transport_kernel measured faster on M5).
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
// So the photon hands the segment to a ring of segments (LDS) and goes on; walker lanes take
// segments from the ring, any lane any segment, refilled after every crossing, so the walk runs
// on nearly full waves and a march step costs one trip.
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
// error stops need a start outside its own cell (faces and cells rounded separately: a start
// within an ulp of a face, e.g. a source on a mid-plane of a grid whose spacing is not a power
// of two; ws.h makes every such segment synchronous), NaNs or an overshoot of one ulp at an
// exact tie of two wall distances
// (probability ~1e-16 per crossing); a deferred segment that nevertheless ends in one (a
// "hazard": its photon has gone on as if the walk had stayed inside) is counted in
// SMCRT_CTR_FAULTS and in smcrt_kernel_times.lean_hazards, never silently dropped. The debug
// knob SMCRT_DEBUG_LEAN_MARGIN=0/all provokes hazards to test that accounting.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "transport.h"
#include "deposit.h"

namespace smcrt {

// test_kernel runs (ws.h: their events stay in the photon waves) run a wave's events once this
// many lanes wait for one (or nothing else is left); 20 measured best in round 3
// (profiles/r03_s3/lean_tune_ab.txt)
#define SMCRT_LEAN_EVENT_LANES 20
constexpr uint32_t ST_ABSORB = 40;  // absorbed; recordWeight waits for the photon's cells
constexpr int LEAN_CELL_BITS = 20;               // per axis in a packed cell word (cell + 1)
constexpr uint64_t LEAN_CELL_MASK = (1ull << LEAN_CELL_BITS) - 1;
constexpr uint64_t LEAN_TFLAG = 1ull << 60, LEAN_FAULT = 1ull << 61;

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

// The photon (registers). Counters and rare per-photon fields are in LDS.
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
  LF_EVQ = 256u,   // the photon's event is queued for the event waves (ws.h)
  LF_SSP = 512u,   // a refraction: X1 moves to the smallStepPos kept in the lane scratch (ws.h)
};
// event results (ws.h ev_code; the low 16 bits carry an emitted photon's layer); a Fresnel
// event reports a fault (EV_RUNAWAY), a reflection or (neither) a refraction
enum : uint32_t { EV_DONE = 1u << 31, EV_ABSORB = 1u << 30, EV_RUNAWAY = 1u << 29, EV_FR_REFLECT = 1u << 28 };
struct LeanPhoton {
  V3 pos, dir;
  Rng rng;
  double tau, taurun, d, minabs;
  int32_t layer;
  int32_t xcell, ycell, zcell;  // valid with LF_CELLS
  uint32_t hop, loopc, st, seq;  // seq: the slot of the next segment
  uint32_t f;                    // LF_* flags
  __device__ __forceinline__ bool has(uint32_t b) const { return (f & b) != 0; }
  __device__ __forceinline__ void set(uint32_t b) { f |= b; }
  __device__ __forceinline__ void clr(uint32_t b) { f &= ~b; }
};

enum : int { LL_INTER = 0, LL_NSCATT, LL_STATUS };  // per-photon fields in LDS (ws.h lu)

}  // namespace smcrt
