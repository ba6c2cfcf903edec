// smcrt.hip — host side of the transport kernels (kernels.h, instantiated by kinst.hip),
// the fold kernels (deposit.h) and the C ABI of include/smcrt.h.
//
// Replaces the body of run_MCRT (/root/reference/src/kernelsMod.f90:1790-1898): the
// OpenMP `parallel do` over photons becomes a persistent grid whose waves pull 64 photon
// indices at a time from a device work queue; the `!$omp atomic` tally updates
// (inttau2.f90:426,433; kernelsMod.f90:2198,2218; detector_base.f90:156,228) become
// no-return fp64 atomics into device-resident tallies; the nscatt `reduction(+:...)` and
// the debug counters are reduced across each wave and added once per wave.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <string>
#include <functional>
#include <vector>

#define SMCRT_FOLD_KERNELS  // deposit.h: the fold kernels are defined in this translation unit
#include "../../include/smcrt.h"
#include "scene_internal.h"
#include "transport.h"
#include "deposit.h"
#include "hosterr.h"

using namespace smcrt;

#include "kernel_ptrs.h"


// The top-level SDF containing each point: maxloc(ds, mask=ds<0), 0 outside every SDF
// (kernelsMod.f90:589-595, 1027-1032: the escape function's launch-cell test). One lane per
// point; the SDF program is walked wave-uniformly as in the transport kernel.
__global__ __launch_bounds__(256) void classify_kernel(const smcrt_sdf_node* __restrict__ nodes,
                                                       const ProgOp* __restrict__ prog, int32_t n_prog,
                                                       const double* __restrict__ pts, int64_t n, int32_t* layer) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i - threadIdx.x < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t j = i < n ? i : n - 1;  // whole waves walk the program together
    const V3 q = v3(pts[3 * j], pts[3 * j + 1], pts[3 * j + 2]);
    const EvalOut r = eval_sdfs<true>(nodes, prog, n_prog, q, false, 0, 0);
    if (i < n) layer[i] = r.maxloc;
  }
}

// ------------------------------------------------------------------ host side ------
thread_local std::string smcrt::g_last_error;

namespace {

int fail(int code, const std::string& msg) { return set_error(code, msg); }

#define HIPCHK(expr)                                                                              \
  do {                                                                                            \
    hipError_t e_ = (expr);                                                                       \
    if (e_ != hipSuccess)                                                                         \
      return fail(SMCRT_ERR_HIP, std::string(#expr " failed: ") + hipGetErrorString(e_));         \
  } while (0)

template <class T>
int dalloc(T** p, size_t n) {
  if (n == 0) n = 1;
  hipError_t e = hipMalloc((void**)p, n * sizeof(T));
  if (e == hipErrorOutOfMemory) return fail(SMCRT_ERR_OOM, "hipMalloc: out of memory");
  if (e != hipSuccess) return fail(SMCRT_ERR_HIP, std::string("hipMalloc: ") + hipGetErrorString(e));
  return SMCRT_OK;
}

}  // namespace

// Record-log slots (and internal launch streams) per scene: launches whose pools are small
// enough run up to MAX_SLOTS deep, so long-tailed launches overlap more than pairwise.
constexpr int MAX_SLOTS = 4;
#ifndef SMCRT_DEEP_SLOT_GIB
#define SMCRT_DEEP_SLOT_GIB 24
#endif
constexpr uint64_t DEEP_SLOT_BYTES = (uint64_t)SMCRT_DEEP_SLOT_GIB << 30;  // a slot pool at most this large: MAX_SLOTS slots

struct smcrt_scene {
  int device = 0;
  int n_nodes = 0, n_top = 0, n_dets = 0;
  smcrt_grid grid{};
  int64_t det_total = 0;
  std::vector<smcrt_sdf_node> h_nodes;
  std::vector<int32_t> h_top;
  std::vector<TopProps> h_props;
  std::vector<smcrt_detector> h_dets;
  std::vector<int64_t> h_det_off;
  smcrt_sdf_node* d_nodes = nullptr;
  ProgOp* d_prog = nullptr;
  int n_prog = 0;
  int coop_lanes = 0;
  double* d_ctab = nullptr;  // the cooperative EVAL's primitive table (transport.h), or NULL
  // far-field march (far.h): KParams::fm_err / fm_step, 0 when the scene does not qualify;
  // the running total of its steps is d_queue[MAX_SLOTS + 1]
  double fm_err = 0.0, fm_step = 0.0;
  unsigned long long far_reported = 0;
  // a top model has a model or modifier among its children, or a top is a modifier: only the
  // general instantiation evaluates composites below the top level (geometry.h node_value), so
  // such scenes always run it: with many tops its COOP variant (cooperative and culled EVALs,
  // round 4), else the serial EVAL; never the lean kernel
  bool nested = false;
  // the fold's workgroup run time: d_queue[MAX_SLOTS + 2] running total (s_memrealtime ticks at
  // wall_khz), reported per CU (one bk_reduce workgroup fills a CU)
  unsigned long long fold_ticks_reported = 0;
  int wall_khz = 100000, n_cus = 256;
  // exact SDF culling (cull.h): grid + lists + the always-evaluated program, one allocation
  CullGrid* d_cull = nullptr;
  void* d_cull_data = nullptr;
  double cull_mean_list = 0.0;
  double inv2[3] = {0.0, 0.0, 0.0};
  int grid_mode = 0;  // transport_kernel<*, GM>: 1 = every 2*max a power of two, 2 = and every n too
  int32_t fe[3] = {0, 0, 0};
  TopProps* d_props = nullptr;
  double* d_faces = nullptr;
  smcrt_detector* d_dets = nullptr;
  int64_t* d_det_off = nullptr;
  unsigned long long* d_queue = nullptr;  // work-queue heads: [i] internal stream i, [MAX_SLOTS] caller stream
  // SMCRT_FLAG_OVERLAP: launches rotate over n_slots internal streams (lstream), so the next
  // launches' blocks fill the CUs their predecessors' tails leave idle
  hipStream_t lstream[MAX_SLOTS] = {};
  hipEvent_t lev[MAX_SLOTS] = {};  // the last launch on lstream[i] is done
  hipEvent_t ev_in = nullptr;              // the caller's work before an overlapped call
  bool lpending[MAX_SLOTS] = {};
  int lturn = 0;
  KCold* d_cold = nullptr;  // launch parameters: COLD_PER_STREAM ring slots per launch stream
  uint64_t cold_seq[MAX_SLOTS + 1] = {};
  // tallies owned by the scene for the synchronous smcrt_run
  double* d_grids = nullptr;  // jmean | absorb | emission
  double* d_small = nullptr;  // det bins | nscatt | moments(24)
  unsigned long long* d_counters = nullptr;
  smcrt_photon_record* d_records = nullptr;
  size_t records_cap = 0;
  hipStream_t stream = nullptr;
  int grid_blocks = 0;
  int grid_blocks_x = 0;  // the XSRC (general emitter) instantiation
  int grid_blocks_ws = 0;    // ws_kernel (ws.h): the lean path with photon, event and walker waves
  int ws_slots = 3;          // its segment slots per photon: 3, or 2 when 3 do not fit the LDS (ws.h)
  // ws_kernel's lane scratch (ws.h WX_*) for scenes with Fresnel interfaces or detectors: one
  // region per launch stream (queue index, launch_one), lscratch_stride bytes apart
  double* d_lscratch = nullptr;
  size_t lscratch_stride = 0;
  // the lean path (ws_kernel) serves this scene: a few tops, bucketed deposition, axes below
  // 2^20 cells, its LDS fits (SMCRT_LEAN=0 keeps transport_kernel)
  bool lean_ok = false;
  // deferred lean-kernel segments that ended in tflag or an error stop (lean.h "hazards"):
  // running total d_queue[MAX_SLOTS + 3], reported by smcrt_scene_kernel_times and counted in
  // SMCRT_CTR_FAULTS by the kernel
  unsigned long long hazards_reported = 0;
  // SMCRT_DEBUG_LEAN_MARGIN (tests only): 1 = "0", no margin; 2 = "all", every segment that
  // starts in the grid is deferred (forces hazards on escaping segments)
  uint32_t lean_debug = 0;
  int64_t lean_launches = 0;  // since the last smcrt_scene_kernel_times
#ifdef SMCRT_DIAG
  unsigned long long* d_done = nullptr;  // per-photon completion times of the last run (SMCRT_DIAG_DONE)
  uint64_t n_done = 0;
#endif
  // SMCRT_LEAN: -1 automatic, 0 off, 1 forced. (Rounds 3-4 chose lean_kernel only up to 5.5
  // voxel crossings per segment: long walks were cheaper in one lane. ws_kernel's walker waves
  // take them at any length: M0, 8.2 crossings per segment, 54.9 vs 43.4-44.2 M photons/s on
  // transport_kernel, profiles/r05_ws/ab_m0.txt.)
  int lean_mode = -1;
  // source spectrum tables of the last general-emitter run (srcplan.h), device copy
  std::vector<double> h_spec;
  double* d_spec = nullptr;
  size_t spec_cap = 0;
  bool lds_faces = false;
  size_t face_bytes = 0;
  uint32_t hist_tiles = 0;  // fused tile histogram in the transport kernel (0: bin_hist kernel)
  bool bucketed = false;    // records go straight into per-tile buckets (deposit.h); else sorted path
  // binned jmean deposition (deposit.h)
  uint32_t n_tiles = 0;
  // Two record-log slots, used by alternate launches: the fold of launch k (on fstream)
  // reads its slot while launch k+1's transport kernel fills the other.
  // record-log slots in use (2, or MAX_SLOTS when a slot's pool is small: ensure_pool), and as
  // many internal launch streams; a launch's fold frees its slot
  int n_slots = 2;
  unsigned long long* d_pool[MAX_SLOTS] = {};  // record log, cap records
  unsigned long long* d_sorted = nullptr;  // tile-sorted records (folds are serial on fstream)
  // bucketed path: per slot the tile of each bucket id (bucket fills use d_chunk_fill, the
  // per-tile bucket counts d_bin_counts); shared by the serial folds: ids in tile order
  uint32_t* d_bucket_tile[MAX_SLOTS] = {};
  uint32_t* d_order = nullptr;
  uint32_t* d_chunk_fill[MAX_SLOTS] = {};
  uint32_t* d_dep_ctl[MAX_SLOTS] = {};  // [0] chunks taken [1] overflow [2] pieces [3] records
  uint32_t* d_tile_count = nullptr;  // n_tiles
  uint32_t* d_tile_start = nullptr;  // n_tiles
  uint32_t* d_bin_counts[MAX_SLOTS] = {};  // [n_tiles][BIN_BLOCKS]
  hipStream_t fstream = nullptr;  // the deposit folds
  hipEvent_t ev_t = nullptr;      // a transport launch finished (fstream waits on it)
  hipEvent_t ev_f[MAX_SLOTS] = {};  // the fold of slot i finished
  bool f_pending[MAX_SLOTS] = {};
  int slot = 0, last_slot = -1;
  size_t scatter_lds = 0;
  Piece* d_pieces = nullptr;
  uint64_t pool_chunks = 0, max_pieces = 0;
  double rpp_est = 1024.0;           // deposit records per photon, refined from past launches
  bool rpp_measured = false;
  uint32_t* h_ctl = nullptr;         // pinned copies of dep_ctl, 8 words per slot ([4] = photons)
  hipEvent_t ctl_ev[MAX_SLOTS] = {};
  bool ctl_pending[MAX_SLOTS] = {};
  bool force_atomic = false;  // SMCRT_DEPOSIT=atomic
  uint64_t pool_cap_chunks = 0;  // SMCRT_POOL_CAP (records; tests of pool exhaustion): 0 = none
  // smcrt_scene_kernel_times: event quads (before / after transport on the launch stream,
  // before / after the deposit fold on fstream) of the launches since the last harvest
  bool timing = false;
  std::vector<hipEvent_t> tev;
  size_t tev_used = 0;
  double t_transport = 0.0, t_deposit = 0.0;
  int64_t t_launches = 0;
  std::mutex mu;
};

constexpr size_t MAX_TIMED = 256;
constexpr uint64_t COLD_PER_STREAM = 16;
constexpr uint64_t COLD_SLOTS = COLD_PER_STREAM * (MAX_SLOTS + 1);  // a ring per launch stream
constexpr uint32_t MAX_FUSED_HIST_TILES = 512;  // 8 KiB of LDS per block for the wave histograms
// Record pool: record indices in the bin kernels are 32-bit, so at most 2^32 - 2^28 records
// (30 GiB, plus the same again for the sorted copy) per launch; a launch that would need more
// is split into sub-batches. POOL_SLACK covers the spread of records per photon between
// batches; a launch that still overflows folds the excess with atomics (exact, slower).
constexpr uint64_t MAX_POOL_RECORDS = (1ull << 32) - (1ull << 28);
constexpr double POOL_SLACK = 1.15;
constexpr uint64_t CALIB_PHOTONS = 1ull << 18;  // first binned launch of a scene above this size  // in-flight launches per scene before a KCold slot is reused  // launches kept before the events are harvested

// Fold the recorded event triples into the sums (waits for them).
static hipError_t harvest_times(smcrt_scene* s) {
  for (size_t i = 0; i < s->tev_used; ++i) {
    hipEvent_t* e = &s->tev[4 * i];
    hipError_t err = hipEventSynchronize(e[1]);
    if (err == hipSuccess) err = hipEventSynchronize(e[3]);
    if (err != hipSuccess) return err;
    float a = 0.f, b = 0.f;
    if ((err = hipEventElapsedTime(&a, e[0], e[1])) != hipSuccess) return err;
    if ((err = hipEventElapsedTime(&b, e[2], e[3])) != hipSuccess) return err;
    s->t_transport += a; s->t_deposit += b; s->t_launches += 1;
  }
  s->tev_used = 0;
  return hipSuccess;
}

// The transport kernel instantiation for this scene (LDS faces? power-of-two grid?).
// Scenes with many tops (coop_lanes > 0) get an instantiation with the cooperative tail EVAL
// and culling; it costs registers (scratch spills), so small scenes never pay for it. With the
// general emitter (XSRC: other sources, batched origins, composites below the top level) that
// is transport_kernel<.., true, true> (round 4; before, such scenes ran the serial EVAL).
static const void* transport_fn(const smcrt_scene* s, bool xsrc) {
  // (the general emitter with the COOP machinery is instantiated with faces in device memory
  // only: three kernels instead of six, the library's build time, for the rare scenes that run
  // it; transport_lds follows)
  return transport_kernel_ptr(s->lds_faces, s->grid_mode, xsrc, s->coop_lanes > 0);
}

// the lean path's dynamic LDS (ws_kernel): staged props + faces, then the block's bucket words
static size_t lean_lds(const smcrt_scene* s) {
  return (s->lds_faces ? s->face_bytes : 0) + (size_t)2 * s->n_tiles * sizeof(uint32_t);
}

// Dynamic LDS of the transport kernel: staged props + faces, detector start points, then the
// deposit words (4 wave tile histograms, or the block's bucket words), then the coop table.
static size_t transport_lds(const smcrt_scene* s, uint32_t dep_words, bool xsrc) {
  const bool ctab = s->d_ctab && s->coop_lanes > 0;  // the COOP instantiations stage it
  const bool faces = s->lds_faces && !(xsrc && s->coop_lanes > 0);  // (transport_fn)
  return (faces ? s->face_bytes : 0) + (s->n_dets ? 3 * 256 * sizeof(double) : 0) +
         (size_t)dep_words * sizeof(uint32_t) + (ctab ? CTAB_DOUBLES * sizeof(double) : 0);
}
// 32-bit LDS words of a block's deposit state (deposit.h): a tile histogram per wave, or one
// 64-bit bucket word per tile shared by the block.
static uint32_t dep_words(const smcrt_scene* s) { return s->bucketed ? 2 * s->n_tiles : 4 * s->hist_tiles; }

// ---- the watchdog (transport.h watchdog_expired): d_queue[MAX_SLOTS + 4] holds the first
// expired wait of the scene's launches, site | (block + 1) << 8
constexpr double DEFAULT_WATCHDOG_MS = 2000.0;  // a wait past 2 s of wall clock is a lost wake-up
static uint32_t* watchdog_word(smcrt_scene* s) { return (uint32_t*)(s->d_queue + MAX_SLOTS + 4); }
static const char* watchdog_site(uint32_t site) {
  switch (site) {
    case WDOG_PHOTON_WAVE: return "ws_kernel photon wave (every live lane waited for an event, a segment or a slot)";
    case WDOG_RING: return "ws_kernel ring producer (the token word's previous lap was never consumed)";
    case WDOG_EVENT_QUEUE: return "ws_kernel event-queue producer (the entry's previous lap was never consumed)";
    case WDOG_BUCKET: return "bucket wait (deposit.h: the pending claim never rebased the tile word)";
    default: return "unknown site";
  }
}
// After the scene's launches have finished: SMCRT_ERR_DEVICE_FAULT naming the first expired
// wait, if any (the word is cleared, so the scene stays usable).
static int take_watchdog(smcrt_scene* s) {
  uint32_t w = 0;
  HIPCHK(hipMemcpy(&w, watchdog_word(s), sizeof w, hipMemcpyDeviceToHost));
  if (!w) return SMCRT_OK;
  HIPCHK(hipMemset(watchdog_word(s), 0, sizeof w));
  return fail(SMCRT_ERR_DEVICE_FAULT, std::string("watchdog: a wait exceeded SMCRT_WATCHDOG_MS at ") +
                                          watchdog_site(w & 0xFFu) + " in block " + std::to_string((w >> 8) - 1u) +
                                          "; the run's tallies are incomplete");
}

static TopProps make_props(const smcrt_sdf_node& nd) {
  TopProps p;  // init_mono, opticalProperties.f90:107-125
  p.kappa = nd.mus + nd.mua;
  if (nd.flags & SMCRT_NODE_ALBEDO_UNGUARDED) p.albedo = nd.mus / p.kappa;  // updateSpectral :198-199
  else p.albedo = (nd.mua < 1e-9) ? 1.0 : nd.mus / p.kappa;
  p.hgg = nd.hgg;
  p.n = nd.n;
  return p;
}

extern "C" {

int smcrt_abi_version(void) { return SMCRT_ABI_VERSION; }

const char* smcrt_last_error(void) { return g_last_error.c_str(); }

int smcrt_device_count(int32_t* count) {
  if (!count) return fail(SMCRT_ERR_INVALID_ARG, "count is NULL");
  int n = 0;
  hipError_t e = hipGetDeviceCount(&n);
  if (e == hipErrorNoDevice) n = 0;
  else if (e != hipSuccess) return fail(SMCRT_ERR_HIP, hipGetErrorString(e));
  *count = n;
  return SMCRT_OK;
}

void smcrt_scene_destroy(smcrt_scene* s) {
  if (!s) return;
  (void)hipSetDevice(s->device);
  if (s->stream) (void)hipStreamSynchronize(s->stream);
  if (s->fstream) (void)hipStreamSynchronize(s->fstream);
  void* ptrs[] = {s->d_lscratch, s->d_ctab, s->d_nodes, s->d_prog, s->d_props, s->d_faces, s->d_dets, s->d_det_off, s->d_spec,
                  s->d_queue, s->d_cold, s->d_grids, s->d_small, s->d_counters, s->d_records,
                  s->d_sorted, s->d_tile_count, s->d_tile_start, s->d_pieces, s->d_order, s->d_cull, s->d_cull_data};
  for (int i = 0; i < MAX_SLOTS; ++i) {
    void* per[] = {s->d_pool[i], s->d_chunk_fill[i], s->d_dep_ctl[i], s->d_bin_counts[i], s->d_bucket_tile[i]};
    for (void* p : per)
      if (p) (void)hipFree(p);
    if (s->ctl_ev[i]) (void)hipEventDestroy(s->ctl_ev[i]);
    if (s->ev_f[i]) (void)hipEventDestroy(s->ev_f[i]);
  }
  if (s->ev_t) (void)hipEventDestroy(s->ev_t);
  for (int i = 0; i < MAX_SLOTS; ++i) {
    if (s->lstream[i]) (void)hipStreamSynchronize(s->lstream[i]);
    if (s->lev[i]) (void)hipEventDestroy(s->lev[i]);
    if (s->lstream[i]) (void)hipStreamDestroy(s->lstream[i]);
  }
  if (s->ev_in) (void)hipEventDestroy(s->ev_in);
  if (s->fstream) (void)hipStreamDestroy(s->fstream);
  for (hipEvent_t e : s->tev) (void)hipEventDestroy(e);
  if (s->h_ctl) (void)hipHostFree(s->h_ctl);
  for (void* p : ptrs)
    if (p) (void)hipFree(p);
  if (s->stream) (void)hipStreamDestroy(s->stream);
  delete s;
}

int smcrt_scene_create(const smcrt_sdf_node* nodes, int32_t n_nodes, const int32_t* top, int32_t n_top,
                       const smcrt_grid* grid, const smcrt_detector* dets, int32_t n_dets, int32_t device,
                       smcrt_scene** out) {
  g_last_error.clear();
  if (!out) return fail(SMCRT_ERR_INVALID_ARG, "out is NULL");
  *out = nullptr;
  if (!nodes || n_nodes < 1 || !top || n_top < 1 || !grid || n_dets < 0 || (n_dets > 0 && !dets))
    return fail(SMCRT_ERR_INVALID_ARG, "bad scene arguments");
  if (grid->nx < 1 || grid->ny < 1 || grid->nz < 1 || !(grid->xmax > 0) || !(grid->ymax > 0) ||
      !(grid->zmax > 0))
    return fail(SMCRT_ERR_INVALID_ARG, "grid dimensions must be positive");
  if ((uint64_t)grid->nx * (uint64_t)grid->ny * (uint64_t)grid->nz >= (1ull << 32))
    return fail(SMCRT_ERR_UNSUPPORTED, "grids of 2^32 or more voxels are not supported");
  for (int32_t i = 0; i < n_nodes; ++i) {
    const smcrt_sdf_node& nd = nodes[i];
    if (nd.kind < SMCRT_SDF_SPHERE || nd.kind > SMCRT_SDF_DISPLACEMENT)
      return fail(SMCRT_ERR_INVALID_ARG, "node " + std::to_string(i) + ": unknown SDF kind");
    if (nd.kind == SMCRT_SDF_MODEL) {
      if (nd.n_children < 1 || nd.first_child < 0 || nd.first_child + nd.n_children > n_nodes)
        return fail(SMCRT_ERR_INVALID_ARG, "model node " + std::to_string(i) + ": bad child range");
      if (nd.op < SMCRT_OP_UNION || nd.op > SMCRT_OP_INTERSECTION)
        return fail(SMCRT_ERR_INVALID_ARG, "model node " + std::to_string(i) + ": bad CSG op");
    } else if (composite_kind(nd.kind)) {  // a modifier wraps exactly one node
      if (nd.n_children != 1 || nd.first_child < 0 || nd.first_child >= n_nodes)
        return fail(SMCRT_ERR_INVALID_ARG, "modifier node " + std::to_string(i) + ": needs exactly one child");
      if (nd.kind == SMCRT_SDF_DISPLACEMENT && nd.param[0] != (double)SMCRT_DISP_SINE)
        return fail(SMCRT_ERR_INVALID_ARG, "displacement node " + std::to_string(i) + ": unknown function");
    }
  }
  // models and modifiers nested at most PROG_MAX_DEPTH levels (geometry.h node_value); this
  // also rejects a composite that contains itself
  {
    std::function<int(int32_t, int)> depth_ok = [&](int32_t idx, int lvl) -> int {
      const smcrt_sdf_node& nd = nodes[idx];
      if (!composite_kind(nd.kind)) return 1;
      if (lvl >= PROG_MAX_DEPTH) return 0;
      for (int32_t c = 0; c < nd.n_children; ++c)
        if (!depth_ok(nd.first_child + c, lvl + 1)) return 0;
      return 1;
    };
    for (int32_t i = 0; i < n_top; ++i)
      if (top[i] >= 0 && top[i] < n_nodes && !depth_ok(top[i], 0))
        return fail(SMCRT_ERR_UNSUPPORTED, "top " + std::to_string(i) + ": models/modifiers nested more than " +
                                               std::to_string(PROG_MAX_DEPTH) + " levels deep are not supported");
  }
  for (int32_t i = 0; i < n_top; ++i)
    if (top[i] < 0 || top[i] >= n_nodes) return fail(SMCRT_ERR_INVALID_ARG, "top index out of range");
  for (int32_t i = 0; i < n_dets; ++i) {
    if (dets[i].kind < SMCRT_DET_CIRCLE || dets[i].kind > SMCRT_DET_FIBRE || dets[i].nbins < 1)
      return fail(SMCRT_ERR_INVALID_ARG, "bad detector " + std::to_string(i));
  }
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) return fail(SMCRT_ERR_NO_DEVICE, "no HIP device");
  if (device < 0 || device >= ndev) return fail(SMCRT_ERR_INVALID_ARG, "device ordinal out of range");

  smcrt_scene* s = new smcrt_scene();
  s->device = device;
  s->n_nodes = n_nodes;
  s->n_top = n_top;
  s->n_dets = n_dets;
  s->grid = *grid;
  s->h_nodes.assign(nodes, nodes + n_nodes);
  s->h_top.assign(top, top + n_top);
  for (int32_t i = 0; i < n_top; ++i) s->h_props.push_back(make_props(nodes[top[i]]));
  s->h_dets.assign(dets, dets + n_dets);
  s->h_det_off.assign((size_t)n_dets + 1, 0);
  for (int32_t i = 0; i < n_dets; ++i) {
    const int64_t nb = dets[i].nbins;
    s->h_det_off[i + 1] = s->h_det_off[i] + (dets[i].kind == SMCRT_DET_CAMERA ? nb * nb : nb);
  }
  s->det_total = s->h_det_off[n_dets];
  // voxel faces, grid.f90:147-157: (i-1)*2*max/n; zface has nz+2 entries
  std::vector<double> faces;
  for (int32_t i = 0; i < grid->nx + 1; ++i) faces.push_back((double)i * 2.0 * grid->xmax / (double)grid->nx);
  for (int32_t i = 0; i < grid->ny + 1; ++i) faces.push_back((double)i * 2.0 * grid->ymax / (double)grid->ny);
  for (int32_t i = 0; i < grid->nz + 2; ++i) faces.push_back((double)i * 2.0 * grid->zmax / (double)grid->nz);

  auto cleanup_fail = [&](int code) {
    std::string msg = g_last_error;
    smcrt_scene_destroy(s);
    g_last_error = msg;
    return code;
  };
  if (hipSetDevice(device) != hipSuccess) return cleanup_fail(fail(SMCRT_ERR_HIP, "hipSetDevice failed"));
  int st;
  // flatten the SDF array into one evaluation program (eval_model fold order)
  std::vector<ProgOp> prog;
  auto translate_only = [&](int32_t idx) -> int32_t {  // 3x3 part of the column-major transform is I
    const double* t = nodes[idx].transform;
    return t[0] == 1.0 && t[1] == 0.0 && t[2] == 0.0 && t[4] == 0.0 && t[5] == 1.0 && t[6] == 0.0 &&
           t[8] == 0.0 && t[9] == 0.0 && t[10] == 1.0;
  };
  std::vector<int32_t> top_first((size_t)n_top + 1, 0);
  for (int32_t i = 0; i < n_top; ++i) {
    const smcrt_sdf_node& nd = nodes[top[i]];
    top_first[i] = (int32_t)prog.size();
    if (!composite_kind(nd.kind)) {
      prog.push_back(ProgOp{top[i], PROG_TOP, i + 1, 0, 0.0, translate_only(top[i]), 0});
    } else if (nd.kind != SMCRT_SDF_MODEL) {  // a top-level modifier: one PROG_SUB op (geometry.h node_value)
      prog.push_back(ProgOp{top[i], PROG_TOP | PROG_SUB, i + 1, 0, 0.0, 0, 0});
    } else {
      // eval_model's left fold, children in order; a child model or modifier is one PROG_SUB
      // op (geometry.h node_value)
      for (int32_t c = 0; c < nd.n_children; ++c) {
        const int32_t ci = nd.first_child + c;
        const bool sub = composite_kind(nodes[ci].kind);
        prog.push_back(ProgOp{ci, (c == 0 ? PROG_CHILD_FIRST : PROG_CHILD) | (sub ? PROG_SUB : 0),
                              c == nd.n_children - 1 ? i + 1 : 0, nd.op, nd.k, sub ? 0 : translate_only(ci), 0});
      }
    }
  }
  s->n_prog = (int)prog.size();
  top_first[n_top] = s->n_prog;
  for (int32_t i = 0; i <= n_top; ++i)  // eval_sdfs_coop's table of each top's first op
    prog.push_back(ProgOp{top_first[i], PROG_TOP, 0, 0, 0.0, 0, 0});
  // A sparse wave evaluates its lanes' SDF arrays one lane at a time across the wave when
  // that is cheaper than the serial per-lane chain over all n_top tops (transport.h).
  for (const ProgOp& op : prog) s->nested = s->nested || (op.action & PROG_SUB) != 0;
  int32_t coop_min = 8;  // (SMCRT_COOP_MIN_TOPS: the fewest tops that get the COOP instantiation)
  if (const char* cm = std::getenv("SMCRT_COOP_MIN_TOPS")) coop_min = std::max(1, std::atoi(cm));
  s->coop_lanes = n_top >= coop_min ? std::max(1, std::min(16, n_top / ((n_top + 63) / 64 + 3))) : 0;
  if (const char* cl = std::getenv("SMCRT_COOP_LANES"))  // (experiments: the sparse-wave threshold)
    if (s->coop_lanes > 0) s->coop_lanes = std::max(1, std::min(64, std::atoi(cl)));
  // The cooperative EVAL's LDS table: at most 64 tops, none of them a model (transport.h).
  // SMCRT_COOP_TAB=0 keeps the global-memory cooperative EVAL.
  std::vector<double> ctab;
  {
    const char* ct = std::getenv("SMCRT_COOP_TAB");
    bool ok = s->coop_lanes > 0 && n_top <= 64 && !(ct && std::string(ct) == "0");
    for (int32_t i = 0; ok && i < n_top; ++i) ok = !composite_kind(nodes[top[i]].kind);
    if (ok) {
      ctab.assign(CTAB_DOUBLES, 0.0);
      for (int32_t i = 0; i < n_top; ++i) {
        const smcrt_sdf_node& nd = nodes[top[i]];
        for (int r = 0; r < 12; ++r) ctab[r * 64 + i] = nd.transform[r];
        for (int r = 0; r < 8; ++r) ctab[(12 + r) * 64 + i] = nd.param[r];
        ctab[20 * 64 + i] = (double)nd.kind + (translate_only(top[i]) ? 16.0 : 0.0);
      }
    }
  }
  // exact culling of the SDF array for many-top scenes (cull.h); SMCRT_CULL=0 turns it off
  CullHost cull;
  {
    const char* ce = std::getenv("SMCRT_CULL");
    const double gh[3] = {grid->xmax, grid->ymax, grid->zmax};
    if (s->coop_lanes > 0 && !(ce && std::string(ce) == "0")) cull = build_cull(nodes, n_nodes, top, n_top, gh);
  }
  // The far-field march and glance (far.h) need every top 1-Lipschitz (exact-distance
  // primitives under translation-only transforms), a full EVAL that yields a certificate (the
  // cooperative LDS table or the culled EVAL) and a bound on the computed values' error: a few
  // ulps of the largest operand, taken here as 2^-44 of the scene's extent. SMCRT_FAR_MARCH=0
  // turns them off.
  if (!ctab.empty() || cull.enabled) {
    const char* fe = std::getenv("SMCRT_FAR_MARCH");
    bool fm = !(fe && std::string(fe) == "0");
    double ext = grid->xmax + grid->ymax + grid->zmax + 1.0;
    double scale = 0.0;
    // A top qualifies if it is such a primitive, or (round 4) a model of qualifying children
    // folded with union, intersection, subtraction or smooth union (min/max of 1-Lipschitz
    // values is 1-Lipschitz, and so is the polynomial smooth minimum: its partials are 1 - h^2/2
    // and h^2/2), at most 4 model levels deep so the fold's few roundings per level stay far
    // below the bound. The near top of a certificate is still a lone sphere or box (far.h).
    // m accumulates the operand magnitudes the error bound scales with.
    std::function<bool(int32_t, int, double&)> far_ok = [&](int32_t idx, int lvl, double& m) -> bool {
      const smcrt_sdf_node& nd = nodes[idx];
      if (nd.kind == SMCRT_SDF_MODEL) {
        const bool op_ok = nd.op == SMCRT_OP_UNION || nd.op == SMCRT_OP_INTERSECTION || nd.op == SMCRT_OP_SUBTRACTION ||
                           (nd.op == SMCRT_OP_SMOOTH_UNION && nd.k > 0.0 && std::isfinite(nd.k));
        if (lvl >= 4 || !op_ok || nd.n_children < 1) return false;
        if (nd.op == SMCRT_OP_SMOOTH_UNION) m = std::max(m, nd.k);
        for (int32_t c = 0; c < nd.n_children; ++c)
          if (!far_ok(nd.first_child + c, lvl + 1, m)) return false;
        return true;
      }
      const int32_t kd = nd.kind;
      if (!translate_only(idx) || !(kd == SMCRT_SDF_SPHERE || kd == SMCRT_SDF_BOX || kd == SMCRT_SDF_TORUS ||
                                    kd == SMCRT_SDF_SEGMENT || kd == SMCRT_SDF_CAPSULE))
        return false;
      double mm = std::fabs(nd.transform[3]) + std::fabs(nd.transform[7]) + std::fabs(nd.transform[11]);
      for (int r = 0; r < 8; ++r) mm += std::fabs(nd.param[r]);
      if (!std::isfinite(mm)) return false;
      m = std::max(m, mm);
      return true;
    };
    for (int32_t i = 0; fm && i < n_top; ++i) {
      double m = 0.0;
      fm = far_ok(top[i], 0, m);
      scale = std::max(scale, m);
    }
    fm = fm && std::isfinite(ext);
    if (fm) {
      s->fm_err = std::ldexp(scale + ext, -44);
      s->fm_step = std::ldexp(scale + ext, -48);
    }
  }
  // n*p/(2*max) may be computed as n*p*inv exactly when 2*max is a power of two
  const double maxes[3] = {grid->xmax, grid->ymax, grid->zmax};
  for (int a = 0; a < 3; ++a) {
    int ex = 0;
    const double m = std::frexp(2.0 * maxes[a], &ex);
    s->inv2[a] = (m == 0.5 && std::isfinite(1.0 / (2.0 * maxes[a]))) ? 1.0 / (2.0 * maxes[a]) : 0.0;
  }
  if ((st = dalloc(&s->d_nodes, n_nodes)) || (st = dalloc(&s->d_prog, prog.size())) || (st = dalloc(&s->d_props, n_top)) ||
      (st = dalloc(&s->d_faces, faces.size())) || (st = dalloc(&s->d_dets, std::max(1, n_dets))) ||
      (st = dalloc(&s->d_det_off, (size_t)n_dets + 1)) || (st = dalloc(&s->d_queue, MAX_SLOTS + 5)) ||
      (st = dalloc(&s->d_cold, COLD_SLOTS)) ||
      (st = dalloc(&s->d_counters, SMCRT_NCOUNTERS)) ||
      (st = dalloc(&s->d_small, (size_t)s->det_total + 1 + 24)))
    return cleanup_fail(st);
  hipError_t e = hipSuccess;
  if (e == hipSuccess) e = hipMemset(s->d_queue, 0, (MAX_SLOTS + 5) * sizeof(unsigned long long));
  if (e == hipSuccess) e = hipMemcpy(s->d_nodes, nodes, sizeof(smcrt_sdf_node) * n_nodes, hipMemcpyHostToDevice);
  if (e == hipSuccess) e = hipMemcpy(s->d_prog, prog.data(), sizeof(ProgOp) * prog.size(), hipMemcpyHostToDevice);
  if (e == hipSuccess && !ctab.empty()) {
    if ((st = dalloc(&s->d_ctab, ctab.size()))) return cleanup_fail(st);
    e = hipMemcpy(s->d_ctab, ctab.data(), sizeof(double) * ctab.size(), hipMemcpyHostToDevice);
  }
  if (e == hipSuccess) e = hipMemcpy(s->d_props, s->h_props.data(), sizeof(TopProps) * n_top, hipMemcpyHostToDevice);
  if (e == hipSuccess) e = hipMemcpy(s->d_faces, faces.data(), sizeof(double) * faces.size(), hipMemcpyHostToDevice);
  if (e == hipSuccess && n_dets)
    e = hipMemcpy(s->d_dets, dets, sizeof(smcrt_detector) * n_dets, hipMemcpyHostToDevice);
  if (e == hipSuccess)
    e = hipMemcpy(s->d_det_off, s->h_det_off.data(), sizeof(int64_t) * (n_dets + 1), hipMemcpyHostToDevice);
  if (e == hipSuccess) e = hipStreamCreateWithFlags(&s->stream, hipStreamNonBlocking);
  for (int i = 0; i < MAX_SLOTS && e == hipSuccess; ++i) {
    e = hipStreamCreateWithFlags(&s->lstream[i], hipStreamNonBlocking);
    if (e == hipSuccess) e = hipEventCreateWithFlags(&s->lev[i], hipEventDisableTiming);
  }
  if (e == hipSuccess) e = hipEventCreateWithFlags(&s->ev_in, hipEventDisableTiming);
  if (e != hipSuccess) return cleanup_fail(fail(SMCRT_ERR_HIP, std::string("scene upload: ") + hipGetErrorString(e)));
  if (cull.enabled) {  // [ProgOp always | u32 off | u32 list | double lb | float elb], each 16-B aligned
    std::vector<ProgOp> pa;
    for (int32_t t : cull.always)
      for (int32_t ip = top_first[t]; ip < top_first[t + 1]; ++ip) pa.push_back(prog[ip]);
    auto al = [](size_t b) { return (b + 15) & ~(size_t)15; };
    const size_t b_pa = al(pa.size() * sizeof(ProgOp)), b_off = al(cull.off.size() * 4),
                 b_list = al(std::max<size_t>(1, cull.list.size()) * 4), b_lb = al(cull.lb.size() * 8),
                 b_elb = al(std::max<size_t>(1, cull.elb.size()) * 4);
    std::vector<unsigned char> blob(b_pa + b_off + b_list + b_lb + b_elb, 0);
    std::memcpy(blob.data(), pa.data(), pa.size() * sizeof(ProgOp));
    std::memcpy(blob.data() + b_pa, cull.off.data(), cull.off.size() * 4);
    std::memcpy(blob.data() + b_pa + b_off, cull.list.data(), cull.list.size() * 4);
    std::memcpy(blob.data() + b_pa + b_off + b_list, cull.lb.data(), cull.lb.size() * 8);
    std::memcpy(blob.data() + b_pa + b_off + b_list + b_lb, cull.elb.data(), cull.elb.size() * 4);
    if ((st = dalloc((unsigned char**)&s->d_cull_data, blob.size())) || (st = dalloc(&s->d_cull, 1)))
      return cleanup_fail(st);
    unsigned char* base = (unsigned char*)s->d_cull_data;
    CullGrid G;
    for (int a = 0; a < 3; ++a) { G.lo[a] = cull.lo[a]; G.n[a] = cull.n[a]; }
    G.cell = cull.cell;
    G.inv_cell = 1.0 / cull.cell;
    G.n_prog_always = (int32_t)pa.size();
    G.prog_always = base;
    G.off = (const uint32_t*)(base + b_pa);
    G.list = (const uint32_t*)(base + b_pa + b_off);
    G.lb = (const double*)(base + b_pa + b_off + b_list);
    G.elb = (const float*)(base + b_pa + b_off + b_list + b_lb);
    e = hipMemcpy(s->d_cull_data, blob.data(), blob.size(), hipMemcpyHostToDevice);
    if (e == hipSuccess) e = hipMemcpy(s->d_cull, &G, sizeof G, hipMemcpyHostToDevice);
    if (e != hipSuccess) return cleanup_fail(fail(SMCRT_ERR_HIP, std::string("cull upload: ") + hipGetErrorString(e)));
    s->cull_mean_list = cull.mean_list;
    if (std::getenv("SMCRT_CULL_LOG"))  // diagnostics
      std::fprintf(stderr, "[cull] %d tops, %zu always, %d x %d x %d cells of %.4g, %.1f tops per cell\n",
                   n_top, cull.always.size(), cull.n[0], cull.n[1], cull.n[2], cull.cell, cull.mean_list);
  }
  {  // binned deposition state (deposit.h)
    const uint64_t nv = (uint64_t)grid->nx * grid->ny * grid->nz;
    const uint64_t tiles = (nv + TILE_VOXELS - 1) / TILE_VOXELS;
    s->n_tiles = (tiles <= MAX_TILES && nv < 0xFFFFFFFFull) ? (uint32_t)tiles : 0;
    const char* fa = std::getenv("SMCRT_DEPOSIT");
    s->force_atomic = fa && std::string(fa) == "atomic";
    if (const char* pc = std::getenv("SMCRT_POOL_CAP"))
      s->pool_cap_chunks = std::max<uint64_t>(1, std::strtoull(pc, nullptr, 10) / CHUNK_RECORDS);
    if (s->n_tiles) {
      if ((st = dalloc(&s->d_tile_count, s->n_tiles)) || (st = dalloc(&s->d_tile_start, s->n_tiles)))
        return cleanup_fail(st);
      for (int i = 0; i < MAX_SLOTS; ++i)
        if ((st = dalloc(&s->d_dep_ctl[i], 8)) || (st = dalloc(&s->d_bin_counts[i], (size_t)s->n_tiles * BIN_BLOCKS)))
          return cleanup_fail(st);
      s->scatter_lds = scatter_lds_bytes(s->n_tiles);
      if (hipFuncSetAttribute((const void*)bin_scatter, hipFuncAttributeMaxDynamicSharedMemorySize,
                              (int)s->scatter_lds) != hipSuccess)
        return cleanup_fail(fail(SMCRT_ERR_HIP, "bin_scatter LDS attribute"));
      // The fold stream gets the highest priority (SMCRT_FOLD_PRIO=0: normal). At the default
      // priority HIP maps it onto one of the process's shared hardware queues (4 by default),
      // behind a launch stream's persistent transport kernels, and a fold waited ~60 ms for
      // them; a high-priority stream has its own queue, and its
      // workgroups are dispatched first when a CU frees.
      const char* fp = std::getenv("SMCRT_FOLD_PRIO");
      int prio_least = 0, prio_greatest = 0;
      const bool fold_prio = !(fp && fp[0] == '0') &&
                             hipDeviceGetStreamPriorityRange(&prio_least, &prio_greatest) == hipSuccess &&
                             prio_greatest != prio_least;
      bool ok = hipHostMalloc((void**)&s->h_ctl, 8 * MAX_SLOTS * sizeof(uint32_t)) == hipSuccess &&
                hipEventCreateWithFlags(&s->ev_t, hipEventDisableTiming) == hipSuccess &&
                (fold_prio ? hipStreamCreateWithPriority(&s->fstream, hipStreamNonBlocking, prio_greatest)
                           : hipStreamCreateWithFlags(&s->fstream, hipStreamNonBlocking)) == hipSuccess;
      for (int i = 0; ok && i < MAX_SLOTS; ++i)
        ok = hipEventCreateWithFlags(&s->ctl_ev[i], hipEventDisableTiming) == hipSuccess &&
             hipEventCreateWithFlags(&s->ev_f[i], hipEventDisableTiming) == hipSuccess;
      if (!ok) return cleanup_fail(fail(SMCRT_ERR_HIP, "pinned/event/stream allocation failed"));
      std::memset(s->h_ctl, 0, 8 * MAX_SLOTS * sizeof(uint32_t));
    }
  }
  int per_cu = 0, cus = 0;
  s->face_bytes = faces.size() * sizeof(double) + sizeof(TopProps) * (size_t)n_top;
  s->lds_faces = s->face_bytes <= 40960;  // stage props + voxel faces in LDS when they fit
  {
    const char* fh = std::getenv("SMCRT_FUSED_HIST");
    const bool fuse = !(fh && std::string(fh) == "0");
    // SMCRT_DEPOSIT=sorted (or a disabled fused histogram) keeps the sorted record path
    const char* dm = std::getenv("SMCRT_DEPOSIT");
    const bool sorted = (dm && std::string(dm) == "sorted") || !fuse;
    s->bucketed = !sorted && s->n_tiles > 0 && s->n_tiles <= MAX_DIRECT_TILES;
    s->hist_tiles = (!s->bucketed && fuse && s->n_tiles > 0 && s->n_tiles <= MAX_FUSED_HIST_TILES) ? s->n_tiles : 0;
  }
  {
    const bool p2 = s->inv2[0] != 0.0 && s->inv2[1] != 0.0 && s->inv2[2] != 0.0;
    const int32_t ns[3] = {grid->nx, grid->ny, grid->nz};
    bool f2 = p2;
    for (int a = 0; a < 3; ++a) {
      if ((ns[a] & (ns[a] - 1)) != 0) { f2 = false; continue; }
      int e2m = 0, en = 0;  // 2*max = 2^(e2m-1), n = 2^(en-1)
      (void)std::frexp(2.0 * maxes[a], &e2m);
      (void)std::frexp((double)ns[a], &en);
      s->fe[a] = e2m - en;  // face k = k * 2*max/n = k * 2^fe
    }
    s->grid_mode = f2 ? 2 : (p2 ? 1 : 0);
  }
  bool fresnel = false;  // two tops with different refractive indices
  for (int32_t i = 1; i < n_top; ++i) fresnel = fresnel || s->h_props[i].n != s->h_props[0].n;
  {  // the lean path (ws.h): scenes with a few tops
    bool ok = s->bucketed && s->coop_lanes == 0 && grid->nx < (1 << 20) - 2 && grid->ny < (1 << 20) - 2 &&
              grid->nz < (1 << 20) - 2;
    // three segment slots per photon when their LDS fits beside the tile words and faces, else
    // two (SMCRT_WS_SLOTS=2 forces two)
    const char* wsl = std::getenv("SMCRT_WS_SLOTS");
    s->ws_slots = (!(wsl && wsl[0] == '2') && lean_lds(s) + kinst_ws_shared_bytes(3) <= 163840) ? 3 : 2;
    ok = ok && lean_lds(s) + kinst_ws_shared_bytes(s->ws_slots) <= 163840;
    const char* le = std::getenv("SMCRT_LEAN");
    s->lean_mode = le ? (std::string(le) == "0" ? 0 : 1) : -1;
    // Scenes with detectors take the lean path only when forced (SMCRT_LEAN=1): record_hits at
    // every segment end keeps their photon waves the bottleneck, and transport_kernel measured
    // faster on M5 (43.0 vs 30.3-31.1 M photons/s). Fresnel scenes take it (reflect_refract runs
    // in the event waves): M3 169.2-169.8 vs 144.0-144.3 (profiles/r05_ws/ab_m3_m5_fresnel_events.txt)
    s->lean_ok = ok && !s->nested && (s->lean_mode == 1 || (s->lean_mode != 0 && n_dets == 0));
    const char* dm = std::getenv("SMCRT_DEBUG_LEAN_MARGIN");
    s->lean_debug = dm ? (std::string(dm) == "all" ? 2u : (std::string(dm) == "0" ? 1u : 0u)) : 0u;
  }
  if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device) != hipSuccess || cus < 1) cus = 256;
  s->n_cus = cus;
  {
    int khz = 0;  // s_memrealtime's rate
    if (hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, device) == hipSuccess && khz > 0) s->wall_khz = khz;
  }
  if (s->lean_ok) {
    hipError_t oe = hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, ws_kernel_ptr(s->lds_faces, s->grid_mode, fresnel || n_dets > 0,
                                                                               s->ws_slots),
                                                                 kinst_ws_threads(), lean_lds(s));
    if (oe != hipSuccess || per_cu < 1) per_cu = 1;
    s->grid_blocks_ws = cus * per_cu;
    if (fresnel || n_dets > 0) {  // the lane scratch, per launch stream
      s->lscratch_stride = (kinst_ws_scratch_bytes((size_t)s->grid_blocks_ws * kinst_ws_photon_lanes()) + 255) & ~(size_t)255;
      if (hipMalloc((void**)&s->d_lscratch, s->lscratch_stride * (MAX_SLOTS + 1)) != hipSuccess) {
        (void)hipGetLastError();
        s->d_lscratch = nullptr;
        s->lean_ok = false;  // (transport_kernel needs none)
      }
    }
  }
  if (std::getenv("SMCRT_VERBOSE"))
    std::fprintf(stderr, "[smcrt] scene: lean %d (ws slots %d, blocks/CU %d, static LDS %zu + dynamic %zu B), transport grid %d\n",
                 (int)s->lean_ok, s->ws_slots, s->grid_blocks_ws / std::max(1, cus), kinst_ws_shared_bytes(s->ws_slots), lean_lds(s),
                 s->grid_blocks);
  for (int x = 0; x < 2; ++x) {
    const void* kfn = transport_fn(s, x == 1);
    hipError_t oe = hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kfn, 256, transport_lds(s, dep_words(s), x == 1));
    if (oe != hipSuccess || per_cu < 1) per_cu = 1;
    (x ? s->grid_blocks_x : s->grid_blocks) = cus * per_cu;
  }
  *out = s;
  return SMCRT_OK;
}

int smcrt_scene_det_bins(const smcrt_scene* s, int64_t* n) {
  if (!s || !n) return fail(SMCRT_ERR_INVALID_ARG, "NULL argument");
  *n = s->det_total;
  return SMCRT_OK;
}

int smcrt_scene_set_optprops(smcrt_scene* s, int32_t i, double mus, double mua, double hgg, double n) {
  return smcrt::scene_set_node_props(s, i, mus, mua, hgg, n, 0);  // a mono: init_mono's rules
}

int smcrt_scene_get_optprops(const smcrt_scene* s, int32_t i, int32_t* layer, double* mus, double* mua, double* hgg,
                             double* n) {
  if (!s || i < 0 || i >= s->n_top) return fail(SMCRT_ERR_INVALID_ARG, "bad scene or index");
  const smcrt_sdf_node& nd = s->h_nodes[s->h_top[i]];
  if (layer) *layer = nd.layer;
  if (mua) *mua = nd.mua;
  if (mus) *mus = s->h_props[i].kappa - nd.mua;  // getKappa() - getMua(), kernelsMod.f90:1574-1575
  if (hgg) *hgg = nd.hgg;
  if (n) *n = nd.n;
  return SMCRT_OK;
}

}  // extern "C"

int smcrt::scene_node_optprops(const smcrt_scene* s, int32_t i, double out[4]) {
  if (!s || i < 0 || i >= s->n_top) return fail(SMCRT_ERR_INVALID_ARG, "bad scene or index");
  const smcrt_sdf_node& nd = s->h_nodes[s->h_top[i]];
  out[0] = nd.mus; out[1] = nd.mua; out[2] = nd.hgg; out[3] = nd.n;
  return SMCRT_OK;
}

int smcrt::scene_set_node_props(smcrt_scene* s, int32_t i, double mus, double mua, double hgg, double n,
                                int32_t flags) {
  if (!s || i < 0 || i >= s->n_top) return fail(SMCRT_ERR_INVALID_ARG, "bad scene or index");
  std::lock_guard<std::mutex> g(s->mu);
  smcrt_sdf_node& nd = s->h_nodes[s->h_top[i]];
  nd.mus = mus; nd.mua = mua; nd.hgg = hgg; nd.n = n;
  nd.flags = flags;
  s->h_props[i] = make_props(nd);
  HIPCHK(hipSetDevice(s->device));
  HIPCHK(hipMemcpyAsync(s->d_props + i, &s->h_props[i], sizeof(TopProps), hipMemcpyHostToDevice, s->stream));
  HIPCHK(hipStreamSynchronize(s->stream));
  return SMCRT_OK;
}

int smcrt::scene_node_flags(const smcrt_scene* s, int32_t i, int32_t* flags) {
  if (!s || i < 0 || i >= s->n_top) return fail(SMCRT_ERR_INVALID_ARG, "bad scene or index");
  *flags = s->h_nodes[s->h_top[i]].flags;
  return SMCRT_OK;
}

int smcrt::scene_device(const smcrt_scene* s) { return s->device; }
void* smcrt::scene_stream(const smcrt_scene* s) { return (void*)s->stream; }

int smcrt::scene_inflight(smcrt_scene* s) {
  std::lock_guard<std::mutex> g(s->mu);
  int n = 0;
  for (int i = 0; i < MAX_SLOTS; ++i) {
    if (s->lpending[i] && hipEventQuery(s->lev[i]) == hipSuccess) s->lpending[i] = false;
    n += s->lpending[i] ? 1 : 0;
  }
  return n;
}
int smcrt::scene_depth(const smcrt_scene* s) { return s->n_slots; }

int smcrt::scene_det_size(const smcrt_scene* s, int32_t d, int64_t* n) {
  if (!s || d < 0 || d >= s->n_dets) return fail(SMCRT_ERR_INVALID_ARG, "bad scene or detector");
  *n = (d + 1 < s->n_dets ? s->h_det_off[d + 1] : s->det_total) - s->h_det_off[d];
  return SMCRT_OK;
}

extern "C" {

// Refine the records-per-photon estimate from the last binned launch, if it has landed.
static void refine_rpp(smcrt_scene* s) {
  for (int i = 0; i < s->n_slots; ++i) {
    const int sl = s->last_slot < 0 ? i : (s->last_slot + 1 + i) % s->n_slots;  // the oldest slot first
    if (s->ctl_pending[sl] && hipEventQuery(s->ctl_ev[sl]) == hipSuccess) {
      s->ctl_pending[sl] = false;
      const uint32_t* h = s->h_ctl + 8 * sl;
      static const bool pool_log = std::getenv("SMCRT_POOL_LOG") != nullptr;  // diagnostics
      if (pool_log)
        std::fprintf(stderr, "[pool] slot %d: %u photons, %u records, %u overflowed, %u of %llu chunks\n", sl, h[4],
                     h[3], h[1], h[0], (unsigned long long)s->pool_chunks);
      if (h[4] > 0) {
        const double rpp = (double)(h[3] + h[1]) / (double)h[4];
        s->rpp_est = std::max(1.0, rpp);
        s->rpp_measured = true;
      }
    }
  }
}

// Wait (host) for every fold in flight: before the shared fold buffers are reallocated.
static hipError_t drain_folds(smcrt_scene* s) {
  if (!s->fstream) return hipSuccess;
  const hipError_t e = hipStreamSynchronize(s->fstream);
  for (bool& f : s->f_pending) f = false;
  return e;
}

// Records the record pool must hold for one launch of n photons.
// Pool records that a launch's records do not fill: per wave, the last chunk (sorted path),
// or the open bucket of every tile plus the unused ids of its batch (bucketed path).
static double pool_slack_records(const smcrt_scene* s) {
  const double waves = (double)std::max(s->grid_blocks, s->grid_blocks_x) * 4.0;
  // bucketed: per block and tile an open bucket and its pre-taken successor, per wave a batch
  return s->bucketed ? (waves / 4.0 * 2.0 * s->n_tiles + waves * BUCKET_BATCH) * BUCKET_RECORDS
                     : waves * CHUNK_RECORDS;
}
static uint64_t pool_records_for(const smcrt_scene* s, uint64_t n) {
  const double want = (double)n * s->rpp_est * POOL_SLACK + pool_slack_records(s);
  return (uint64_t)std::min(want, (double)MAX_POOL_RECORDS);
}

// Make sure the record pool holds `records` (grow only). Returns false if it cannot.
static bool ensure_pool(smcrt_scene* s, uint64_t records) {
  // (the pool is counted in CHUNK_RECORDS units on both paths: a chunk is 64 buckets)
  uint64_t chunks = (records + CHUNK_RECORDS - 1) / CHUNK_RECORDS;
  if (s->pool_cap_chunks) chunks = std::min(chunks, s->pool_cap_chunks);
  if (chunks <= s->pool_chunks) return true;
  // grow with 25% headroom so launch-to-launch jitter of the estimate never reallocates
  // (a reallocation synchronises the device)
  chunks = std::min<uint64_t>(chunks + chunks / 4, MAX_POOL_RECORDS / CHUNK_RECORDS);
  if (s->pool_cap_chunks) chunks = std::min(chunks, s->pool_cap_chunks);
  // the launches and folds in flight (on any stream) use these buffers
  (void)hipDeviceSynchronize();
  (void)drain_folds(s);
  auto release = [&]() {
    void* old[] = {s->d_sorted, s->d_pieces, s->d_order};
    for (void* p : old)
      if (p) (void)hipFree(p);
    for (int i = 0; i < MAX_SLOTS; ++i) {
      void* per[] = {s->d_pool[i], s->d_chunk_fill[i], s->d_bucket_tile[i]};
      for (void* p : per)
        if (p) (void)hipFree(p);
      s->d_pool[i] = nullptr;
      s->d_chunk_fill[i] = s->d_bucket_tile[i] = nullptr;
    }
    s->d_sorted = nullptr;
    s->d_order = nullptr;
    s->d_pieces = nullptr;
    s->pool_chunks = 0;
  };
  release();
  const uint64_t cap = chunks * CHUNK_RECORDS;
  // pools run MAX_SLOTS deep while MAX_SLOTS of them fit in 60 % of the device's memory (at
  // least DEEP_SLOT_BYTES each; SMCRT_DEEP_SLOT_GIB overrides the size), larger ones two:
  // tail-bound scenes (M4, M5) need the depth to fill the CUs a launch's last photons leave
  // idle. Scenes of the lean kernel and of the far-field march keep two (with eight hardware
  // queues, i.e. launches really four deep, two slots measured M1 211 vs 194-202 M photons/s
  // and M2 15.5-16.4 vs 14.3-14.8 M, same box, profiles/r03_s3/hwq_slots_ab.txt).
  // SMCRT_SLOTS=2 / =4 overrides.
  {
    const char* ns = std::getenv("SMCRT_SLOTS");
    const int want = ns ? std::max(2, std::min(MAX_SLOTS, std::atoi(ns))) : (s->lean_ok || s->fm_err > 0.0 ? 2 : MAX_SLOTS);
    uint64_t deep = DEEP_SLOT_BYTES;
    size_t mfree = 0, mtotal = 0;
    if (hipMemGetInfo(&mfree, &mtotal) == hipSuccess)
      deep = std::max<uint64_t>(deep, (uint64_t)(0.6 * (double)mtotal) / MAX_SLOTS);
    const char* dg = std::getenv("SMCRT_DEEP_SLOT_GIB");
    if (dg) deep = (uint64_t)std::strtoull(dg, nullptr, 10) << 30;
    s->n_slots = cap * 8 <= deep ? want : 2;
    s->slot = 0;    // (the device is idle here: every slot and stream is free)
    s->lturn = 0;
    s->last_slot = -1;
  }
  // pieces <= records / piece size + one partial piece per tile (deposit.h bin_scan, bk_scan)
  const uint64_t pieces = std::min<uint64_t>(cap / MIN_PIECE_RECORDS, REDUCE_PIECES + 1) + s->n_tiles + 1;
  const uint64_t buckets = cap / BUCKET_RECORDS;
  bool ok = hipMalloc((void**)&s->d_pieces, pieces * sizeof(Piece)) == hipSuccess;
  for (int i = 0; ok && i < s->n_slots; ++i) {
    ok = hipMalloc((void**)&s->d_pool[i], cap * 8) == hipSuccess;
    if (ok && s->bucketed)  // bucket fills and bucket tiles, per slot
      ok = hipMalloc((void**)&s->d_chunk_fill[i], buckets * 4) == hipSuccess &&
           hipMalloc((void**)&s->d_bucket_tile[i], buckets * 4) == hipSuccess;
    else if (ok)  // chunk fills, per slot
      ok = hipMalloc((void**)&s->d_chunk_fill[i], chunks * 4) == hipSuccess;
  }
  if (ok && s->bucketed)  // the tile-ordered bucket id list (folds are serial)
    ok = hipMalloc((void**)&s->d_order, buckets * 4) == hipSuccess;
  else if (ok)  // the tile-sorted copy of the records
    ok = hipMalloc((void**)&s->d_sorted, cap * 8) == hipSuccess;
  if (!ok) {
    (void)hipGetLastError();
    release();
    return false;
  }
  s->pool_chunks = chunks;
  s->max_pieces = pieces;
  return true;
}

// One transport launch on `stream` into record slot `sl` (binned), then its deposit fold on
// s->fstream, ordered after the launch by an event. The fold of the previous launch may still
// run while this transport kernel does: they touch different slots (and jmean is only
// written by folds, which are serial on fstream).
static int launch_one(smcrt_scene* s, KParams K, KCold Ch, bool xsrc, hipStream_t stream, int sl, int qi) {
  const bool binned = K.rec_pool != nullptr;
  if (binned && s->f_pending[sl]) HIPCHK(hipStreamWaitEvent(stream, s->ev_f[sl], 0));  // slot free
  Ch.queue = s->d_queue + qi;  // (a queue head per stream: overlapped launches run concurrently)
  Ch.lane_scratch = s->d_lscratch ? (double*)((char*)s->d_lscratch + (size_t)qi * s->lscratch_stride) : nullptr;
  HIPCHK(hipMemsetAsync(Ch.queue, 0, sizeof(unsigned long long), stream));
  // this launch's cold parameters: a ring slot, written in stream order before the kernel.
  // (Each stream has its own ring of slots, so a slot is only ever rewritten in stream order
  // after the launch that read it.)
  KCold* C = s->d_cold + (size_t)qi * COLD_PER_STREAM + (s->cold_seq[qi]++ % COLD_PER_STREAM);
  HIPCHK(hipMemcpyAsync(C, &Ch, sizeof(KCold), hipMemcpyHostToDevice, stream));
  if (binned) {
    HIPCHK(hipMemsetAsync(s->d_dep_ctl[sl], 0, 8 * sizeof(uint32_t), stream));
    if (K.bucket_tiles)  // per-tile bucket counts
      HIPCHK(hipMemsetAsync(s->d_bin_counts[sl], 0, (size_t)s->n_tiles * sizeof(uint32_t), stream));
    else if (K.hist_tiles)
      HIPCHK(hipMemsetAsync(s->d_bin_counts[sl], 0, (size_t)s->n_tiles * BIN_BLOCKS * sizeof(uint32_t), stream));
  }
  hipEvent_t* ev = nullptr;
  if (s->timing) {
    if (s->tev_used == MAX_TIMED) HIPCHK(harvest_times(s));
    if (4 * (s->tev_used + 1) > s->tev.size())
      for (int i = 0; i < 4; ++i) {
        hipEvent_t e;
        HIPCHK(hipEventCreate(&e));
        s->tev.push_back(e);
      }
    ev = &s->tev[4 * s->tev_used++];
    HIPCHK(hipEventRecord(ev[0], stream));
  }
  const uint64_t waves_needed = (Ch.n_photons + 63) / 64;
  const uint64_t blocks_needed = (waves_needed + 3) / 4;
  // the lean path (ws_kernel, ws.h) when the scene and the run qualify: bucketed path-length
  // deposition, unit weights (no survival bias), a plain source
  const bool lean = !xsrc && s->lean_ok && K.bucket_tiles && (K.flags & SMCRT_FLAG_PATHLENGTH) &&
                    !(K.flags & SMCRT_FLAG_SURVIVAL_BIAS);
  const uint64_t ws_needed = (Ch.n_photons + kinst_ws_photon_lanes() - 1) / kinst_ws_photon_lanes();
  const int blocks = (int)std::min<uint64_t>(
      (uint64_t)(lean ? s->grid_blocks_ws : (xsrc ? s->grid_blocks_x : s->grid_blocks)),
      std::max<uint64_t>(1, lean ? ws_needed : blocks_needed));
  if (lean) {
    ++s->lean_launches;
    const KCold* Cc = C;
    const smcrt_sdf_node* a_nodes = K.nodes;
    const ProgOp* a_prog = K.prog;
    void* args[] = {(void*)&K, (void*)&a_nodes, (void*)&a_prog, (void*)&Cc};
    HIPCHK(hipLaunchKernel(ws_kernel_ptr(s->lds_faces, s->grid_mode, s->d_lscratch != nullptr, s->ws_slots), dim3(blocks), dim3(kinst_ws_threads()), args,
                           lean_lds(s), stream));
  } else {
    const KCold* Cc = C;
    const smcrt_sdf_node* a_nodes = K.nodes;
    const ProgOp* a_prog = K.prog;
    const smcrt_detector* a_dets = K.dets;
    const int64_t* a_off = K.det_off;
    void* args[] = {(void*)&K, (void*)&a_nodes, (void*)&a_prog, (void*)&a_dets, (void*)&a_off, (void*)&Cc};
    HIPCHK(hipLaunchKernel(transport_fn(s, xsrc), dim3(blocks), dim3(256), args, transport_lds(s, dep_words(s), xsrc), stream));
  }
  HIPCHK(hipGetLastError());
  if (ev) HIPCHK(hipEventRecord(ev[1], stream));
  if (binned) {
    hipStream_t fs = s->fstream;
    HIPCHK(hipEventRecord(s->ev_t, stream));
    HIPCHK(hipStreamWaitEvent(fs, s->ev_t, 0));
    if (ev) HIPCHK(hipEventRecord(ev[2], fs));
    const uint32_t nch = (uint32_t)s->pool_chunks;
    const uint64_t nv = (uint64_t)s->grid.nx * s->grid.ny * s->grid.nz;
    if (K.bucket_tiles) {  // bucketed: list each tile's buckets, then sum them
      hipLaunchKernelGGL(bk_scan, dim3(1), dim3(1024), 0, fs, s->d_bin_counts[sl], s->n_tiles, s->d_tile_start,
                         s->d_tile_count, s->d_pieces, s->d_dep_ctl[sl]);
      hipLaunchKernelGGL(bk_place, dim3(BIN_BLOCKS), dim3(BIN_THREADS), 0, fs, s->d_bucket_tile[sl], s->d_dep_ctl[sl],
                         K.n_buckets, s->n_tiles, s->d_tile_count, s->d_order);
#ifndef SMCRT_ABL_NO_FOLD  // timing ablation only: records are never summed (not exact)
      hipLaunchKernelGGL(bk_reduce, dim3(1024), dim3(RED_THREADS), 0, fs, s->d_pool[sl], s->d_order, s->d_chunk_fill[sl],
                         s->d_pieces, s->d_dep_ctl[sl], nv, Ch.jmean, s->d_queue + MAX_SLOTS + 2);
#endif
    } else {
    if (!K.hist_tiles)  // else the transport kernel built the counts
      hipLaunchKernelGGL(bin_hist, dim3(BIN_BLOCKS), dim3(BIN_THREADS), 0, fs, s->d_pool[sl], s->d_chunk_fill[sl],
                         s->d_dep_ctl[sl], nch, s->n_tiles, s->d_bin_counts[sl]);
    hipLaunchKernelGGL(bin_rowscan, dim3(s->n_tiles), dim3(BIN_BLOCKS), 0, fs, s->d_bin_counts[sl],
                       s->d_tile_count);
    hipLaunchKernelGGL(bin_scan, dim3(1), dim3(1024), 0, fs, s->d_tile_count, s->n_tiles, s->d_tile_start,
                       s->d_pieces, s->d_dep_ctl[sl]);
    hipLaunchKernelGGL(bin_scatter, dim3(BIN_BLOCKS), dim3(BIN_THREADS), s->scatter_lds, fs, s->d_pool[sl],
                       s->d_chunk_fill[sl], s->d_dep_ctl[sl], nch, s->n_tiles, s->d_tile_start, s->d_bin_counts[sl],
                       s->d_sorted, (uint64_t)s->pool_chunks * CHUNK_RECORDS);
    hipLaunchKernelGGL(bin_reduce, dim3(1024), dim3(1024), 0, fs, s->d_sorted, s->d_pieces, s->d_dep_ctl[sl], nv,
                       Ch.jmean);
    }
    HIPCHK(hipGetLastError());
    // remember how many records this launch produced (read back lazily, never waited for)
    HIPCHK(hipMemcpyAsync(s->h_ctl + 8 * sl, s->d_dep_ctl[sl], 4 * sizeof(uint32_t), hipMemcpyDeviceToHost, fs));
    HIPCHK(hipMemcpyAsync(s->h_ctl + 8 * sl + 5, s->d_dep_ctl[sl] + 5, 2 * sizeof(uint32_t), hipMemcpyDeviceToHost, fs));
    HIPCHK(hipEventRecord(s->ctl_ev[sl], fs));
    s->ctl_pending[sl] = true;
    if (ev) HIPCHK(hipEventRecord(ev[3], fs));
    HIPCHK(hipEventRecord(s->ev_f[sl], fs));
    s->f_pending[sl] = true;
    s->last_slot = sl;
  } else if (ev) {  // no fold: an empty interval
    HIPCHK(hipEventRecord(ev[2], stream));
    HIPCHK(hipEventRecord(ev[3], stream));
  }
#ifdef SMCRT_DIAG
  {
    unsigned long long h[72], ht[9], hc[6];
    HIPCHK(hipStreamSynchronize(stream));
    kinst_diag_gather(h, ht, hc);
    if (lean) {  // ws_kernel's tallies (ws.h WD_*)
      const double wi = (double)std::max(1ull, h[20]), pt = (double)std::max(1ull, h[24]);
      std::fprintf(stderr, "[diag-ws] walker iters %llu: idle %.3f, busy lanes/iter %.1f, pending lanes/iter %.1f | "
                   "photon trips %llu: sleep %.3f, idle lanes %.1f, sync-waiting %.2f, slot-blocked %.2f, EVAL lanes "
                   "%.1f, pushes %.2f, P7 runs %.3f (lanes/run %.1f), event-waiting %.2f | producer waits %llu | event "
                   "iters %llu, lanes/iter %.1f\n",
                   h[20], h[21] / wi, h[22] / wi, h[23] / wi, h[24], h[25] / pt, h[30] / pt, h[27] / pt, h[26] / pt,
                   h[31] / pt, h[32] / pt, h[28] / pt, (double)h[29] / (double)std::max(1ull, h[28]), h[36] / pt, h[33],
                   h[34], (double)h[35] / (double)std::max(1ull, h[34]));
      // region times (ws.h WST): shares of each role's wave time
      const char* np[8] = {"fetch", "poll", "eval", "p3p4", "handout", "p5p6", "p7", "p8"};
      double tp = 0, tw = 0, te = 0;
      for (int i = 0; i < 8; ++i) tp += (double)h[37 + i];
      for (int i = 0; i < 4; ++i) tw += (double)h[45 + i];
      te = (double)h[49] + (double)h[50];
      std::fprintf(stderr, "[diag-ws-time] photon:");
      for (int i = 0; i < 8; ++i) std::fprintf(stderr, " %s=%.3f", np[i], (double)h[37 + i] / std::max(1.0, tp));
      std::fprintf(stderr, " | walker: claim=%.3f idle=%.3f walk=%.3f finish=%.3f | event: run=%.3f idle=%.3f | "
                   "ticks photon/walker/event %.3g/%.3g/%.3g\n", h[45] / std::max(1.0, tw), h[46] / std::max(1.0, tw),
                   h[47] / std::max(1.0, tw), h[48] / std::max(1.0, tw), h[49] / std::max(1.0, te),
                   h[50] / std::max(1.0, te), tp, tw, te);
    }
    unsigned long long lt = 0;
    for (int i = 0; i < 64; ++i) lt += h[i];
    std::fprintf(stderr, "[diag] waves %llu, longest wave %llu trips %llu ticks\n", h[70], h[68], h[69]);
    std::fprintf(stderr, "[diag] trips %llu dda %llu eval %llu p7 %llu | lane-trips %llu:", h[64], h[65], h[66],
                 h[67], lt);
    for (int i = 0; i < 64; ++i)
      if (h[i]) std::fprintf(stderr, " %s%d=%.3f", i >= 32 ? "seg:" : "", i & 31, (double)h[i] / (double)lt);
    std::fprintf(stderr, "\n");

    double tt = 0;
    for (int i = 1; i < 9; ++i) tt += (double)ht[i];
    const char* nm_t[9] = {"", "fetch", "eval", "p3", "p4", "dda", "p5p6", "p7", "p8"};
    const char* nm_l[9] = {"", "fetch", "eval", "p3p4", "push", "walk", "p5p6", "p7", "p8"};
    const char* const* nm = lean ? nm_l : nm_t;
    std::fprintf(stderr, "[diag-time]");
    for (int i = 1; i < 9; ++i) std::fprintf(stderr, " %s=%.3f", nm[i], (double)ht[i] / tt);
    std::fprintf(stderr, "\n");

    if (hc[0] + hc[2])
      std::fprintf(stderr, "[diag-cull] culled lane-EVALs %llu, bound fallbacks %llu (%.4f), capture/outside %llu, "
                   "mean list %.1f, wave-EVALs %llu with a full fallback %.3f\n", hc[0], hc[1],
                   (double)hc[1] / (double)std::max(1ull, hc[0]), hc[2], (double)hc[3] / (double)std::max(1ull, hc[0]),
                   hc[4], (double)hc[5] / (double)std::max(1ull, hc[4]));
  }
#endif
  return SMCRT_OK;
}

// Batched point sources (smcrt_run_origins): device origin table and per-origin detector totals.
struct OriginRun {
  const double* d_origins;
  double* d_totals;
  uint64_t per_origin, first;
};

static int launch(smcrt_scene* s, const smcrt_source* src, const smcrt_run_config* cfg,
                  const smcrt_device_tallies& dt, hipStream_t stream, const OriginRun* orun = nullptr) {
  if (src->kind < SMCRT_SRC_POINT || src->kind > SMCRT_SRC_APERTURE) return fail(SMCRT_ERR_INVALID_ARG, "bad source kind");
  if (cfg->n_photons == 0) return SMCRT_OK;
  // sources other than point/uniform/pencil, a sampled spectrum or batched origins: the
  // general emitter
  const bool xsrc = src_needs_plan(src) || orun || s->nested;
  SrcPlan plan;
  std::memset(&plan, 0, sizeof plan);
  if (xsrc) {
    std::vector<double> px, py, pc;
    const char* perr = "";
    const int pst = build_src_plan(src, &s->grid, &plan, px, py, pc, &perr);
    if (pst) return fail(pst, perr);
    std::vector<double> tab;
    tab.reserve(px.size() + py.size() + pc.size());
    tab.insert(tab.end(), px.begin(), px.end());
    tab.insert(tab.end(), py.begin(), py.end());
    tab.insert(tab.end(), pc.begin(), pc.end());
    if (!tab.empty()) {
      if (tab != s->h_spec) {  // new tables: wait for launches that may still read the old ones
        HIPCHK(hipStreamSynchronize(stream));
        if (s->stream != stream) HIPCHK(hipStreamSynchronize(s->stream));
        if (tab.size() > s->spec_cap) {
          if (s->d_spec) HIPCHK(hipFree(s->d_spec));
          s->d_spec = nullptr;
          s->spec_cap = 0;
          HIPCHK(hipMalloc((void**)&s->d_spec, tab.size() * sizeof(double)));
          s->spec_cap = tab.size();
        }
        HIPCHK(hipMemcpy(s->d_spec, tab.data(), tab.size() * sizeof(double), hipMemcpyHostToDevice));
        s->h_spec = tab;
      }
      plan.spec_x = px.empty() ? nullptr : s->d_spec;
      plan.spec_y = py.empty() ? nullptr : s->d_spec + px.size();
      plan.cdf = s->d_spec + px.size() + py.size();
    }
    if (orun) {
      plan.origins = orun->d_origins;
      plan.det_totals = orun->d_totals;
      plan.per_origin = orun->per_origin;
      plan.first = orun->first;
    }
  }
  KParams K;
  K.nodes = s->d_nodes;
  K.prog = s->d_prog;
  K.n_prog = s->n_prog;
  K.coop_lanes = s->coop_lanes;
  K.cull = s->d_cull;
  K.ctab = s->d_ctab;
  const bool far = s->fm_err > 0.0 && (cfg->flags & SMCRT_FLAG_PATHLENGTH);
  K.fm_err = far ? s->fm_err : 0.0;
  K.fm_step = s->fm_step;
  K.inv2x = s->inv2[0]; K.inv2y = s->inv2[1]; K.inv2z = s->inv2[2];
  K.fex = s->fe[0]; K.fey = s->fe[1]; K.fez = s->fe[2];
  K.props = s->d_props;
  K.xface = s->d_faces;
  K.yface = s->d_faces + (s->grid.nx + 1);
  K.zface = s->d_faces + (s->grid.nx + 1) + (s->grid.ny + 1);
  K.dets = s->d_dets;
  K.det_off = s->d_det_off;
  K.n_top = s->n_top;
  K.n_dets = s->n_dets;
  K.nx = s->grid.nx; K.ny = s->grid.ny; K.nz = s->grid.nz;
  K.xmax = s->grid.xmax; K.ymax = s->grid.ymax; K.zmax = s->grid.zmax;
  K.flags = cfg->flags;
  KCold Ch;
  Ch.src = *src;
  Ch.plan = plan;
  K.key0 = (uint32_t)cfg->seed;
  K.key1 = (uint32_t)(cfg->seed >> 32);
  Ch.jmean = dt.jmean; Ch.absorb = dt.absorb; Ch.emission = dt.emission;
  Ch.chunk_fill = nullptr; Ch.dep_ctl = nullptr; Ch.bin_counts = nullptr;  // (per slot, below)
  Ch.bucket_tile = nullptr; Ch.bucket_fill = nullptr; Ch.tile_nb = nullptr;
  Ch.det_bins = dt.det_bins; Ch.nscatt = dt.nscatt; Ch.moments = dt.moments;
  Ch.counters = (unsigned long long*)dt.counters;
  Ch.queue = nullptr;  // (set per launch: launch_one)
  Ch.far_steps = s->d_queue + MAX_SLOTS + 1;
  Ch.lean_hazards = s->d_queue + MAX_SLOTS + 3;
  Ch.lane_scratch = nullptr;  // (per launch stream: launch_one)
  Ch.watchdog = watchdog_word(s);
#ifdef SMCRT_DIAG
  Ch.done_time = nullptr;
  Ch.done_base = cfg->first_photon;
  if (const char* dd = std::getenv("SMCRT_DIAG_DONE")) {  // (diagnostic builds: completion times)
    if (dd[0] == '1' && !orun) {
      if (s->d_done) (void)hipFree(s->d_done);
      s->d_done = nullptr;
      s->n_done = cfg->n_photons;
      HIPCHK(hipMalloc(&s->d_done, sizeof(unsigned long long) * s->n_done));
      HIPCHK(hipMemsetAsync(s->d_done, 0, sizeof(unsigned long long) * s->n_done, stream));
      Ch.done_time = s->d_done;
    }
  }
#endif
  {  // every cross-wave wait is bounded (transport.h watchdog_expired); 0 ms: unbounded
    const char* wm = std::getenv("SMCRT_WATCHDOG_MS");
    const double ms = wm ? std::strtod(wm, nullptr) : (double)DEFAULT_WATCHDOG_MS;
    Ch.watchdog_ticks = ms > 0.0 ? (uint64_t)(ms * (double)s->wall_khz) : 0ull;
  }
  K.rec_pool = nullptr; K.n_chunks = 0; K.hist_tiles = 0; K.bucket_tiles = 0; K.n_buckets = 0;
  {
    const char* cd = std::getenv("SMCRT_DEBUG_CLAIM_DELAY");
    K.claim_delay = cd ? (uint32_t)std::strtoul(cd, nullptr, 10) : 0u;
  }
  K.lean_debug = s->lean_debug;
  if (const char* de = std::getenv("SMCRT_DEBUG_DROP_EVENT"))  // (tests only: the watchdog's proof)
    if (de[0] == '1') K.lean_debug |= 4u;
  {  // lean_margin per axis (lean.h, ws.h), with the operations the kernel used to do
    const double eps = 1e-8, mf = (K.lean_debug & 3u) ? 0.0 : 2.0 * eps;
    const double mx = mf * (double)(K.nx + 2), my = mf * (double)(K.ny + 2), mz = mf * (double)(K.nz + 2);
    K.lean_lo[0] = mx; K.lean_lo[1] = my; K.lean_lo[2] = mz;
    K.lean_hi[0] = 2.0 * K.xmax - mx; K.lean_hi[1] = 2.0 * K.ymax - my; K.lean_hi[2] = 2.0 * K.zmax - mz;
  }

  // binned deposition needs path-length tallies into jmean with unit weights (fp32 record
  // values are exact only then) and a grid of at most MAX_TILES tiles
  const bool binned = dt.jmean && (cfg->flags & SMCRT_FLAG_PATHLENGTH) && !(cfg->flags & SMCRT_FLAG_SURVIVAL_BIAS) &&
                      s->n_tiles > 0 && !s->force_atomic;
  const bool overlap = (cfg->flags & SMCRT_FLAG_OVERLAP) != 0;
  if (overlap) {  // the internal streams start after the caller's earlier work
    HIPCHK(hipEventRecord(s->ev_in, stream));
    for (int i = 0; i < MAX_SLOTS; ++i) HIPCHK(hipStreamWaitEvent(s->lstream[i], s->ev_in, 0));
  } else {  // a plain launch runs after every overlapped one (same tallies, same buffers)
    for (int i = 0; i < MAX_SLOTS; ++i)
      if (s->lpending[i]) HIPCHK(hipStreamWaitEvent(stream, s->lev[i], 0));
  }
  for (int i = 0; i < MAX_SLOTS; ++i)  // launches known to have finished need no more waits
    if (s->lpending[i] && hipEventQuery(s->lev[i]) == hipSuccess) s->lpending[i] = false;
  for (uint64_t done = 0; done < cfg->n_photons;) {
    refine_rpp(s);
    uint64_t n = cfg->n_photons - done;
    K.rec_pool = nullptr; K.n_chunks = 0; K.hist_tiles = 0; K.bucket_tiles = 0; K.n_buckets = 0;
    bool calibrate = false;
    if (binned) {
      // records per photon are scene-dependent: the scene's first large launch starts with a
      // small calibration batch whose count is waited for once, then batches are sized to it
      if (!s->rpp_measured && n > CALIB_PHOTONS) { n = CALIB_PHOTONS; calibrate = true; }
      const uint64_t want = pool_records_for(s, n);
      if (!ensure_pool(s, want)) (void)ensure_pool(s, want / 4);  // smaller pool, more batches
      if (s->pool_chunks) {
        const double usable = (double)(s->pool_chunks * CHUNK_RECORDS) - pool_slack_records(s);
        n = std::min<uint64_t>(n, (uint64_t)std::max(65536.0, usable / (s->rpp_est * POOL_SLACK)));
        // (taken after ensure_pool: it may have reallocated the pool)
        K.rec_pool = s->d_pool[s->slot];
        Ch.chunk_fill = s->d_chunk_fill[s->slot];  // (ensure_pool may have reallocated them)
        Ch.dep_ctl = s->d_dep_ctl[s->slot];
        Ch.bin_counts = s->d_bin_counts[s->slot];
        K.n_chunks = (uint32_t)s->pool_chunks;
        K.hist_tiles = s->hist_tiles;
        if (s->bucketed) {
          Ch.bucket_fill = s->d_chunk_fill[s->slot];
          Ch.bucket_tile = s->d_bucket_tile[s->slot];
          Ch.tile_nb = s->d_bin_counts[s->slot];
          K.bucket_tiles = s->n_tiles;
          K.n_buckets = (uint32_t)(s->pool_chunks * (CHUNK_RECORDS / BUCKET_RECORDS));
        }
      }
    }
    Ch.n_photons = n;
    Ch.first_photon = orun ? done : cfg->first_photon + done;  // (origins: the global queue index)
    Ch.records = dt.records ? dt.records + done : nullptr;
    const int sl = s->slot;
    if (K.rec_pool) {
      // (the slot's previous readback must land before its photon count is replaced)
      if (s->ctl_pending[sl]) { HIPCHK(hipEventSynchronize(s->ctl_ev[sl])); refine_rpp(s); }
      s->h_ctl[8 * sl + 4] = (uint32_t)std::min<uint64_t>(n, 0xFFFFFFFFull);
    }
    int st;
    if (overlap) {
      const int q = s->lturn;
      s->lturn = (s->lturn + 1) % s->n_slots;
      st = launch_one(s, K, Ch, xsrc, s->lstream[q], sl, q);
      if (!st && hipEventRecord(s->lev[q], s->lstream[q]) != hipSuccess) st = fail(SMCRT_ERR_HIP, "event record failed");
      s->lpending[q] = true;
    } else {
      st = launch_one(s, K, Ch, xsrc, stream, sl, MAX_SLOTS);
    }
    if (st) return st;
    if (K.rec_pool) s->slot = (s->slot + 1) % s->n_slots;
    if (calibrate && K.rec_pool) {
      HIPCHK(hipEventSynchronize(s->ctl_ev[sl]));
      refine_rpp(s);
    }
    done += n;
  }
  // the tallies are complete in `stream` order at return, unless the caller defers the folds
  if (!(cfg->flags & (SMCRT_FLAG_ASYNC_FOLD | SMCRT_FLAG_OVERLAP)) && s->last_slot >= 0 && s->f_pending[s->last_slot])
    HIPCHK(hipStreamWaitEvent(stream, s->ev_f[s->last_slot], 0));
  return SMCRT_OK;
}

int smcrt_run_device(smcrt_scene* s, const smcrt_source* src, const smcrt_run_config* cfg,
                     smcrt_device_tallies* dev, void* stream) {
  g_last_error.clear();
  if (!s || !src || !cfg || !dev) return fail(SMCRT_ERR_INVALID_ARG, "NULL argument");
  std::lock_guard<std::mutex> g(s->mu);
  HIPCHK(hipSetDevice(s->device));
  return launch(s, src, cfg, *dev, (hipStream_t)stream);
}

}  // extern "C"

// smcrt_run's body; `orun` (batched origins) is set by smcrt_run_origins. Caller holds s->mu.
static int run_sync(smcrt_scene* s, const smcrt_source* src, const smcrt_run_config* cfg_in, smcrt_tallies* io,
                    const OriginRun* orun) {
  // A synchronous run returns complete tallies: its folds always join s->stream before the
  // copies, whatever the caller's flags say (SMCRT_FLAG_ASYNC_FOLD is for smcrt_run_device).
  smcrt_run_config cfg_local = *cfg_in;
  cfg_local.flags &= ~(uint32_t)(SMCRT_FLAG_ASYNC_FOLD | SMCRT_FLAG_OVERLAP);
  const smcrt_run_config* cfg = &cfg_local;
  const int64_t nv = (int64_t)s->grid.nx * s->grid.ny * s->grid.nz;
  const bool want[3] = {io->jmean || io->jmean_f64, io->absorb || io->absorb_f64, io->emission || io->emission_f64};
  if (!s->d_grids && (want[0] || want[1] || want[2])) {
    int st = dalloc(&s->d_grids, (size_t)nv * 3);
    if (st) return st;
  }
  const bool rec = (cfg->flags & SMCRT_FLAG_RECORD_PHOTONS) && io->records;
  if (rec && s->records_cap < cfg->n_photons) {
    if (s->d_records) { HIPCHK(hipFree(s->d_records)); s->d_records = nullptr; }
    int st = dalloc(&s->d_records, cfg->n_photons);
    if (st) return st;
    s->records_cap = cfg->n_photons;
  }
  smcrt_device_tallies dt{};
  for (int t = 0; t < 3; ++t) {
    if (!want[t]) continue;
    double* p = s->d_grids + (size_t)t * nv;
    HIPCHK(hipMemsetAsync(p, 0, sizeof(double) * nv, s->stream));
    if (t == 0) dt.jmean = p;
    if (t == 1) dt.absorb = p;
    if (t == 2) dt.emission = p;
  }
  HIPCHK(hipMemsetAsync(s->d_small, 0, sizeof(double) * (s->det_total + 25), s->stream));
  HIPCHK(hipMemsetAsync(s->d_counters, 0, sizeof(unsigned long long) * SMCRT_NCOUNTERS, s->stream));
  dt.det_bins = s->det_total ? s->d_small : nullptr;
  dt.nscatt = s->d_small + s->det_total;
  dt.moments = s->d_small + s->det_total + 1;
  dt.counters = (uint64_t*)s->d_counters;
  dt.records = rec ? s->d_records : nullptr;
  int st = launch(s, src, cfg, dt, s->stream, orun);
  if (st) return st;
  hipError_t e = hipStreamSynchronize(s->stream);
  if (e != hipSuccess) return fail(SMCRT_ERR_DEVICE_FAULT, std::string("transport kernel: ") + hipGetErrorString(e));
  if ((st = take_watchdog(s))) return st;
  // copy back and accumulate
  std::vector<double> h;
  float* gf[3] = {io->jmean, io->absorb, io->emission};
  double* gd[3] = {io->jmean_f64, io->absorb_f64, io->emission_f64};
  for (int t = 0; t < 3; ++t) {
    if (!want[t]) continue;
    h.resize((size_t)nv);
    HIPCHK(hipMemcpy(h.data(), s->d_grids + (size_t)t * nv, sizeof(double) * nv, hipMemcpyDeviceToHost));
    for (int64_t i = 0; i < nv; ++i) {
      if (gf[t]) gf[t][i] = (float)((double)gf[t][i] + h[i]);
      if (gd[t]) gd[t][i] += h[i];
    }
  }
  std::vector<double> small((size_t)s->det_total + 25);
  HIPCHK(hipMemcpy(small.data(), s->d_small, sizeof(double) * small.size(), hipMemcpyDeviceToHost));
  if (io->det_bins)
    for (int64_t i = 0; i < s->det_total; ++i) io->det_bins[i] += small[i];
  if (io->nscatt) *io->nscatt += small[s->det_total];
  if (io->moments)
    for (int i = 0; i < 24; ++i) io->moments[i] += small[s->det_total + 1 + i];
  if (io->counters) {
    unsigned long long c[SMCRT_NCOUNTERS];
    HIPCHK(hipMemcpy(c, s->d_counters, sizeof(c), hipMemcpyDeviceToHost));
    for (int i = 0; i < SMCRT_NCOUNTERS; ++i) io->counters[i] += c[i];
  }
  if (rec)
    HIPCHK(hipMemcpy(io->records, s->d_records, sizeof(smcrt_photon_record) * cfg->n_photons, hipMemcpyDeviceToHost));
  return SMCRT_OK;
}

extern "C" {

int smcrt_run(smcrt_scene* s, const smcrt_source* src, const smcrt_run_config* cfg, smcrt_tallies* io) {
  g_last_error.clear();
  if (!s || !src || !cfg || !io) return fail(SMCRT_ERR_INVALID_ARG, "NULL argument");
  std::lock_guard<std::mutex> g(s->mu);
  HIPCHK(hipSetDevice(s->device));
  return run_sync(s, src, cfg, io, nullptr);
}

int smcrt_run_origins(smcrt_scene* s, const smcrt_source* src, const double* origins, int64_t n_origins,
                      const smcrt_run_config* cfg, double* det_totals, smcrt_tallies* io) {
  g_last_error.clear();
  if (!s || !cfg || !io || (n_origins > 0 && !origins)) return fail(SMCRT_ERR_INVALID_ARG, "NULL argument");
  if (n_origins < 0) return fail(SMCRT_ERR_INVALID_ARG, "n_origins < 0");
  if (cfg->flags & SMCRT_FLAG_RECORD_PHOTONS) return fail(SMCRT_ERR_INVALID_ARG, "photon records are not kept for batched origins");
  if (n_origins > 0xFFFFFFFFll) return fail(SMCRT_ERR_INVALID_ARG, "more than 2^32 origins");
  if (n_origins == 0 || cfg->n_photons == 0) return SMCRT_OK;
  if (cfg->n_photons > UINT64_MAX / (uint64_t)n_origins) return fail(SMCRT_ERR_INVALID_ARG, "photon count overflows");
  std::lock_guard<std::mutex> g(s->mu);
  HIPCHK(hipSetDevice(s->device));
  smcrt_source p;  // the escape function's packet = photon("point") (kernelsMod.f90:162-166)
  if (src) p = *src;
  else std::memset(&p, 0, sizeof p);
  p.kind = SMCRT_SRC_POINT;
  const size_t nt = (size_t)n_origins * (size_t)std::max(s->n_dets, 1);
  double* d_org = nullptr;
  double* d_tot = nullptr;
  int st = dalloc(&d_org, (size_t)n_origins * 3);
  if (!st) st = dalloc(&d_tot, nt);
  if (!st) {
    OriginRun orun{d_org, s->n_dets ? d_tot : nullptr, cfg->n_photons, cfg->first_photon};
    smcrt_run_config c = *cfg;
    c.n_photons = cfg->n_photons * (uint64_t)n_origins;
    hipError_t e = hipMemcpy(d_org, origins, sizeof(double) * 3 * (size_t)n_origins, hipMemcpyHostToDevice);
    if (e == hipSuccess) e = hipMemset(d_tot, 0, sizeof(double) * nt);
    if (e != hipSuccess) st = fail(SMCRT_ERR_HIP, std::string("origin upload: ") + hipGetErrorString(e));
    if (!st) st = run_sync(s, &p, &c, io, &orun);
    if (!st && det_totals && s->n_dets) {
      std::vector<double> h(nt);
      e = hipMemcpy(h.data(), d_tot, sizeof(double) * nt, hipMemcpyDeviceToHost);
      if (e != hipSuccess) st = fail(SMCRT_ERR_HIP, std::string("totals: ") + hipGetErrorString(e));
      else for (size_t i = 0; i < nt; ++i) det_totals[i] += h[i];
    }
  }
  if (d_org) (void)hipFree(d_org);
  if (d_tot) (void)hipFree(d_tot);
  return st;
}

#ifdef SMCRT_DIAG
// Diagnostic builds only (not in include/smcrt.h): read and clear the kernel's lane-state
// occupancy (72) and per-phase s_memtime sums (9).
int smcrt_diag_read(unsigned long long* out) {
  HIPCHK(hipDeviceSynchronize());
  unsigned long long hc[6];
  kinst_diag_gather(out, out + 72, hc);
  return SMCRT_OK;
}
// The completion time (s_memrealtime ticks) of each photon of the scene's last run made with
// SMCRT_DIAG_DONE=1 (n of them; 0 = not completed), and the tick rate in kHz.
int smcrt_diag_done_times(smcrt_scene* s, unsigned long long* out, uint64_t n, int32_t* khz) {
  if (!s || !out || !s->d_done || n > s->n_done) return fail(SMCRT_ERR_INVALID_ARG, "no completion times");
  HIPCHK(hipDeviceSynchronize());
  HIPCHK(hipMemcpy(out, s->d_done, sizeof(unsigned long long) * n, hipMemcpyDeviceToHost));
  if (khz) *khz = s->wall_khz;
  return SMCRT_OK;
}
#endif

int smcrt_scene_info(const smcrt_scene* s, smcrt_grid* grid, int32_t* n_top, int32_t* n_dets) {
  if (!s) return fail(SMCRT_ERR_INVALID_ARG, "scene is NULL");
  if (grid) *grid = s->grid;
  if (n_top) *n_top = s->n_top;
  if (n_dets) *n_dets = s->n_dets;
  return SMCRT_OK;
}

int smcrt_scene_classify(smcrt_scene* s, const double* points, int64_t n, int32_t* layer, double* kappa) {
  g_last_error.clear();
  if (!s || (n > 0 && (!points || !layer))) return fail(SMCRT_ERR_INVALID_ARG, "NULL argument");
  if (n <= 0) return SMCRT_OK;
  std::lock_guard<std::mutex> g(s->mu);
  HIPCHK(hipSetDevice(s->device));
  double* d_pts = nullptr;
  int32_t* d_lay = nullptr;
  int st = dalloc(&d_pts, (size_t)n * 3);
  if (!st) st = dalloc(&d_lay, (size_t)n);
  if (!st) {
    hipError_t e = hipMemcpy(d_pts, points, sizeof(double) * 3 * (size_t)n, hipMemcpyHostToDevice);
    if (e == hipSuccess) {
      const int blocks = (int)std::min<int64_t>((n + 255) / 256, 65535);
      hipLaunchKernelGGL(classify_kernel, dim3(blocks), dim3(256), 0, s->stream, (const smcrt_sdf_node*)s->d_nodes,
                         (const ProgOp*)s->d_prog, (int32_t)s->n_prog, (const double*)d_pts, n, d_lay);
      e = hipGetLastError();
    }
    if (e == hipSuccess) e = hipStreamSynchronize(s->stream);
    if (e == hipSuccess) e = hipMemcpy(layer, d_lay, sizeof(int32_t) * (size_t)n, hipMemcpyDeviceToHost);
    if (e != hipSuccess) st = fail(SMCRT_ERR_HIP, std::string("classify: ") + hipGetErrorString(e));
  }
  if (!st && kappa)
    for (int64_t i = 0; i < n; ++i) kappa[i] = layer[i] > 0 ? s->h_props[layer[i] - 1].kappa : 0.0;
  if (d_pts) (void)hipFree(d_pts);
  if (d_lay) (void)hipFree(d_lay);
  return st;
}

int smcrt_scene_fence(smcrt_scene* s, void* stream) {
  g_last_error.clear();
  if (!s) return fail(SMCRT_ERR_INVALID_ARG, "scene is NULL");
  std::lock_guard<std::mutex> g(s->mu);
  HIPCHK(hipSetDevice(s->device));
  for (int i = 0; i < MAX_SLOTS; ++i)  // overlapped launches (their folds are ordered after them)
    if (s->lpending[i]) HIPCHK(hipStreamWaitEvent((hipStream_t)stream, s->lev[i], 0));
  if (s->last_slot >= 0 && s->f_pending[s->last_slot])  // folds are serial: the last covers all
    HIPCHK(hipStreamWaitEvent((hipStream_t)stream, s->ev_f[s->last_slot], 0));
  return SMCRT_OK;
}

int smcrt_scene_check(smcrt_scene* s) {
  g_last_error.clear();
  if (!s) return fail(SMCRT_ERR_INVALID_ARG, "scene is NULL");
  std::lock_guard<std::mutex> g(s->mu);
  HIPCHK(hipSetDevice(s->device));
  for (int i = 0; i < MAX_SLOTS; ++i)
    if (s->lstream[i]) {
      const hipError_t e = hipStreamSynchronize(s->lstream[i]);
      if (e != hipSuccess) return fail(SMCRT_ERR_DEVICE_FAULT, std::string("transport kernel: ") + hipGetErrorString(e));
    }
  for (hipStream_t st : {s->stream, s->fstream})
    if (st) {
      const hipError_t e = hipStreamSynchronize(st);
      if (e != hipSuccess) return fail(SMCRT_ERR_DEVICE_FAULT, std::string("transport kernel: ") + hipGetErrorString(e));
    }
  return take_watchdog(s);
}

int smcrt_scene_set_timing(smcrt_scene* s, int32_t enable) {
  if (!s) return fail(SMCRT_ERR_INVALID_ARG, "scene is NULL");
  std::lock_guard<std::mutex> g(s->mu);
  s->timing = enable != 0;
  return SMCRT_OK;
}

int smcrt_scene_kernel_times(smcrt_scene* s, smcrt_kernel_times* out) {
  if (!s || !out) return fail(SMCRT_ERR_INVALID_ARG, "NULL argument");
  std::lock_guard<std::mutex> g(s->mu);
  HIPCHK(hipSetDevice(s->device));
  HIPCHK(harvest_times(s));
  out->transport_ms = s->t_transport;
  out->deposit_ms = s->t_deposit;
  out->launches = s->t_launches;
  out->lean_launches = s->lean_launches;
  s->lean_launches = 0;
  unsigned long long far = 0;  // (a running total: steps of launches still running count later)
  HIPCHK(hipMemcpy(&far, s->d_queue + MAX_SLOTS + 1, sizeof(far), hipMemcpyDeviceToHost));
  out->far_steps = (int64_t)(far - s->far_reported);
  s->far_reported = far;
  unsigned long long ticks = 0;  // bk_reduce workgroup run time (running total, wall-clock ticks)
  HIPCHK(hipMemcpy(&ticks, s->d_queue + MAX_SLOTS + 2, sizeof(ticks), hipMemcpyDeviceToHost));
  out->fold_cu_ms = (double)(ticks - s->fold_ticks_reported) / (double)s->wall_khz / (double)s->n_cus;
  s->fold_ticks_reported = ticks;
  unsigned long long hz = 0;  // deferred lean segments that ended in tflag / an error stop (running total)
  HIPCHK(hipMemcpy(&hz, s->d_queue + MAX_SLOTS + 3, sizeof(hz), hipMemcpyDeviceToHost));
  out->lean_hazards = (int64_t)(hz - s->hazards_reported);
  s->hazards_reported = hz;
  s->t_transport = s->t_deposit = 0.0;
  s->t_launches = 0;
  return SMCRT_OK;
}

int smcrt_normalise_fluence(float* g, const smcrt_grid* grid, uint64_t nphotons) {
  if (!g || !grid || nphotons == 0) return fail(SMCRT_ERR_INVALID_ARG, "bad arguments");
  // writer.f90:25-52, evaluated in double as the Fortran expression is
  const double xmax = grid->xmax, ymax = grid->ymax, zmax = grid->zmax;
  const double f = (2.0 * xmax * 2.0 * ymax * 2.0 * zmax) /
                   ((double)nphotons * (2.0 * xmax / grid->nx) * (2.0 * ymax / grid->ny) * (2.0 * zmax / grid->nz));
  const int64_t nv = (int64_t)grid->nx * grid->ny * grid->nz;
  for (int64_t i = 0; i < nv; ++i) g[i] = (float)((double)g[i] * f);
  return SMCRT_OK;
}

}  // extern "C"
