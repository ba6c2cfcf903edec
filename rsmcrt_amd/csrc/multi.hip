// multi.hip — photon shards over several GPUs and ONE packed RCCL reduction of the tallies
// (include/smcrt.h "multi-GPU"; SURVEY.md §8(b) n_gpus, §8(e)).
//
// Reference: run_MCRT splits `do j = 1, nphotons` statically over OpenMP threads
// (/root/reference/src/kernelsMod.f90:1859) and its MPI build sums the module-global
// tallies onto the root (mpi_reduce, kernelsMod.f90:2351-2357). Here a photon's Philox stream
// is keyed by its global index, so a shard of the index range on each GPU computes exactly
// the photons one GPU would; the single exchange per run is one collective over a packed fp64
// buffer (grids | detector bins | nscatt, moments, counters), over xGMI between the GPUs.
//
// RCCL is resolved with dlopen on first use (librccl.so.1: the ROCm install's, or the copy a
// host process such as torch has already loaded), so the library has no link-time RCCL
// dependency and the CPU-only paths never touch it.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>
#include <dlfcn.h>

#include <algorithm>
#include <chrono>
#include <cstdlib>
#include <thread>
#include <cstring>
#include <mutex>
#include <string>
#include <vector>

#include "../../include/smcrt.h"
#include "hosterr.h"
#include "scene_internal.h"

using smcrt::g_last_error;
using smcrt::set_error;

namespace {

// ------------------------------------------------------------------ RCCL loader -------
struct Rccl {
  bool ok = false;
  std::string err;
  ncclResult_t (*get_unique_id)(ncclUniqueId*) = nullptr;
  ncclResult_t (*comm_init_rank)(ncclComm_t*, int, ncclUniqueId, int) = nullptr;
  ncclResult_t (*comm_init_all)(ncclComm_t*, int, const int*) = nullptr;
  ncclResult_t (*comm_destroy)(ncclComm_t) = nullptr;
  ncclResult_t (*all_reduce)(const void*, void*, size_t, ncclDataType_t, ncclRedOp_t, ncclComm_t,
                             hipStream_t) = nullptr;
  ncclResult_t (*reduce)(const void*, void*, size_t, ncclDataType_t, ncclRedOp_t, int, ncclComm_t,
                         hipStream_t) = nullptr;
  ncclResult_t (*group_start)() = nullptr;
  ncclResult_t (*group_end)() = nullptr;
  const char* (*error_string)(ncclResult_t) = nullptr;
  ncclResult_t (*comm_count)(const ncclComm_t, int*) = nullptr;      // (optional: smcrt_comm_info)
  ncclResult_t (*comm_user_rank)(const ncclComm_t, int*) = nullptr;  // (optional)
};

const Rccl& rccl() {
  static Rccl r;
  static std::once_flag once;
  std::call_once(once, [] {
    void* h = dlopen("librccl.so.1", RTLD_NOW | RTLD_GLOBAL);
    if (!h) h = dlopen("/opt/rocm/lib/librccl.so.1", RTLD_NOW | RTLD_GLOBAL);
    if (!h) {
      const char* e = dlerror();
      r.err = std::string("cannot load librccl.so.1: ") + (e ? e : "?");
      return;
    }
    auto sym = [&](const char* name) {
      void* p = dlsym(h, name);
      if (!p && r.err.empty()) r.err = std::string("librccl.so.1 lacks ") + name;
      return p;
    };
    r.get_unique_id = (decltype(r.get_unique_id))sym("ncclGetUniqueId");
    r.comm_init_rank = (decltype(r.comm_init_rank))sym("ncclCommInitRank");
    r.comm_init_all = (decltype(r.comm_init_all))sym("ncclCommInitAll");
    r.comm_destroy = (decltype(r.comm_destroy))sym("ncclCommDestroy");
    r.all_reduce = (decltype(r.all_reduce))sym("ncclAllReduce");
    r.reduce = (decltype(r.reduce))sym("ncclReduce");
    r.group_start = (decltype(r.group_start))sym("ncclGroupStart");
    r.group_end = (decltype(r.group_end))sym("ncclGroupEnd");
    r.error_string = (decltype(r.error_string))sym("ncclGetErrorString");
    r.comm_count = (decltype(r.comm_count))dlsym(h, "ncclCommCount");
    r.comm_user_rank = (decltype(r.comm_user_rank))dlsym(h, "ncclCommUserRank");
    r.ok = r.err.empty();
  });
  return r;
}

int fail(int code, const std::string& msg) { return set_error(code, msg); }

#define HIPCHK(expr)                                                                      \
  do {                                                                                    \
    hipError_t e_ = (expr);                                                               \
    if (e_ != hipSuccess)                                                                 \
      return fail(SMCRT_ERR_HIP, std::string(#expr " failed: ") + hipGetErrorString(e_)); \
  } while (0)

#define NCCLCHK(expr)                                                                                  \
  do {                                                                                                 \
    ncclResult_t r_ = (expr);                                                                          \
    if (r_ != ncclSuccess)                                                                             \
      return fail(SMCRT_ERR_RCCL, std::string(#expr " failed: ") + rccl().error_string(r_));           \
  } while (0)

// ------------------------------------------------------------------ packed layout ----
struct Offsets {
  int64_t jmean = -1, absorb = -1, emission = -1, det = -1, nscatt = 0, moments = 0, counters = 0, total = 0;
};

Offsets offsets(const smcrt_pack_layout& L) {
  Offsets o;
  int64_t at = 0;
  if (L.fields & SMCRT_PACK_JMEAN) { o.jmean = at; at += L.n_voxels; }
  if (L.fields & SMCRT_PACK_ABSORB) { o.absorb = at; at += L.n_voxels; }
  if (L.fields & SMCRT_PACK_EMISSION) { o.emission = at; at += L.n_voxels; }
  if (L.fields & SMCRT_PACK_DET_BINS) { o.det = at; at += L.n_det_bins; }
  o.nscatt = at; at += 1;
  o.moments = at; at += 24;
  o.counters = at; at += SMCRT_NCOUNTERS;
  o.total = at;
  return o;
}

bool layout_ok(const smcrt_pack_layout* L) {
  return L && L->n_voxels >= 0 && L->n_det_bins >= 0 && (L->fields & ~0xFu) == 0;
}

// counters travel as doubles (exact below 2^53)
__global__ void counters_to_f64(const unsigned long long* __restrict__ c, double* __restrict__ out) {
  const int i = threadIdx.x;
  if (i < SMCRT_NCOUNTERS) out[i] = c ? (double)c[i] : 0.0;
}
__global__ void counters_from_f64(const double* __restrict__ in, unsigned long long* __restrict__ c) {
  const int i = threadIdx.x;
  if (i < SMCRT_NCOUNTERS) c[i] = (unsigned long long)in[i];
}

// the device buffers of `dev`, in packed order, with their packed offsets
struct Span {
  double* dev;
  int64_t off, n;
};

}  // namespace

struct smcrt_comm {
  ncclComm_t comm = nullptr;
  int32_t n_ranks = 0, rank = 0, device = 0;
  double* d_buf = nullptr;  // packed buffer (grown on demand)
  size_t cap = 0;
};

struct smcrt_multi {
  std::vector<int32_t> devices;
  std::vector<smcrt_scene*> scenes;
  std::vector<ncclComm_t> comms;
  // per device: resident fp64 accumulators in the packed layout of every field (grids, det
  // bins, scalars, counters as doubles) and the device's uint64 counters; photons accumulate
  // here across smcrt_multi_accumulate calls until smcrt_multi_collect reduces them
  std::vector<double*> d_buf;
  std::vector<unsigned long long*> d_ctr;
  smcrt_pack_layout layout{};
  Offsets o;
  smcrt_grid grid{};
  int64_t n_det_bins = 0;
  std::vector<uint64_t> photons;  // photons each device ran since the last collect
  std::mutex mu;
};

extern "C" {

int smcrt_pack_size(const smcrt_pack_layout* layout, int64_t* n) {
  if (!layout_ok(layout) || !n) return fail(SMCRT_ERR_INVALID_ARG, "bad pack layout");
  *n = offsets(*layout).total;
  return SMCRT_OK;
}

int smcrt_pack_host(const smcrt_pack_layout* layout, const smcrt_tallies* t, double* buf) {
  if (!layout_ok(layout) || !t || !buf) return fail(SMCRT_ERR_INVALID_ARG, "bad pack arguments");
  const Offsets o = offsets(*layout);
  std::fill(buf, buf + o.total, 0.0);
  const int64_t nv = layout->n_voxels;
  const float* gf[3] = {t->jmean, t->absorb, t->emission};
  const double* gd[3] = {t->jmean_f64, t->absorb_f64, t->emission_f64};
  const int64_t go[3] = {o.jmean, o.absorb, o.emission};
  for (int k = 0; k < 3; ++k) {
    if (go[k] < 0) continue;
    double* d = buf + go[k];
    if (gd[k]) std::copy(gd[k], gd[k] + nv, d);
    else if (gf[k]) for (int64_t i = 0; i < nv; ++i) d[i] = (double)gf[k][i];
  }
  if (o.det >= 0 && t->det_bins) std::copy(t->det_bins, t->det_bins + layout->n_det_bins, buf + o.det);
  if (t->nscatt) buf[o.nscatt] = *t->nscatt;
  if (t->moments) std::copy(t->moments, t->moments + 24, buf + o.moments);
  if (t->counters)
    for (int i = 0; i < SMCRT_NCOUNTERS; ++i) buf[o.counters + i] = (double)t->counters[i];
  return SMCRT_OK;
}

int smcrt_unpack_host(const smcrt_pack_layout* layout, const double* buf, smcrt_tallies* t) {
  if (!layout_ok(layout) || !t || !buf) return fail(SMCRT_ERR_INVALID_ARG, "bad unpack arguments");
  const Offsets o = offsets(*layout);
  const int64_t nv = layout->n_voxels;
  float* gf[3] = {t->jmean, t->absorb, t->emission};
  double* gd[3] = {t->jmean_f64, t->absorb_f64, t->emission_f64};
  const int64_t go[3] = {o.jmean, o.absorb, o.emission};
  for (int k = 0; k < 3; ++k) {
    if (go[k] < 0) continue;
    const double* s = buf + go[k];
    for (int64_t i = 0; i < nv; ++i) {  // as run_sync accumulates a run's totals
      if (gf[k]) gf[k][i] = (float)((double)gf[k][i] + s[i]);
      if (gd[k]) gd[k][i] += s[i];
    }
  }
  if (o.det >= 0 && t->det_bins)
    for (int64_t i = 0; i < layout->n_det_bins; ++i) t->det_bins[i] += buf[o.det + i];
  if (t->nscatt) *t->nscatt += buf[o.nscatt];
  if (t->moments)
    for (int i = 0; i < 24; ++i) t->moments[i] += buf[o.moments + i];
  if (t->counters)
    for (int i = 0; i < SMCRT_NCOUNTERS; ++i) t->counters[i] += (uint64_t)buf[o.counters + i];
  return SMCRT_OK;
}

// ------------------------------------------------------------------ one process per GPU ----
int smcrt_comm_unique_id(uint8_t* id) {
  g_last_error.clear();
  if (!id) return fail(SMCRT_ERR_INVALID_ARG, "id is NULL");
  const Rccl& R = rccl();
  if (!R.ok) return fail(SMCRT_ERR_RCCL, R.err);
  ncclUniqueId u;
  NCCLCHK(R.get_unique_id(&u));
  static_assert(sizeof(u) == SMCRT_UNIQUE_ID_BYTES, "ncclUniqueId size");
  std::memcpy(id, &u, sizeof u);
  return SMCRT_OK;
}

int smcrt_comm_init_rank(const uint8_t* id, int32_t n_ranks, int32_t rank, int32_t device, smcrt_comm** out) {
  g_last_error.clear();
  if (!id || !out || n_ranks < 1 || rank < 0 || rank >= n_ranks) return fail(SMCRT_ERR_INVALID_ARG, "bad comm arguments");
  *out = nullptr;
  const Rccl& R = rccl();
  if (!R.ok) return fail(SMCRT_ERR_RCCL, R.err);
  HIPCHK(hipSetDevice(device));
  ncclUniqueId u;
  std::memcpy(&u, id, sizeof u);
  ncclComm_t c = nullptr;
  NCCLCHK(R.comm_init_rank(&c, n_ranks, u, rank));
  smcrt_comm* cm = new smcrt_comm();
  cm->comm = c;
  cm->n_ranks = n_ranks;
  cm->rank = rank;
  cm->device = device;
  *out = cm;
  return SMCRT_OK;
}

int smcrt_comm_info(const smcrt_comm* cm, int32_t* n_ranks, int32_t* rank, int32_t* device) {
  g_last_error.clear();
  if (!cm) return fail(SMCRT_ERR_INVALID_ARG, "comm is NULL");
  int n = cm->n_ranks, r = cm->rank;
  const Rccl& R = rccl();
  if (R.ok && R.comm_count) NCCLCHK(R.comm_count(cm->comm, &n));  // what the communicator itself reports
  if (R.ok && R.comm_user_rank) NCCLCHK(R.comm_user_rank(cm->comm, &r));
  if (n_ranks) *n_ranks = n;
  if (rank) *rank = r;
  if (device) *device = cm->device;
  return SMCRT_OK;
}

void smcrt_comm_destroy(smcrt_comm* cm) {
  if (!cm) return;
  (void)hipSetDevice(cm->device);
  if (cm->d_buf) (void)hipFree(cm->d_buf);
  if (cm->comm && rccl().ok) (void)rccl().comm_destroy(cm->comm);
  delete cm;
}

int smcrt_reduce_device_tallies(smcrt_scene* scene, smcrt_comm* cm, smcrt_device_tallies* dev, int32_t root,
                                void* stream) {
  g_last_error.clear();
  if (!scene || !cm || !dev) return fail(SMCRT_ERR_INVALID_ARG, "NULL argument");
  if (root >= cm->n_ranks) return fail(SMCRT_ERR_INVALID_ARG, "root out of range");
  if (smcrt::scene_device(scene) != cm->device) return fail(SMCRT_ERR_INVALID_ARG, "scene and comm are on different devices");
  const Rccl& R = rccl();
  if (!R.ok) return fail(SMCRT_ERR_RCCL, R.err);
  smcrt_grid g;
  int st = smcrt_scene_info(scene, &g, nullptr, nullptr);
  if (st) return st;
  smcrt_pack_layout L{};
  L.n_voxels = (int64_t)g.nx * g.ny * g.nz;
  if ((st = smcrt_scene_det_bins(scene, &L.n_det_bins))) return st;
  L.fields = (dev->jmean ? SMCRT_PACK_JMEAN : 0u) | (dev->absorb ? SMCRT_PACK_ABSORB : 0u) |
             (dev->emission ? SMCRT_PACK_EMISSION : 0u) | (dev->det_bins ? SMCRT_PACK_DET_BINS : 0u);
  const Offsets o = offsets(L);
  HIPCHK(hipSetDevice(cm->device));
  hipStream_t s = (hipStream_t)stream;
  if ((size_t)o.total > cm->cap) {
    HIPCHK(hipStreamSynchronize(s));  // the old buffer may still be in use on the stream
    if (cm->d_buf) HIPCHK(hipFree(cm->d_buf));
    cm->d_buf = nullptr;
    cm->cap = 0;
    HIPCHK(hipMalloc((void**)&cm->d_buf, sizeof(double) * (size_t)o.total));
    cm->cap = (size_t)o.total;
  }
  double* B = cm->d_buf;
  const Span spans[] = {{dev->jmean, o.jmean, L.n_voxels},   {dev->absorb, o.absorb, L.n_voxels},
                        {dev->emission, o.emission, L.n_voxels}, {dev->det_bins, o.det, L.n_det_bins},
                        {dev->nscatt, o.nscatt, 1},          {dev->moments, o.moments, 24}};
  HIPCHK(hipMemsetAsync(B + o.nscatt, 0, sizeof(double) * (size_t)(o.total - o.nscatt), s));
  for (const Span& sp : spans)
    if (sp.dev && sp.off >= 0 && sp.n > 0)
      HIPCHK(hipMemcpyAsync(B + sp.off, sp.dev, sizeof(double) * (size_t)sp.n, hipMemcpyDeviceToDevice, s));
  hipLaunchKernelGGL(counters_to_f64, dim3(1), dim3(64), 0, s, (const unsigned long long*)dev->counters,
                     B + o.counters);
  HIPCHK(hipGetLastError());
  if (root < 0) NCCLCHK(R.all_reduce(B, B, (size_t)o.total, ncclFloat64, ncclSum, cm->comm, s));
  else NCCLCHK(R.reduce(B, B, (size_t)o.total, ncclFloat64, ncclSum, root, cm->comm, s));
  if (root < 0 || root == cm->rank) {
    for (const Span& sp : spans)
      if (sp.dev && sp.off >= 0 && sp.n > 0)
        HIPCHK(hipMemcpyAsync(sp.dev, B + sp.off, sizeof(double) * (size_t)sp.n, hipMemcpyDeviceToDevice, s));
    if (dev->counters) {
      hipLaunchKernelGGL(counters_from_f64, dim3(1), dim3(64), 0, s, (const double*)(B + o.counters),
                         (unsigned long long*)dev->counters);
      HIPCHK(hipGetLastError());
    }
  }
  return SMCRT_OK;
}

// ------------------------------------------------------------------ one process, n GPUs ----
void smcrt_multi_destroy(smcrt_multi* m) {
  if (!m) return;
  for (smcrt_scene* s : m->scenes) smcrt_scene_destroy(s);  // (waits for its launches first)
  for (size_t i = 0; i < m->devices.size(); ++i) {
    (void)hipSetDevice(m->devices[i]);
    if (i < m->d_buf.size() && m->d_buf[i]) (void)hipFree(m->d_buf[i]);
    if (i < m->d_ctr.size() && m->d_ctr[i]) (void)hipFree(m->d_ctr[i]);
  }
  for (ncclComm_t c : m->comms)
    if (c && rccl().ok) (void)rccl().comm_destroy(c);
  delete m;
}

int smcrt_multi_create(const smcrt_sdf_node* nodes, int32_t n_nodes, const int32_t* top, int32_t n_top,
                       const smcrt_grid* grid, const smcrt_detector* dets, int32_t n_dets, const int32_t* devices,
                       int32_t n_devices, smcrt_multi** out) {
  g_last_error.clear();
  if (!out) return fail(SMCRT_ERR_INVALID_ARG, "out is NULL");
  *out = nullptr;
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) return fail(SMCRT_ERR_NO_DEVICE, "no HIP device");
  std::vector<int32_t> devs;
  if (devices && n_devices > 0) devs.assign(devices, devices + n_devices);
  else for (int32_t i = 0; i < (n_devices > 0 ? n_devices : ndev); ++i) devs.push_back(i);
  for (size_t i = 0; i < devs.size(); ++i) {
    if (devs[i] < 0 || devs[i] >= ndev) return fail(SMCRT_ERR_INVALID_ARG, "device ordinal out of range");
    for (size_t j = 0; j < i; ++j)
      if (devs[j] == devs[i]) return fail(SMCRT_ERR_INVALID_ARG, "a device is listed twice");
  }
  const Rccl& R = rccl();
  if (!R.ok) return fail(SMCRT_ERR_RCCL, R.err);
  smcrt_multi* m = new smcrt_multi();
  m->devices = devs;
  m->grid = *grid;
  auto bail = [&](int code) {
    const std::string msg = g_last_error;
    smcrt_multi_destroy(m);
    g_last_error = msg;
    return code;
  };
  for (int32_t d : devs) {
    smcrt_scene* s = nullptr;
    const int st = smcrt_scene_create(nodes, n_nodes, top, n_top, grid, dets, n_dets, d, &s);
    if (st) return bail(st);
    m->scenes.push_back(s);
  }
  if (smcrt_scene_det_bins(m->scenes[0], &m->n_det_bins)) return bail(SMCRT_ERR_INVALID_ARG);
  m->comms.assign(devs.size(), nullptr);
  const ncclResult_t r = R.comm_init_all(m->comms.data(), (int)devs.size(), devs.data());
  if (r != ncclSuccess) {
    std::fill(m->comms.begin(), m->comms.end(), nullptr);
    return bail(fail(SMCRT_ERR_RCCL, std::string("ncclCommInitAll failed: ") + R.error_string(r)));
  }
  m->layout.n_voxels = (int64_t)grid->nx * grid->ny * grid->nz;
  m->layout.n_det_bins = m->n_det_bins;
  m->layout.fields = SMCRT_PACK_JMEAN | SMCRT_PACK_ABSORB | SMCRT_PACK_EMISSION |
                     (m->n_det_bins > 0 ? SMCRT_PACK_DET_BINS : 0u);
  m->o = offsets(m->layout);
  m->d_buf.assign(devs.size(), nullptr);
  m->d_ctr.assign(devs.size(), nullptr);
  m->photons.assign(devs.size(), 0);
  for (size_t g = 0; g < devs.size(); ++g) {
    if (hipSetDevice(devs[g]) != hipSuccess ||
        hipMalloc((void**)&m->d_buf[g], sizeof(double) * (size_t)m->o.total) != hipSuccess ||
        hipMalloc((void**)&m->d_ctr[g], sizeof(unsigned long long) * SMCRT_NCOUNTERS) != hipSuccess ||
        hipMemset(m->d_buf[g], 0, sizeof(double) * (size_t)m->o.total) != hipSuccess ||
        hipMemset(m->d_ctr[g], 0, sizeof(unsigned long long) * SMCRT_NCOUNTERS) != hipSuccess) {
      (void)hipGetLastError();
      return bail(fail(SMCRT_ERR_OOM, "multi: device accumulators could not be allocated"));
    }
  }
  *out = m;
  return SMCRT_OK;
}

int smcrt_multi_info(const smcrt_multi* m, int32_t* n) {
  if (!m || !n) return fail(SMCRT_ERR_INVALID_ARG, "NULL argument");
  *n = (int32_t)m->devices.size();
  return SMCRT_OK;
}

smcrt_scene* smcrt_multi_scene(smcrt_multi* m, int32_t i) {
  if (!m || i < 0 || i >= (int32_t)m->scenes.size()) return nullptr;
  return m->scenes[(size_t)i];
}

// The device tallies of slot g (pointers into its packed accumulator).
static smcrt_device_tallies device_tallies(const smcrt_multi* m, size_t g) {
  smcrt_device_tallies dt;
  std::memset(&dt, 0, sizeof dt);
  double* B = m->d_buf[g];
  const Offsets& o = m->o;
  dt.jmean = B + o.jmean;
  dt.absorb = B + o.absorb;
  dt.emission = B + o.emission;
  if (o.det >= 0) dt.det_bins = B + o.det;
  dt.nscatt = B + o.nscatt;
  dt.moments = B + o.moments;
  dt.counters = (uint64_t*)m->d_ctr[g];
  return dt;
}

// Throw away everything accumulated since the last collect (after a failed launch): wait for
// every device, zero its accumulators and photon count, so that a later collect never adds
// partial tallies whose photons no caller counted.
static void discard_locked(smcrt_multi* m) {
  for (size_t g = 0; g < m->devices.size(); ++g) {
    if (hipSetDevice(m->devices[g]) != hipSuccess) continue;
    (void)hipDeviceSynchronize();
    if (m->d_buf[g]) (void)hipMemset(m->d_buf[g], 0, sizeof(double) * (size_t)m->o.total);
    if (m->d_ctr[g]) (void)hipMemset(m->d_ctr[g], 0, sizeof(unsigned long long) * SMCRT_NCOUNTERS);
    m->photons[g] = 0;
  }
}

// Photons [first, first + n) in chunks handed to whichever device has a free launch slot
// (guided: a chunk is half of what is left per device, at least `min_chunk`), each an
// overlapped smcrt_run_device into that device's accumulators. A chunk's results do not
// depend on the device it lands on (Philox streams keyed by the global photon index), so a
// tail-bound scene keeps every GPU busy until the end instead of waiting for the slowest of
// n static shards. Returns when every chunk is launched; nothing is waited for.
static int accumulate_locked(smcrt_multi* m, const smcrt_source* src, const smcrt_run_config* cfg) {
  if (cfg->flags & SMCRT_FLAG_RECORD_PHOTONS)
    return fail(SMCRT_ERR_INVALID_ARG, "photon records are not kept by the multi-GPU path (use smcrt_run)");
  const size_t n = m->devices.size();
  uint64_t min_chunk = 1ull << 20;
  if (const char* e = std::getenv("SMCRT_MULTI_CHUNK")) min_chunk = std::max<uint64_t>(1, std::strtoull(e, nullptr, 10));
  smcrt_run_config c = *cfg;
  c.flags = (cfg->flags | SMCRT_FLAG_OVERLAP | SMCRT_FLAG_ASYNC_FOLD) & ~(uint32_t)SMCRT_FLAG_RECORD_PHOTONS;
  const uint64_t N = cfg->n_photons;
  uint64_t issued = 0;
  while (issued < N) {
    bool launched = false;
    for (size_t g = 0; g < n && issued < N; ++g) {
      smcrt_scene* s = m->scenes[g];
      if (smcrt::scene_inflight(s) >= smcrt::scene_depth(s)) continue;
      const uint64_t rem = N - issued;
      uint64_t k = std::max<uint64_t>(min_chunk, rem / (2 * n));
      if (k > rem) k = rem;
      c.n_photons = k;
      c.first_photon = cfg->first_photon + issued;
      smcrt_device_tallies dt = device_tallies(m, g);
      const int rs = smcrt_run_device(s, src, &c, &dt, smcrt::scene_stream(s));
      if (rs) {  // (the chunks already launched would leave partial tallies behind)
        const std::string msg = g_last_error;
        discard_locked(m);
        return fail(rs, msg + " (smcrt_multi_accumulate: the photons accumulated since the last collect were discarded)");
      }
      m->photons[g] += k;
      issued += k;
      launched = true;
    }
    if (!launched) std::this_thread::sleep_for(std::chrono::microseconds(200));
  }
  return SMCRT_OK;
}

// One packed RCCL reduce of every device's accumulators onto the first device, added into
// `io` as smcrt_run adds a run's totals; the accumulators are zeroed for the next photons.
static int collect_locked(smcrt_multi* m, smcrt_tallies* io) {
  const Rccl& R = rccl();
  if (!R.ok) return fail(SMCRT_ERR_RCCL, R.err);
  const size_t n = m->devices.size();
  const Offsets& o = m->o;
  for (size_t g = 0; g < n; ++g) {
    smcrt_scene* s = m->scenes[g];
    hipStream_t st = (hipStream_t)smcrt::scene_stream(s);
    const int fs = smcrt_scene_fence(s, st);  // every launch and fold of this device
    if (fs) return fs;
    HIPCHK(hipSetDevice(m->devices[g]));
    hipLaunchKernelGGL(counters_to_f64, dim3(1), dim3(64), 0, st, (const unsigned long long*)m->d_ctr[g],
                       m->d_buf[g] + o.counters);
    HIPCHK(hipGetLastError());
  }
  NCCLCHK(R.group_start());
  for (size_t g = 0; g < n; ++g) {
    HIPCHK(hipSetDevice(m->devices[g]));
    NCCLCHK(R.reduce(m->d_buf[g], m->d_buf[g], (size_t)o.total, ncclFloat64, ncclSum, 0, m->comms[g],
                     (hipStream_t)smcrt::scene_stream(m->scenes[g])));
  }
  NCCLCHK(R.group_end());
  for (size_t g = n; g-- > 0;) {  // root last: its copy is the sum
    HIPCHK(hipSetDevice(m->devices[g]));
    const hipError_t e = hipStreamSynchronize((hipStream_t)smcrt::scene_stream(m->scenes[g]));
    if (e != hipSuccess)
      return fail(SMCRT_ERR_DEVICE_FAULT, std::string("device ") + std::to_string(m->devices[g]) + ": " +
                                              hipGetErrorString(e));
  }
  for (size_t g = 0; g < n; ++g) {  // the watchdog of every device's launches (smcrt_scene_check)
    const int ws = smcrt_scene_check(m->scenes[g]);
    if (ws) return ws;
  }
  std::vector<double> h((size_t)o.total);
  HIPCHK(hipSetDevice(m->devices[0]));
  HIPCHK(hipMemcpy(h.data(), m->d_buf[0], sizeof(double) * h.size(), hipMemcpyDeviceToHost));
  for (size_t g = 0; g < n; ++g) {
    hipStream_t st = (hipStream_t)smcrt::scene_stream(m->scenes[g]);
    HIPCHK(hipSetDevice(m->devices[g]));
    HIPCHK(hipMemsetAsync(m->d_buf[g], 0, sizeof(double) * (size_t)o.total, st));
    HIPCHK(hipMemsetAsync(m->d_ctr[g], 0, sizeof(unsigned long long) * SMCRT_NCOUNTERS, st));
    m->photons[g] = 0;
  }
  return smcrt_unpack_host(&m->layout, h.data(), io);  // (NULL tallies of io are skipped)
}

int smcrt_multi_accumulate(smcrt_multi* m, const smcrt_source* src, const smcrt_run_config* cfg) {
  g_last_error.clear();
  if (!m || !src || !cfg) return fail(SMCRT_ERR_INVALID_ARG, "NULL argument");
  std::lock_guard<std::mutex> guard(m->mu);
  return accumulate_locked(m, src, cfg);
}

int smcrt_multi_collect(smcrt_multi* m, smcrt_tallies* io) {
  g_last_error.clear();
  if (!m || !io) return fail(SMCRT_ERR_INVALID_ARG, "NULL argument");
  std::lock_guard<std::mutex> guard(m->mu);
  return collect_locked(m, io);
}

int smcrt_multi_device_photons(const smcrt_multi* m, uint64_t* photons) {
  if (!m || !photons) return fail(SMCRT_ERR_INVALID_ARG, "NULL argument");
  for (size_t g = 0; g < m->photons.size(); ++g) photons[g] = m->photons[g];
  return SMCRT_OK;
}

int smcrt_multi_run(smcrt_multi* m, const smcrt_source* src, const smcrt_run_config* cfg, smcrt_tallies* io) {
  g_last_error.clear();
  if (!m || !src || !cfg || !io) return fail(SMCRT_ERR_INVALID_ARG, "NULL argument");
  if ((cfg->flags & SMCRT_FLAG_RECORD_PHOTONS) && io->records)
    return fail(SMCRT_ERR_INVALID_ARG, "photon records are not kept by smcrt_multi_run (use smcrt_run)");
  std::lock_guard<std::mutex> guard(m->mu);
  smcrt_run_config c = *cfg;
  c.flags &= ~(uint32_t)SMCRT_FLAG_RECORD_PHOTONS;
  const int st = accumulate_locked(m, src, &c);
  if (st) return st;
  return collect_locked(m, io);
}

}  // extern "C"
