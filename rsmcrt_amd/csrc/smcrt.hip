// smcrt.hip — transport kernel and the C ABI of include/smcrt.h.
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
#include <cstring>
#include <mutex>
#include <string>
#include <vector>

#include "../../include/smcrt.h"
#include "transport.h"

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

__global__ __launch_bounds__(256) void transport_kernel(KParams K) {
  Lane L;
#pragma unroll
  for (int i = 0; i < SMCRT_NCOUNTERS; ++i) L.c.v[i] = 0;
  L.nscatt = 0.0;
  L.fault = false;
  const int lane = threadIdx.x & 63;
  const bool rec_on = (K.flags & SMCRT_FLAG_RECORD_PHOTONS) && K.records;
  for (;;) {
    unsigned long long base = 0;
    if (lane == 0) base = atomicAdd(K.queue, 64ull);
    base = __shfl(base, 0, 64);
    if (base >= K.n_photons) break;
    const uint64_t j = base + (uint64_t)lane;
    if (j < K.n_photons) run_photon(K, L, K.first_photon + j, rec_on ? K.records + j : nullptr);
  }
  if (K.counters) {
#pragma unroll
    for (int i = 0; i < SMCRT_NCOUNTERS; ++i) {
      const uint32_t s = wave_sum_u32(L.c.v[i]);
      if (lane == 0 && s) atomicAdd(K.counters + i, (unsigned long long)s);
    }
  }
  if (K.nscatt) {
    const double s = wave_sum_f64(L.nscatt);
    if (lane == 0 && s != 0.0) atomic_add_nr(K.nscatt, s);
  }
}

// ------------------------------------------------------------------ host side ------
namespace {

thread_local std::string g_err;

int fail(int code, const std::string& msg) {
  g_err = msg;
  return code;
}

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
  int32_t* d_top = nullptr;
  TopProps* d_props = nullptr;
  double* d_faces = nullptr;
  smcrt_detector* d_dets = nullptr;
  int64_t* d_det_off = nullptr;
  unsigned long long* d_queue = nullptr;
  // tallies owned by the scene for the synchronous smcrt_run
  double* d_grids = nullptr;  // jmean | absorb | emission
  double* d_small = nullptr;  // det bins | nscatt | moments(24)
  unsigned long long* d_counters = nullptr;
  smcrt_photon_record* d_records = nullptr;
  size_t records_cap = 0;
  hipStream_t stream = nullptr;
  int grid_blocks = 0;
  std::mutex mu;
};

static TopProps make_props(const smcrt_sdf_node& nd) {
  TopProps p;  // init_mono, opticalProperties.f90:107-125
  p.kappa = nd.mus + nd.mua;
  p.albedo = (nd.mua < 1e-9) ? 1.0 : nd.mus / p.kappa;
  p.hgg = nd.hgg;
  p.n = nd.n;
  return p;
}

extern "C" {

int smcrt_abi_version(void) { return SMCRT_ABI_VERSION; }

const char* smcrt_last_error(void) { return g_err.c_str(); }

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
  void* ptrs[] = {s->d_nodes, s->d_top, s->d_props, s->d_faces, s->d_dets, s->d_det_off,
                  s->d_queue, s->d_grids, s->d_small, s->d_counters, s->d_records};
  for (void* p : ptrs)
    if (p) (void)hipFree(p);
  if (s->stream) (void)hipStreamDestroy(s->stream);
  delete s;
}

int smcrt_scene_create(const smcrt_sdf_node* nodes, int32_t n_nodes, const int32_t* top, int32_t n_top,
                       const smcrt_grid* grid, const smcrt_detector* dets, int32_t n_dets, int32_t device,
                       smcrt_scene** out) {
  g_err.clear();
  if (!out) return fail(SMCRT_ERR_INVALID_ARG, "out is NULL");
  *out = nullptr;
  if (!nodes || n_nodes < 1 || !top || n_top < 1 || !grid || n_dets < 0 || (n_dets > 0 && !dets))
    return fail(SMCRT_ERR_INVALID_ARG, "bad scene arguments");
  if (grid->nx < 1 || grid->ny < 1 || grid->nz < 1 || !(grid->xmax > 0) || !(grid->ymax > 0) ||
      !(grid->zmax > 0))
    return fail(SMCRT_ERR_INVALID_ARG, "grid dimensions must be positive");
  for (int32_t i = 0; i < n_nodes; ++i) {
    const smcrt_sdf_node& nd = nodes[i];
    if (nd.kind < SMCRT_SDF_SPHERE || nd.kind > SMCRT_SDF_MODEL)
      return fail(SMCRT_ERR_INVALID_ARG, "node " + std::to_string(i) + ": unknown SDF kind");
    if (nd.kind == SMCRT_SDF_MODEL) {
      if (nd.n_children < 1 || nd.first_child < 0 || nd.first_child + nd.n_children > n_nodes)
        return fail(SMCRT_ERR_INVALID_ARG, "model node " + std::to_string(i) + ": bad child range");
      if (nd.op < SMCRT_OP_UNION || nd.op > SMCRT_OP_INTERSECTION)
        return fail(SMCRT_ERR_INVALID_ARG, "model node " + std::to_string(i) + ": bad CSG op");
      for (int32_t c = 0; c < nd.n_children; ++c)
        if (nodes[nd.first_child + c].kind == SMCRT_SDF_MODEL)
          return fail(SMCRT_ERR_UNSUPPORTED, "nested models are not supported");
    }
  }
  for (int32_t i = 0; i < n_top; ++i)
    if (top[i] < 0 || top[i] >= n_nodes) return fail(SMCRT_ERR_INVALID_ARG, "top index out of range");
  for (int32_t i = 0; i < n_dets; ++i) {
    if (dets[i].kind == SMCRT_DET_FIBRE) return fail(SMCRT_ERR_UNSUPPORTED, "fibre detector not supported");
    if (dets[i].kind < SMCRT_DET_CIRCLE || dets[i].kind > SMCRT_DET_CAMERA || dets[i].nbins < 1)
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
    std::string msg = g_err;
    smcrt_scene_destroy(s);
    g_err = msg;
    return code;
  };
  if (hipSetDevice(device) != hipSuccess) return cleanup_fail(fail(SMCRT_ERR_HIP, "hipSetDevice failed"));
  int st;
  if ((st = dalloc(&s->d_nodes, n_nodes)) || (st = dalloc(&s->d_top, n_top)) || (st = dalloc(&s->d_props, n_top)) ||
      (st = dalloc(&s->d_faces, faces.size())) || (st = dalloc(&s->d_dets, std::max(1, n_dets))) ||
      (st = dalloc(&s->d_det_off, (size_t)n_dets + 1)) || (st = dalloc(&s->d_queue, 1)) ||
      (st = dalloc(&s->d_counters, SMCRT_NCOUNTERS)) ||
      (st = dalloc(&s->d_small, (size_t)s->det_total + 1 + 24)))
    return cleanup_fail(st);
  hipError_t e = hipSuccess;
  if (e == hipSuccess) e = hipMemcpy(s->d_nodes, nodes, sizeof(smcrt_sdf_node) * n_nodes, hipMemcpyHostToDevice);
  if (e == hipSuccess) e = hipMemcpy(s->d_top, top, sizeof(int32_t) * n_top, hipMemcpyHostToDevice);
  if (e == hipSuccess) e = hipMemcpy(s->d_props, s->h_props.data(), sizeof(TopProps) * n_top, hipMemcpyHostToDevice);
  if (e == hipSuccess) e = hipMemcpy(s->d_faces, faces.data(), sizeof(double) * faces.size(), hipMemcpyHostToDevice);
  if (e == hipSuccess && n_dets)
    e = hipMemcpy(s->d_dets, dets, sizeof(smcrt_detector) * n_dets, hipMemcpyHostToDevice);
  if (e == hipSuccess)
    e = hipMemcpy(s->d_det_off, s->h_det_off.data(), sizeof(int64_t) * (n_dets + 1), hipMemcpyHostToDevice);
  if (e == hipSuccess) e = hipStreamCreateWithFlags(&s->stream, hipStreamNonBlocking);
  if (e != hipSuccess) return cleanup_fail(fail(SMCRT_ERR_HIP, std::string("scene upload: ") + hipGetErrorString(e)));
  int per_cu = 0, cus = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, transport_kernel, 256, 0) != hipSuccess || per_cu < 1)
    per_cu = 1;
  if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device) != hipSuccess || cus < 1) cus = 256;
  s->grid_blocks = cus * per_cu;
  *out = s;
  return SMCRT_OK;
}

int smcrt_scene_det_bins(const smcrt_scene* s, int64_t* n) {
  if (!s || !n) return fail(SMCRT_ERR_INVALID_ARG, "NULL argument");
  *n = s->det_total;
  return SMCRT_OK;
}

int smcrt_scene_set_optprops(smcrt_scene* s, int32_t i, double mus, double mua, double hgg, double n) {
  if (!s || i < 0 || i >= s->n_top) return fail(SMCRT_ERR_INVALID_ARG, "bad scene or index");
  std::lock_guard<std::mutex> g(s->mu);
  smcrt_sdf_node& nd = s->h_nodes[s->h_top[i]];
  nd.mus = mus; nd.mua = mua; nd.hgg = hgg; nd.n = n;
  s->h_props[i] = make_props(nd);
  HIPCHK(hipSetDevice(s->device));
  HIPCHK(hipMemcpyAsync(s->d_props + i, &s->h_props[i], sizeof(TopProps), hipMemcpyHostToDevice, s->stream));
  HIPCHK(hipStreamSynchronize(s->stream));
  return SMCRT_OK;
}

static int launch(smcrt_scene* s, const smcrt_source* src, const smcrt_run_config* cfg,
                  const smcrt_device_tallies& dt, hipStream_t stream) {
  if (src->kind < SMCRT_SRC_POINT || src->kind > SMCRT_SRC_PENCIL) return fail(SMCRT_ERR_INVALID_ARG, "bad source kind");
  if (cfg->n_photons == 0) return SMCRT_OK;
  KParams K;
  K.nodes = s->d_nodes;
  K.top = s->d_top;
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
  K.src = *src;
  K.n_photons = cfg->n_photons;
  K.first_photon = cfg->first_photon;
  K.seed = cfg->seed;
  K.jmean = dt.jmean; K.absorb = dt.absorb; K.emission = dt.emission;
  K.det_bins = dt.det_bins; K.nscatt = dt.nscatt; K.moments = dt.moments;
  K.counters = (unsigned long long*)dt.counters;
  K.records = dt.records;
  K.queue = s->d_queue;
  HIPCHK(hipMemsetAsync(s->d_queue, 0, sizeof(unsigned long long), stream));
  const uint64_t waves_needed = (cfg->n_photons + 63) / 64;
  const uint64_t blocks_needed = (waves_needed + 3) / 4;
  const int blocks = (int)std::min<uint64_t>((uint64_t)s->grid_blocks, std::max<uint64_t>(1, blocks_needed));
  hipLaunchKernelGGL(transport_kernel, dim3(blocks), dim3(256), 0, stream, K);
  HIPCHK(hipGetLastError());
  return SMCRT_OK;
}

int smcrt_run_device(smcrt_scene* s, const smcrt_source* src, const smcrt_run_config* cfg,
                     smcrt_device_tallies* dev, void* stream) {
  g_err.clear();
  if (!s || !src || !cfg || !dev) return fail(SMCRT_ERR_INVALID_ARG, "NULL argument");
  std::lock_guard<std::mutex> g(s->mu);
  HIPCHK(hipSetDevice(s->device));
  return launch(s, src, cfg, *dev, (hipStream_t)stream);
}

int smcrt_run(smcrt_scene* s, const smcrt_source* src, const smcrt_run_config* cfg, smcrt_tallies* io) {
  g_err.clear();
  if (!s || !src || !cfg || !io) return fail(SMCRT_ERR_INVALID_ARG, "NULL argument");
  std::lock_guard<std::mutex> g(s->mu);
  HIPCHK(hipSetDevice(s->device));
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
  int st = launch(s, src, cfg, dt, s->stream);
  if (st) return st;
  hipError_t e = hipStreamSynchronize(s->stream);
  if (e != hipSuccess) return fail(SMCRT_ERR_DEVICE_FAULT, std::string("transport kernel: ") + hipGetErrorString(e));
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
