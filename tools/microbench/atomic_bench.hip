// Microbenchmark: scattered atomic-add throughput into a 128^3 tally grid on gfx950.
// Question it answers: which accumulation form should the fluence deposition use?
//   agent-scope atomics (one shared grid) vs workgroup-scope atomics into per-XCD replicas,
//   f32 vs f64 vs u64 fixed point, random voxels vs ray-walk (DDA-like) voxel sequences,
//   linear (x-fastest) vs 4x4x4-bricked layout.
// Build: hipcc --offload-arch=gfx950 -O3 atomic_bench.hip -o atomic_bench
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <vector>
#include <cstring>

#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { \
  printf("HIP error %s at %s:%d\n", hipGetErrorString(e), __FILE__, __LINE__); return 1; } } while (0)

constexpr int N = 128;
constexpr int NV = N * N * N;

__device__ __forceinline__ uint32_t hash32(uint32_t x) {
  x ^= x >> 16; x *= 0x7feb352dU; x ^= x >> 15; x *= 0x846ca68bU; x ^= x >> 16; return x;
}

__device__ __forceinline__ int xcc_id() {
  // HW_REG_XCC_ID = 20, bits [3:0]
  return __builtin_amdgcn_s_getreg((3 << 11) | (0 << 6) | 20) & 7;
}

__device__ __forceinline__ uint32_t lin(int i, int j, int k) { return (uint32_t)i + N * ((uint32_t)j + N * (uint32_t)k); }
__device__ __forceinline__ uint32_t brick(int i, int j, int k) {
  // 4x4x4 bricks of 64 voxels (256 B of f32), bricks laid x-fastest
  uint32_t b = (uint32_t)(i >> 2) + (N / 4) * ((uint32_t)(j >> 2) + (N / 4) * (uint32_t)(k >> 2));
  return b * 64 + (i & 3) + 4 * ((j & 3) + 4 * (k & 3));
}

enum { T_F32 = 0, T_F64 = 1, T_U64 = 2 };
enum { S_AGENT = 0, S_WG_XCD = 1 };
enum { A_RANDOM = 0, A_WALK = 1, A_WALK_BRICK = 2 };

template <int TY, int SC, int AC>
__global__ __launch_bounds__(256) void kbench(void* grid, int iters) {
  const uint32_t tid = blockIdx.x * blockDim.x + threadIdx.x;
  size_t rep = 0;
  if constexpr (SC == S_WG_XCD) rep = (size_t)xcc_id() * NV;
  uint32_t h = hash32(tid * 0x9E3779B9u + 17u);
  int ci = h & (N - 1), cj = (h >> 7) & (N - 1), ck = (h >> 14) & (N - 1);
  int axis_seq = 0;
  for (int it = 0; it < iters; ++it) {
    uint32_t idx;
    if constexpr (AC == A_RANDOM) {
      h = hash32(h + it);
      idx = h & (NV - 1);
    } else {
      // ray-walk: step one voxel along an axis chosen from a slowly varying random sequence
      if ((it & 15) == 0) { h = hash32(h + 0x1234567u); axis_seq = h; }
      int ax = (axis_seq >> (2 * (it & 15))) & 3; if (ax == 3) ax = 0;
      int sg = ((h >> 30) & 1) ? 1 : -1;
      if (ax == 0) ci = (ci + sg) & (N - 1); else if (ax == 1) cj = (cj + sg) & (N - 1); else ck = (ck + sg) & (N - 1);
      idx = (AC == A_WALK) ? lin(ci, cj, ck) : brick(ci, cj, ck);
    }
    if constexpr (TY == T_F32) {
      float* g = (float*)grid + rep;
      if constexpr (SC == S_AGENT) atomicAdd(g + idx, 1.0f);
      else __hip_atomic_fetch_add(g + idx, 1.0f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    } else if constexpr (TY == T_F64) {
      double* g = (double*)grid + rep;
      if constexpr (SC == S_AGENT) atomicAdd(g + idx, 1.0);
      else __hip_atomic_fetch_add(g + idx, 1.0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    } else {
      unsigned long long* g = (unsigned long long*)grid + rep;
      if constexpr (SC == S_AGENT) atomicAdd(g + idx, 1ull);
      else __hip_atomic_fetch_add(g + idx, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    }
  }
}

template <int TY, int SC, int AC>
int run(const char* name, void* dgrid, size_t bytes, int blocks, int iters) {
  CHECK(hipMemset(dgrid, 0, bytes));
  hipEvent_t a, b; CHECK(hipEventCreate(&a)); CHECK(hipEventCreate(&b));
  kbench<TY, SC, AC><<<blocks, 256>>>(dgrid, iters);  // warm
  CHECK(hipDeviceSynchronize());
  CHECK(hipMemset(dgrid, 0, bytes));
  const int reps = 5;
  CHECK(hipEventRecord(a));
  for (int r = 0; r < reps; ++r) kbench<TY, SC, AC><<<blocks, 256>>>(dgrid, iters);
  CHECK(hipEventRecord(b));
  CHECK(hipEventSynchronize(b));
  float ms = 0; CHECK(hipEventElapsedTime(&ms, a, b));
  double nadd = (double)blocks * 256 * iters * reps;
  // verify total
  size_t elems = bytes / (TY == T_F32 ? 4 : 8);
  double total = 0;
  if (TY == T_F32) { std::vector<float> h(elems); CHECK(hipMemcpy(h.data(), dgrid, bytes, hipMemcpyDeviceToHost)); for (auto v : h) total += v; }
  else if (TY == T_F64) { std::vector<double> h(elems); CHECK(hipMemcpy(h.data(), dgrid, bytes, hipMemcpyDeviceToHost)); for (auto v : h) total += v; }
  else { std::vector<unsigned long long> h(elems); CHECK(hipMemcpy(h.data(), dgrid, bytes, hipMemcpyDeviceToHost)); for (auto v : h) total += (double)v; }
  printf("%-28s %8.3f ms  %8.2f Gatomic/s  total_ok=%d\n", name, ms / reps, nadd / (ms * 1e-3) / 1e9, total == nadd ? 1 : 0);
  CHECK(hipEventDestroy(a)); CHECK(hipEventDestroy(b));
  return 0;
}

int main() {
  void* d; size_t maxbytes = (size_t)8 * NV * 8;
  CHECK(hipMalloc(&d, maxbytes));
  const int blocks = 256 * 8, iters = 256;
  size_t f32_1 = (size_t)NV * 4, f32_8 = 8 * f32_1, f64_1 = (size_t)NV * 8, f64_8 = 8 * f64_1;
  run<T_F32, S_AGENT, A_RANDOM>("f32 agent random", d, f32_1, blocks, iters);
  run<T_F32, S_WG_XCD, A_RANDOM>("f32 wg-xcd random", d, f32_8, blocks, iters);
  run<T_F32, S_AGENT, A_WALK>("f32 agent walk", d, f32_1, blocks, iters);
  run<T_F32, S_WG_XCD, A_WALK>("f32 wg-xcd walk", d, f32_8, blocks, iters);
  run<T_F32, S_AGENT, A_WALK_BRICK>("f32 agent walk-brick", d, f32_1, blocks, iters);
  run<T_F32, S_WG_XCD, A_WALK_BRICK>("f32 wg-xcd walk-brick", d, f32_8, blocks, iters);
  run<T_F64, S_AGENT, A_RANDOM>("f64 agent random", d, f64_1, blocks, iters);
  run<T_F64, S_WG_XCD, A_RANDOM>("f64 wg-xcd random", d, f64_8, blocks, iters);
  run<T_F64, S_AGENT, A_WALK_BRICK>("f64 agent walk-brick", d, f64_1, blocks, iters);
  run<T_F64, S_WG_XCD, A_WALK_BRICK>("f64 wg-xcd walk-brick", d, f64_8, blocks, iters);
  run<T_U64, S_AGENT, A_RANDOM>("u64 agent random", d, f64_1, blocks, iters);
  run<T_U64, S_WG_XCD, A_RANDOM>("u64 wg-xcd random", d, f64_8, blocks, iters);
  run<T_U64, S_AGENT, A_WALK_BRICK>("u64 agent walk-brick", d, f64_1, blocks, iters);
  run<T_U64, S_WG_XCD, A_WALK_BRICK>("u64 wg-xcd walk-brick", d, f64_8, blocks, iters);
  run<T_U64, S_WG_XCD, A_WALK>("u64 wg-xcd walk", d, f64_8, blocks, iters);
  CHECK(hipFree(d));
  return 0;
}
