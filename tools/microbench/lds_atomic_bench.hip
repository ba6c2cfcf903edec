// Microbenchmark: LDS atomic-add throughput of the fold's access pattern on gfx950 (bk_reduce:
// 1024 threads, one 16384-voxel tile accumulator in LDS, random voxel per record).
// Question: which LDS accumulation form is cheapest per record: ds_add_f64, ds_add_u64 (fixed
// point), ds_add_f32, ds_add_u32, or an fp64 accumulator split in two fp32 halves?
// Build: hipcc --offload-arch=gfx950 -O3 lds_atomic_bench.hip -o lds_atomic_bench
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { \
  printf("HIP error %s at %s:%d\n", hipGetErrorString(e), __FILE__, __LINE__); return 1; } } while (0)

constexpr int TV = 16384;

__device__ __forceinline__ uint32_t hash32(uint32_t x) {
  x ^= x >> 16; x *= 0x7feb352dU; x ^= x >> 15; x *= 0x846ca68bU; x ^= x >> 16; return x;
}

enum { T_F64 = 0, T_U64 = 1, T_F32 = 2, T_U32 = 3 };

template <int TY>
__global__ __launch_bounds__(1024) void kbench(double* out, int iters) {
  __shared__ double acc64[TV];
  float* acc32 = (float*)acc64;
  unsigned long long* accu = (unsigned long long*)acc64;
  uint32_t* accu32 = (uint32_t*)acc64;
  for (int i = threadIdx.x; i < TV; i += 1024) acc64[i] = 0.0;
  __syncthreads();
  uint32_t h = hash32(blockIdx.x * 1024 + threadIdx.x);
  for (int it = 0; it < iters; ++it) {
    h = hash32(h + it);
    const uint32_t v = h & (TV - 1);
    const float val = (float)(h >> 20) * 1e-6f;
    if constexpr (TY == T_F64) atomicAdd(&acc64[v], (double)val);
    else if constexpr (TY == T_U64) atomicAdd(&accu[v], (unsigned long long)(h >> 8));
    else if constexpr (TY == T_F32) atomicAdd(&acc32[v], val);
    else atomicAdd(&accu32[v], h >> 8);
  }
  __syncthreads();
  double s = 0.0;
  for (int i = threadIdx.x; i < TV; i += 1024) s += acc64[i];
  if (s == 12345.0) out[0] = s;
}

template <int TY>
int run(const char* name, double* d) {
  const int blocks = 256 * 4, iters = 4096;
  hipEvent_t a, b;
  CHECK(hipEventCreate(&a)); CHECK(hipEventCreate(&b));
  hipLaunchKernelGGL(kbench<TY>, dim3(blocks), dim3(1024), 0, 0, d, 16);
  CHECK(hipDeviceSynchronize());
  CHECK(hipEventRecord(a));
  hipLaunchKernelGGL(kbench<TY>, dim3(blocks), dim3(1024), 0, 0, d, iters);
  CHECK(hipEventRecord(b));
  CHECK(hipEventSynchronize(b));
  float ms = 0;
  CHECK(hipEventElapsedTime(&ms, a, b));
  const double n = (double)blocks * 1024 * iters;
  int dev = 0, cus = 0, khz = 0;
  hipGetDevice(&dev);
  hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
  hipDeviceGetAttribute(&khz, hipDeviceAttributeClockRate, dev);
  printf("%-4s %8.3f ms  %7.2f G atomics/s  %.3f per CU-cycle (%d CUs, %d MHz)\n", name, ms, n / ms * 1e-6,
         n / (ms * 1e-3) / cus / (khz * 1e3), cus, khz / 1000);
  return 0;
}

int main() {
  double* d;
  CHECK(hipMalloc(&d, 64));
  if (run<T_F64>("f64", d) || run<T_U64>("u64", d) || run<T_F32>("f32", d) || run<T_U32>("u32", d)) return 1;
  return 0;
}
