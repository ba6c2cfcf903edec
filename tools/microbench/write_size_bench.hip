// Microbenchmark: what WRITE_SIZE (rocprofv3, L2 memory-side write bytes) reports for the
// transport kernel's record stores, 8-byte stores filed into many slowly filling buckets.
// Kernels (R records of 8 B each, R * 8 bytes stored, no atomics: device-scope atomics are
// memory-side requests that WRITE_SIZE counts too):
//   contig   — each lane stores 8 B at consecutive addresses (a wave stores 512 B contiguous);
//   own<S>   — each lane fills its own 128-B line over 16 stores (lane g, store i: line
//              (i / 16) * lanes + g, slot i % 16), so every wave store touches 64 lines and
//              `lanes` lines (64 MiB) are partly written at any time, like the transport
//              kernel's open buckets; s_sleep(S) between stores sets how long a line takes to
//              fill (S = 0: fast; S = 96: ~40 us per line, the transport kernel's rate).
// Compare each kernel's WRITE_SIZE with R * 8 bytes: contig calibrates the counter for 8-B
// stores; own0 vs own96 separates a counting artefact of scattered 8-B stores from partly
// written lines leaving L2 before they are full.
// Build: hipcc --offload-arch=gfx950 -O3 write_size_bench.hip -o write_size_bench
// Run:   rocprofv3 --pmc WRITE_SIZE --kernel-trace -- ./write_size_bench
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { \
  printf("HIP error %s at %s:%d\n", hipGetErrorString(e), __FILE__, __LINE__); return 1; } } while (0)

__device__ __forceinline__ uint32_t hash32(uint32_t x) {
  x ^= x >> 16; x *= 0x7feb352dU; x ^= x >> 15; x *= 0x846ca68bU; x ^= x >> 16; return x;
}

__global__ __launch_bounds__(256) void contig(unsigned long long* out, uint64_t per_thread) {
  const uint64_t nthreads = (uint64_t)gridDim.x * blockDim.x;
  const uint64_t gid = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  for (uint64_t i = 0; i < per_thread; ++i) out[i * nthreads + gid] = gid ^ i;
}

template <int S>
__global__ __launch_bounds__(256) void own_lines(unsigned long long* out, uint32_t per_thread) {
  const uint64_t lanes = (uint64_t)gridDim.x * blockDim.x;
  const uint64_t gid = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  for (uint32_t i = 0; i < per_thread; ++i) {
    if (S > 0) __builtin_amdgcn_s_sleep(S);
    out[((uint64_t)(i >> 4) * lanes + gid) * 16 + (i & 15u)] = (gid << 20) ^ i;
  }
}

int main() {
  const uint32_t blocks = 256 * 8, threads = 256;
  const uint64_t nthreads = (uint64_t)blocks * threads;
  const uint32_t per_thread = 512;  // 2^28 records, 2 GiB stored per kernel
  const uint64_t records = nthreads * per_thread;
  unsigned long long* out;
  CHECK(hipMalloc(&out, records * 8));
  hipEvent_t a, b;
  CHECK(hipEventCreate(&a)); CHECK(hipEventCreate(&b));
  auto timed = [&](const char* name, auto launch) -> int {
    CHECK(hipDeviceSynchronize());
    CHECK(hipEventRecord(a));
    launch();
    CHECK(hipEventRecord(b));
    CHECK(hipEventSynchronize(b));
    float ms = 0;
    CHECK(hipEventElapsedTime(&ms, a, b));
    printf("%-8s %8.3f ms  %llu records, %.3f GB stored, %.1f GB/s\n", name, ms, (unsigned long long)records,
           records * 8e-9, records * 8e-6 / ms);
    return 0;
  };
  if (timed("contig", [&] { hipLaunchKernelGGL(contig, dim3(blocks), dim3(threads), 0, 0, out, (uint64_t)per_thread); }))
    return 1;
  if (timed("own0", [&] { hipLaunchKernelGGL(own_lines<0>, dim3(blocks), dim3(threads), 0, 0, out, per_thread); }))
    return 1;
  if (timed("own24", [&] { hipLaunchKernelGGL(own_lines<24>, dim3(blocks), dim3(threads), 0, 0, out, per_thread); }))
    return 1;
  if (timed("own96", [&] { hipLaunchKernelGGL(own_lines<96>, dim3(blocks), dim3(threads), 0, 0, out, per_thread); }))
    return 1;
  return 0;
}
