// Issue cost of the fp64/int ops the transport kernel leans on (one wave-instruction's
// SIMD cycles): 8 independent chains per lane, 3 waves per SIMD, whole chip.
// build: hipcc -O3 --offload-arch=gfx950 valu_rates.hip -o valu_rates
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

constexpr int ITERS = 4096;

#define KERNEL(NAME, T, INIT, OP)                                             \
  __global__ void NAME(T* out, T seed) {                                      \
    T a0 = seed + (T)threadIdx.x, a1 = a0 + (T)1, a2 = a0 + (T)2, a3 = a0 + (T)3; \
    T a4 = a0 + (T)4, a5 = a0 + (T)5, a6 = a0 + (T)6, a7 = a0 + (T)7;         \
    INIT;                                                                     \
    for (int i = 0; i < ITERS; ++i) {                                         \
      OP(a0); OP(a1); OP(a2); OP(a3); OP(a4); OP(a5); OP(a6); OP(a7);         \
    }                                                                         \
    out[blockIdx.x * blockDim.x + threadIdx.x] = a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7; \
  }

#define OP_MUL(a) a = a * k
#define OP_ADD(a) a = a + k
#define OP_FMA(a) a = __builtin_fma(a, k, k2)
#define OP_RCP(a) a = __builtin_amdgcn_rcp(a)
#define OP_DIV(a) a = k / a
#define OP_SQRT(a) a = __builtin_sqrt(a)
#define OP_MAD64(a) a = (uint64_t)(uint32_t)a * 0xD2511F53u + (a >> 32)
#define OP_CVT(a) a = (double)(float)a * k

KERNEL(k_mul, double, const double k = 1.0000001, OP_MUL)
KERNEL(k_add, double, const double k = 1e-9, OP_ADD)
KERNEL(k_fma, double, const double k = 0.9999999; const double k2 = 1e-9, OP_FMA)
KERNEL(k_rcp, double, , OP_RCP)
KERNEL(k_div, double, const double k = 1.0000001, OP_DIV)
KERNEL(k_sqrt, double, , OP_SQRT)
KERNEL(k_mad64, uint64_t, , OP_MAD64)
KERNEL(k_cvt, double, const double k = 1.0000001, OP_CVT)

int main() {
  int cus = 0;
  hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
  int clk = 0;
  hipDeviceGetAttribute(&clk, hipDeviceAttributeClockRate, 0);
  const int threads = 256, blocks = cus * 3;  // 3 waves per SIMD
  double* out;
  hipMalloc(&out, sizeof(double) * blocks * threads);
  hipEvent_t e0, e1;
  hipEventCreate(&e0); hipEventCreate(&e1);
  struct K { const char* n; void (*f)(double*, double); bool u64; };
  auto run = [&](const char* name, auto kern, auto seed) {
    using S = decltype(seed);
    hipLaunchKernelGGL(kern, dim3(blocks), dim3(threads), 0, 0, (S*)out, seed);
    hipDeviceSynchronize();
    hipEventRecord(e0);
    for (int r = 0; r < 5; ++r) hipLaunchKernelGGL(kern, dim3(blocks), dim3(threads), 0, 0, (S*)out, seed);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms = 0; hipEventElapsedTime(&ms, e0, e1);
    const double waves_per_simd = 3.0;
    const double instr = 5.0 * ITERS * 8 * waves_per_simd;  // per SIMD
    const double cyc = ms * 1e-3 * clk * 1e3;               // SIMD clock cycles
    printf("%-8s %8.3f ms  %6.2f cycles per wave-op (clock %d MHz)\n", name, ms, cyc / instr, clk / 1000);
  };
  run("mul_f64", k_mul, 1.0);
  run("add_f64", k_add, 1.0);
  run("fma_f64", k_fma, 1.0);
  run("rcp_f64", k_rcp, 1.0);
  run("div_f64", k_div, 1.0);
  run("sqrt_f64", k_sqrt, 2.0);
  run("mad_u64", k_mad64, (uint64_t)12345);
  run("cvt+mul", k_cvt, 1.0);
  return 0;
}
