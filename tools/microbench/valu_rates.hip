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

// 32-bit ops through inline asm (plain C chains of integer adds are folded by the compiler)
#define OP_ADD32(a) asm volatile("v_add_u32 %0, %0, %1" : "+v"(a) : "v"(k))
#define OP_XOR32(a) asm volatile("v_xor_b32 %0, %0, %1" : "+v"(a) : "v"(k))
#define OP_MULF32(a) asm volatile("v_mul_f32 %0, %0, %1" : "+v"(a) : "v"(k))
#define OP_ADDF64A(a) asm volatile("v_add_f64 %0, %0, %1" : "+v"(a) : "v"(k))
KERNEL(k_add32, uint32_t, const uint32_t k = 0x9E3779B9u, OP_ADD32)
KERNEL(k_xor32, uint32_t, const uint32_t k = 0x9E3779B9u, OP_XOR32)
KERNEL(k_mulf32, float, const float k = 1.0000001f, OP_MULF32)
KERNEL(k_addf64a, double, const double k = 1e-9, OP_ADDF64A)
// fp64 adds in chains 0-3 and 32-bit adds in chains 4-7 of the same wave: do the two overlap?
__global__ void k_mix(double* out, double seed) {
  double a0 = seed + threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3;
  uint32_t b0 = threadIdx.x, b1 = b0 + 1, b2 = b0 + 2, b3 = b0 + 3;
  const double k = 1e-9;
  const uint32_t kk = 0x9E3779B9u;
  for (int i = 0; i < ITERS; ++i) {
#define A64(a) asm volatile("v_add_f64 %0, %0, %1" : "+v"(a) : "v"(k))
#define A32(b) asm volatile("v_add_u32 %0, %0, %1" : "+v"(b) : "v"(kk))
    A64(a0); A32(b0); A64(a1); A32(b1); A64(a2); A32(b2); A64(a3); A32(b3);
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = a0 + a1 + a2 + a3 + (double)(b0 ^ b1 ^ b2 ^ b3);
}
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
    fflush(stdout);
  };
  run("add_u32", k_add32, (uint32_t)7);
  run("mul_f32", k_mulf32, 1.0f);
  run("xor_u32", k_xor32, (uint32_t)7);
  run("add_f64a", k_addf64a, 1.0);
  run("mix64+32", k_mix, 1.0);
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
