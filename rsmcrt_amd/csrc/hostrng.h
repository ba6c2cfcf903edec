// hostrng.h — host-side Philox4x32-10 streams of libsmcrt.so (the generator of the transport
// kernel, detmath.h, on the host). Each host driver draws from its own counter family, which
// no photon stream uses (photon counters have word 1 = 0):
//   word 1 = 1: inverse-MCRT guesses (inverse.cpp)
//   word 1 = 2: spectral optical properties (spectral.cpp)
// Draw d of a stream is the (d & 1) half of block (d >> 1, word1, 0, 0xFFFFFFFF) under the
// key (seed_lo, seed_hi), mapped to a 53-bit double in [0, 1) like ran2 (random_mod.f90:83-90).
#pragma once
#include <stdint.h>

namespace smcrt {

inline void host_philox(uint32_t c[4], uint32_t k0, uint32_t k1) {  // Salmon et al. 2011
  for (int r = 0; r < 10; ++r) {
    if (r > 0) { k0 += 0x9E3779B9u; k1 += 0xBB67AE85u; }
    const uint64_t p0 = (uint64_t)0xD2511F53u * c[0], p1 = (uint64_t)0xCD9E8D57u * c[2];
    const uint32_t n0 = (uint32_t)(p1 >> 32) ^ c[1] ^ k0, n2 = (uint32_t)(p0 >> 32) ^ c[3] ^ k1;
    c[1] = (uint32_t)p1; c[3] = (uint32_t)p0; c[0] = n0; c[2] = n2;
  }
}

struct HostStream {
  uint32_t k0, k1, word1;
  uint64_t d = 0;
  double next() {
    uint32_t c[4] = {(uint32_t)(d >> 1), word1, 0u, 0xFFFFFFFFu};
    host_philox(c, k0, k1);
    const uint64_t u = (d & 1) ? (((uint64_t)c[3] << 32) | c[2]) : (((uint64_t)c[1] << 32) | c[0]);
    ++d;
    return (double)(u >> 11) * 0x1.0p-53;
  }
};

constexpr uint32_t STREAM_INVERSE = 1, STREAM_SPECTRAL = 2;

}  // namespace smcrt
