// Philox4x32-10 core (Salmon et al. 2011), shared by device kernels (via philox.h) and the native host
// runtime (runtime.cpp, plain C++).  Bit-identical to qfedx_amd/utils/seeding.py::philox4x32.
#pragma once
#include <stdint.h>

#if defined(__HIPCC__)
#define QFX_HD __host__ __device__
#else
#define QFX_HD
#endif

namespace qfx {

struct u32x4 { uint32_t x, y, z, w; };

QFX_HD inline void mulhilo32(uint32_t a, uint32_t b, uint32_t& hi, uint32_t& lo) {
  const uint64_t p = (uint64_t)a * (uint64_t)b;
  hi = (uint32_t)(p >> 32);
  lo = (uint32_t)p;
}

QFX_HD inline u32x4 philox4x32_10(u32x4 c, uint32_t k0, uint32_t k1) {
#if defined(__HIPCC__) || defined(__clang__)
#pragma unroll
#else
#pragma GCC unroll 10
#endif
  for (int i = 0; i < 10; ++i) {
    uint32_t hi0, lo0, hi1, lo1;
    mulhilo32(0xD2511F53u, c.x, hi0, lo0);
    mulhilo32(0xCD9E8D57u, c.z, hi1, lo1);
    c = {hi1 ^ c.y ^ k0, lo1, hi0 ^ c.w ^ k1, lo0};
    k0 += 0x9E3779B9u;
    k1 += 0xBB67AE85u;
  }
  return c;
}

// uniform in (0, 1] for element e of a stream: counter (e/4, stream, 0, 0), word e%4, (w + 1) 2^-32
// computed in double and rounded to float (seeding.philox_uniform / philox_uniform_rows)
QFX_HD inline float philox_uniform_host(uint64_t e, uint32_t k0, uint32_t k1, uint32_t stream) {
  const uint64_t blk = e >> 2;
  const u32x4 o = philox4x32_10({(uint32_t)blk, (uint32_t)(blk >> 32), stream, 0u}, k0, k1);
  const uint32_t w = (e & 3) == 0 ? o.x : (e & 3) == 1 ? o.y : (e & 3) == 2 ? o.z : o.w;
  return (float)(((double)w + 1.0) * (1.0 / 4294967296.0));
}

}  // namespace qfx
