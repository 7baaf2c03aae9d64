// Philox4x32-10 counter-based RNG (Salmon et al. 2011), device + host.
// Bit-identical to qfedx_amd/utils/seeding.py::philox4x32 (the CPU oracle); keyed by
// (seed, purpose, round, client) so every random stream is independent of the rank layout.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "philox_core.h"

namespace qfx {

// standard normal for element e of a stream: pairs (2i, 2i+1) come from counter e/4, Box-Muller in
// double on the (0,1] float uniforms - matches seeding.philox_normal element-for-element
__device__ inline float philox_normal_at(uint64_t e, uint32_t k0, uint32_t k1, uint32_t stream) {
  const uint64_t blk = e >> 2;
  const u32x4 o = philox4x32_10({(uint32_t)blk, (uint32_t)(blk >> 32), stream, 0u}, k0, k1);
  const bool second_pair = (e >> 1) & 1;
  const uint32_t w1 = second_pair ? o.z : o.x;
  const uint32_t w2 = second_pair ? o.w : o.y;
  const float u1f = (float)(((double)w1 + 1.0) * (1.0 / 4294967296.0));
  const float u2f = (float)(((double)w2 + 1.0) * (1.0 / 4294967296.0));
  const double r = sqrt(-2.0 * log((double)u1f));
  const double th = 6.283185307179586 * (double)u2f;
  return (float)((e & 1) ? r * sin(th) : r * cos(th));
}

// uniform in (0, 1] for element e of a stream: counter (e/4, stream), word e%4 - matches
// seeding.philox_uniform / philox_uniform_rows element-for-element
__device__ inline float philox_uniform_at(uint64_t e, uint32_t k0, uint32_t k1, uint32_t stream) {
  const uint64_t blk = e >> 2;
  const u32x4 o = philox4x32_10({(uint32_t)blk, (uint32_t)(blk >> 32), stream, 0u}, k0, k1);
  const uint32_t w = (e & 3) == 0 ? o.x : (e & 3) == 1 ? o.y : (e & 3) == 2 ? o.z : o.w;
  return (float)(((double)w + 1.0) * (1.0 / 4294967296.0));
}

// readout noise on one <Z> marginal (K19): confusion z' = (1 - p01 - p10) z + p10 - p01, then with
// shots > 0 the shot estimate 1 - 2 k / shots, k ~ Binomial(shots, (1 - z') / 2) drawn exactly as
// the count of uniforms u_i <= p1 over elements [e0, e0 + shots) of the stream
__device__ inline float noisy_z(float z, float p01, float p10, int shots, uint32_t k0, uint32_t k1,
                                uint32_t stream, uint64_t e0) {
  z = fmaf(1.f - p01 - p10, z, p10 - p01);
  if (shots <= 0) return z;
  const float p1 = fminf(fmaxf(0.5f * (1.f - z), 0.f), 1.f);
  int cnt = 0;
  uint64_t e = e0;
  const uint64_t end = e0 + (uint64_t)shots;
  while (e < end) {   // one Philox block serves up to 4 consecutive shots
    const uint64_t blk = e >> 2;
    const u32x4 o = philox4x32_10({(uint32_t)blk, (uint32_t)(blk >> 32), stream, 0u}, k0, k1);
    const uint32_t w4[4] = {o.x, o.y, o.z, o.w};
    for (int j = (int)(e & 3); j < 4 && e < end; ++j, ++e)
      cnt += ((float)(((double)w4[j] + 1.0) * (1.0 / 4294967296.0)) <= p1) ? 1 : 0;
  }
  return 1.f - 2.f * (float)cnt / (float)shots;
}

}  // namespace qfx
