// Noiseless per-sample readout + cross entropy, shared by the readout/CE kernel (train_kernels.hip) and the MFMA
// engine's first adjoint pass, which computes its sample's dL/d<Z> itself (hea_mfma.hip, fused readout): both paths
// run the same operations in the same order, so they give the same values.
#pragma once
#include <hip/hip_runtime.h>

namespace qfx_ro {

constexpr int RO_CMAX = 8;

// zs[c] = sum_u part[s][u][c] in tile order.  Loads are issued in batches of 8 tiles (predicated) so their latencies
// overlap instead of serialising one dependent load per tile.
__device__ __forceinline__ void tile_sums(const float* __restrict__ part, long s, int tps, int C, float (&zs)[RO_CMAX]) {
#pragma unroll
  for (int c = 0; c < RO_CMAX; ++c) zs[c] = 0.f;
  const float* base = part + (size_t)s * tps * C;
  for (int u0 = 0; u0 < tps; u0 += 8) {
    float v[8][RO_CMAX];
#pragma unroll
    for (int du = 0; du < 8; ++du)
#pragma unroll
      for (int c = 0; c < RO_CMAX; ++c) v[du][c] = (u0 + du < tps && c < C) ? base[(size_t)(u0 + du) * C + c] : 0.f;
#pragma unroll
    for (int du = 0; du < 8; ++du)
#pragma unroll
      for (int c = 0; c < RO_CMAX; ++c) zs[c] += v[du][c];
  }
}

// Logits a z + b, softmax cross entropy of label yy with loss weight ws: dl[c] = (p_c - [c == yy]) ws (dL/dlogit),
// the weighted loss term ws (lse - logit_yy) and the hit (argmax == yy, ws > 0).
__device__ __forceinline__ void ce_sample(const float (&z)[RO_CMAX], const float* a, const float* b, int C, int yy, float ws,
                                          float (&dl)[RO_CMAX], float& loss, float& hit) {
  float lg[RO_CMAX];
  float m = -INFINITY;
#pragma unroll
  for (int c = 0; c < RO_CMAX; ++c) {
    if (c >= C) break;
    lg[c] = fmaf(a[c], z[c], b[c]);
    m = fmaxf(m, lg[c]);
  }
  float se = 0.f;
  int am = 0;
#pragma unroll
  for (int c = 0; c < RO_CMAX; ++c) {
    if (c >= C) break;
    se += expf(lg[c] - m);
    if (lg[c] > lg[am]) am = c;
  }
  const float lse = m + logf(se);
  float ly = 0.f;
#pragma unroll
  for (int c = 0; c < RO_CMAX; ++c) {
    dl[c] = 0.f;
    if (c >= C) break;
    if (c == yy) ly = lg[c];
    const float p = expf(lg[c] - lse);
    dl[c] = (p - (c == yy ? 1.f : 0.f)) * ws;
  }
  loss = ws * (lse - ly);
  hit = (am == yy && ws > 0.f) ? 1.f : 0.f;
}

}  // namespace qfx_ro
