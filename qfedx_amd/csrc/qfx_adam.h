// Client-batched Adam, one parameter of one client row: the element update shared by qfx_adam_kernel
// (csrc/train_kernels.hip) and the Adam epilogue of hea_grad_reduce_kernel (csrc/hea_mfma.hip), so the fused and
// the separate launch produce bitwise the same parameters.
#pragma once
#include <hip/hip_runtime.h>
#include <math.h>

#include "hea_args.h"   // QfxAdamArgs


// p[i] (row k, element i of P) with gradient gi; the row's first element also writes the step counter
// t_out[k] = t_in[k] + active[k].  Rows with active[k] == 0 are left untouched.
__device__ __forceinline__ void qfx_adam_elem(float* __restrict__ p, float gi, float* __restrict__ m,
                                              float* __restrict__ v, const float* __restrict__ t_in,
                                              float* __restrict__ t_out, const float* __restrict__ active, int k,
                                              long i, bool first, float lr, float b1, float b2, float eps) {
  const float act = active[k];
  const float tk = t_in[k] + act;
  if (first) t_out[k] = tk;
  if (act == 0.f) return;
  const float mi = __fmaf_rn(b1, m[i], (1.f - b1) * gi);
  const float vi = __fmaf_rn(b2, v[i], (1.f - b2) * gi * gi);
  m[i] = mi;
  v[i] = vi;
  const float mh = mi / (1.f - powf(b1, tk));
  const float vh = vi / (1.f - powf(b2, tk));
  p[i] = __fmaf_rn(-lr, mh / (sqrtf(vh) + eps), p[i]);
}
