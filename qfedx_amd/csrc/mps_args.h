// Launch arguments of the CNOT-chain MPS kernel (csrc/mps_chain.hip), shared with its bindings (mps_bindings.cpp).
#pragma once
#include <cstdint>

constexpr int QFX_MPS_RMAX = 8;

struct QfxMpsArgs {
  const float* x;              // [S][x_stride] feature angles
  const float* theta;          // [K][t_stride] (RX of (layer l, qubit q) at 2 (l n + q), RZ at + 1)
  const float* w;              // [S][C] dL/d<Z_c> (gradient mode) or nullptr (<Z> only)
  float* z;                    // [S][C]
  float* grad;                 // [S][2 n L] per-sample angle gradients (gradient mode)
  float* rp;                   // scratch, complex [S][n][64]: right environments Rp_{q+1}
  float* ro;                   // scratch, complex [S][qmax + 1][64]: RO_{q+1} (gradient mode)
  int x_stride, t_stride, spc, S, n, L, feature, C, qmax;
  int readout[QFX_MPS_RMAX];
};
