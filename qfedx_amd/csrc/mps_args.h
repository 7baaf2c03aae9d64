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
  // fused readout (gradient mode, w == nullptr): logits a <Z> + b from theta[ro_off ..] (a) and [ro_off + C ..] (b),
  // softmax cross entropy of label y with loss weight wts, dL/d<Z> = a dl formed in the kernel; per sample out:
  // dl [S][C] (dL/dlogit), lossv / hitv [S] (y == nullptr: no fused readout)
  const long long* y;
  const float* wts;
  int ro_off;
  float* dl;
  float* lossv;
  float* hitv;
};

// Launch arguments of the generic MPO-product MPS kernel (csrc/mps_mpo.hip; tables: quantum/mps_mpo.py).
constexpr int QFX_MPO_DMAX = 16;       // max bond (4 two-qubit gates across any cut)
constexpr int QFX_MPO_MAXPG = 64;      // max parametric rotations on one qubit

struct QfxMpoArgs {
  const float* ang;            // [S][G] gate angles (gate_angles of the lowered program)
  const int* gkind;            // [G] gate kinds (quantum/circuit.py KIND)
  const int* events;           // per-qubit event lists (mps_mpo.compile_mpo)
  const int* sinfo;            // [n][8] (event offset, count, pass-through pairs, their count, rotations, 0, 0, 0)
  const int* nbits;            // [n - 1] bond bits of every cut
  const float* w;              // [S][C] dL/d<Z_c> (gradient mode) or nullptr
  float* z;                    // [S][C]
  float* dang;                 // [S][G] dL/d(angle) of RX / RY / RZ / P gates (gradient mode; others untouched)
  float* rp;                   // scratch, complex [S][n][256]: right environments R_{q+1}
  float* ro;                   // scratch, complex [S][qmax + 1][256]: RO_{q+1} (gradient mode)
  int S, G, n, C, qmax;
  int readout[QFX_MPS_RMAX];
};
