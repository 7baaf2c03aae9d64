// Gradient sink of the CFed step kernels (csrc/cnn_kernels.hip), shared with the host bindings.
#pragma once

// Where a CNN step kernel's parameter-gradient entries go.  pout == nullptr: the gradient rows grad [K][P].
// Otherwise the client's local SGD-momentum step is applied right there instead of storing the gradient
// (torch.optim.SGD semantics, bitwise those of qfx_sgdm_kernel): b = g on the client's first step (t_in[k] == 0),
// else mu * buf + g; buf = b when keep; pout[k][e] = pin[k * pstride + e] - lr * b; rows with act[k] == 0 copy pin.
// pin may be the global parameters with pstride 0: the first local step of a round reads theta directly (no
// per-client row initialisation) and writes the stepped rows.  The gradient is never materialised or re-read.
struct CnnSgd {
  float* grad;
  const float* pin;
  long pstride;
  float* pout;
  float* buf;
  const float* t_in;
  float* t_out;          // written by the head kernel: t_out[k] = t_in[k] + act[k]
  const float* act;
  float lr, mu;
  int keep;
};
