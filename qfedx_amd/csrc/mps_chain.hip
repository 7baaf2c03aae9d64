// Exact matrix-product-state contraction of the CNOT-chain hardware-efficient VQC, one wave per sample (the MPS
// backend's fast path; math and float64 oracle: qfedx_amd/quantum/mps_chain.py).
//
// Qubit q's column maps its left / right bond words (a, b: one bit per layer, the CNOTs from q - 1 and to q + 1) to
//     A_q[a, :, b] = P_{b_L} X^{a_L} G_L ... P_{b_1} X^{a_1} G_1 F(x_q)|0>        (G_l = RZ(phi) RX(theta))
// an exact MPS of bond D = 2^L <= 8 built column by column - lane (a, b) of the wave computes A_q[a, :, b] - with no
// MPO application, QR or SVD.  Transfer environments are D x D matrices (lane (a, a') holds one entry):
//   right sweep   Rp_q = sum_s conj(A_q[s]) Rp_{q+1} A_q[s]^T                           (stored per cut, scratch)
//   <Z_c>         contraction of Lp_c, conj(A_c) Z A_c and Rp_{c+1}                      (mode expz)
//   gradients     RO (the observable O = sum_c w_c Z_c right of a cut) for the readout cuts, then a left sweep
//                 carrying Lp and LO: at column q, Ybar = d<O>/dA_q (a D x 2 x D tensor, lane (a', b') holds a
//                 2-vector) and reverse mode through the lane's own 2 x 2 gate chain gives all 2L angle
//                 derivatives of the column at once (2 Re, summed over the wave).
// Cost O(n D^3) per sample: a 48-qubit 3-layer sample is ~50K complex multiply-adds - the torch einsum network of
// the generic MPS backend spent ~100 ms per 2048-sample step in launches and small batched GEMMs.
#include <hip/hip_runtime.h>

#include <cstdint>

#include "mps_args.h"
#include "qfx_readout.h"

namespace qfx_mps {

constexpr int DM = 8;          // max bond (L <= 3)
constexpr int WPB = 4;         // waves (samples) per block
constexpr int RMAX = QFX_MPS_RMAX;   // readout qubits

using MpsArgs = QfxMpsArgs;

__device__ __forceinline__ float2 cmul(float2 a, float2 b) { return make_float2(a.x * b.x - a.y * b.y, a.x * b.y + a.y * b.x); }
// conj(a) * b
__device__ __forceinline__ float2 cjmul(float2 a, float2 b) { return make_float2(a.x * b.x + a.y * b.y, a.x * b.y - a.y * b.x); }
__device__ __forceinline__ float2 cadd(float2 a, float2 b) { return make_float2(a.x + b.x, a.y + b.y); }
__device__ __forceinline__ float2 csc(float2 a, float s) { return make_float2(a.x * s, a.y * s); }
__device__ __forceinline__ void wave_lds() { __asm__ volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); }
__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// One column's gate chain for lane (a, b): the 2-vector A_q[a, :, b], and (for the reverse) the vectors entering each
// layer's RX (vp) and RZ (vm).
struct Col {
  float2 v0, v1;
  float2 vp[3][2], vm[3][2];
  float ct[3], st[3], cp[3], sp[3];
};

__device__ __forceinline__ void build_col(const MpsArgs& g, const float* th, float xq, int q, int a, int b, Col& c) {
  float s0, c0;
  sincosf(0.5f * xq, &s0, &c0);   // (precise: the __sincosf error drifted the norm by ~3e-5 over 48 x 3 gates)
  if (g.feature == 1) {                    // rx
    c.v0 = make_float2(c0, 0.f);
    c.v1 = make_float2(0.f, -s0);
  } else if (g.feature == 2) {             // rz
    c.v0 = make_float2(c0, -s0);
    c.v1 = make_float2(0.f, 0.f);
  } else {                                 // ry
    c.v0 = make_float2(c0, 0.f);
    c.v1 = make_float2(s0, 0.f);
  }
#pragma unroll
  for (int l = 0; l < 3; ++l) {
    if (l >= g.L) break;
    const int k = 2 * (l * g.n + q);
    sincosf(0.5f * th[k], &c.st[l], &c.ct[l]);
    sincosf(0.5f * th[k + 1], &c.sp[l], &c.cp[l]);
    c.vp[l][0] = c.v0;
    c.vp[l][1] = c.v1;
    // RX: [c, -i s; -i s, c]     (-i s z = (s z.y, -s z.x))
    const float2 r0 = make_float2(c.ct[l] * c.v0.x + c.st[l] * c.v1.y, c.ct[l] * c.v0.y - c.st[l] * c.v1.x);
    const float2 r1 = make_float2(c.ct[l] * c.v1.x + c.st[l] * c.v0.y, c.ct[l] * c.v1.y - c.st[l] * c.v0.x);
    c.vm[l][0] = r0;
    c.vm[l][1] = r1;
    // RZ: diag(e^{-i phi/2}, e^{i phi/2})
    c.v0 = cmul(r0, make_float2(c.cp[l], -c.sp[l]));
    c.v1 = cmul(r1, make_float2(c.cp[l], c.sp[l]));
    if (q > 0 && ((a >> l) & 1)) {         // X^{a_l}: target of CNOT(q - 1, q)
      const float2 t = c.v0;
      c.v0 = c.v1;
      c.v1 = t;
    }
    if (q < g.n - 1) {                     // P_{b_l}: control of CNOT(q, q + 1)
      if ((b >> l) & 1) c.v0 = make_float2(0.f, 0.f);
      else c.v1 = make_float2(0.f, 0.f);
    }
  }
}

// Reverse mode through lane (a, b)'s chain: u = dO/dA[a, :, b] (the coefficient of A, not of conj(A)); out[2 l] /
// out[2 l + 1] += 2 Re(d/d theta_l) / (d/d phi_l) of sum_s u_s A_s.
__device__ __forceinline__ void reverse_col(const MpsArgs& g, const Col& c, int q, int a, int b, float2 u0, float2 u1,
                                            float* out) {
#pragma unroll
  for (int l = 2; l >= 0; --l) {
    if (l >= g.L) continue;
    if (q < g.n - 1) {                     // P_b (symmetric)
      if ((b >> l) & 1) u0 = make_float2(0.f, 0.f);
      else u1 = make_float2(0.f, 0.f);
    }
    if (q > 0 && ((a >> l) & 1)) {
      const float2 t = u0;
      u0 = u1;
      u1 = t;
    }
    // RZ output components y0 = e- m0, y1 = e+ m1; dy/dphi = (-i/2) z_s y_s
    const float2 em = make_float2(c.cp[l], -c.sp[l]), ep = make_float2(c.cp[l], c.sp[l]);
    const float2 y0 = cmul(c.vm[l][0], em), y1 = cmul(c.vm[l][1], ep);
    // sum_s u_s dy_s = (-i/2)(u0 y0 - u1 y1): Re = 0.5 Im(u0 y0 - u1 y1)
    const float2 d = make_float2(cmul(u0, y0).x - cmul(u1, y1).x, cmul(u0, y0).y - cmul(u1, y1).y);
    out[2 * l + 1] += d.y;                  // 2 Re((-i/2) d) = Im d
    // back through RZ: u_s *= e-+ (transpose of a diagonal)
    u0 = cmul(u0, em);
    u1 = cmul(u1, ep);
    // RX output r = RX vp; dr/dtheta = (-i/2) X r: sum_s u_s dr_s = (-i/2)(u0 r1 + u1 r0)
    const float2 r0 = c.vm[l][0], r1 = c.vm[l][1];
    const float2 e = cadd(cmul(u0, r1), cmul(u1, r0));
    out[2 * l] += e.y;
    // back through RX (symmetric): u' = RX^T u = RX u
    const float2 n0 = make_float2(c.ct[l] * u0.x + c.st[l] * u1.y, c.ct[l] * u0.y - c.st[l] * u1.x);
    const float2 n1 = make_float2(c.ct[l] * u1.x + c.st[l] * u0.y, c.ct[l] * u1.y - c.st[l] * u0.x);
    u0 = n0;
    u1 = n1;
  }
}

__global__ void __launch_bounds__(64 * WPB) mps_chain_kernel(MpsArgs g) {
  __shared__ float2 As[WPB][2][DM * DM];   // A[s][a * 8 + b]
  __shared__ float2 U1[WPB][2][DM * DM];   // U[s][a' * 8 + b]
  __shared__ float2 U2[WPB][2][DM * DM];
  __shared__ float2 E1[WPB][DM * DM];      // Lp (left sweep) / R (right sweep)
  __shared__ float2 E2[WPB][DM * DM];      // LO / RO
  __shared__ float2 E3[WPB][DM * DM];      // Rp_{q+1} / RO_{q+1} staging
  __shared__ float2 E4[WPB][DM * DM];
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int s = blockIdx.x * WPB + wave;
  if (s >= g.S) return;                    // whole waves only: no block barrier below
  const int x_ = lane >> 3, y_ = lane & 7;
  const int D = 1 << g.L, n = g.n;
  const float* th = g.theta + (size_t)(s / g.spc) * g.t_stride;
  const float* xs = g.x + (size_t)s * g.x_stride;
  float2* A0 = As[wave][0];
  float2* A1 = As[wave][1];
  float2* R = E1[wave];
  float2* rp = reinterpret_cast<float2*>(g.rp) + (size_t)s * n * 64;
  const bool fused = g.y != nullptr;                 // gradient mode, dL/d<Z> formed from the kernel's own <Z>
  const bool grad = g.w != nullptr || fused;
  float wq[RMAX];
  int rq[RMAX];
#pragma unroll
  for (int i = 0; i < RMAX; ++i) {
    rq[i] = i < g.C ? g.readout[i] : -1;
    wq[i] = (grad && !fused && i < g.C) ? g.w[(size_t)s * g.C + i] : 0.f;
  }
  auto wof = [&](int q) {                  // weight of Z_q in O (0 off the readout)
    float v = 0.f;
#pragma unroll
    for (int i = 0; i < RMAX; ++i) v += rq[i] == q ? wq[i] : 0.f;
    return v;
  };
  auto put_col = [&](const Col& c, int Dl, int Dr) {
    if (x_ < Dl && y_ < Dr) {
      A0[x_ * 8 + y_] = c.v0;
      A1[x_ * 8 + y_] = c.v1;
    }
    wave_lds();
  };
  // env_right: out[a][a'] = sum_{s, b, b'} conj(A[a,s,b]) (zs) A[a',s,b'] Rin[b][b']  (lane (a, a'))
  // via Y[a'][s][b] = sum_b' A[a',s,b'] Rin[b][b'] (lane (a', b), into U1)
  auto env_right = [&](const float2* Rin, int Dl, int Dr, float2* Y) {
    if (x_ < Dl && y_ < Dr) {
      float2 y0 = make_float2(0.f, 0.f), y1 = y0;
      for (int bp = 0; bp < Dr; ++bp) {
        const float2 r = Rin[y_ * 8 + bp];
        y0 = cadd(y0, cmul(A0[x_ * 8 + bp], r));
        y1 = cadd(y1, cmul(A1[x_ * 8 + bp], r));
      }
      Y[x_ * 8 + y_] = y0;
      Y[64 + x_ * 8 + y_] = y1;
    }
    wave_lds();
  };
  auto env_right_fin = [&](const float2* Y, int Dl, int Dr, float zsign1, float2& out) {
    out = make_float2(0.f, 0.f);
    if (x_ < Dl && y_ < Dl) {
      for (int b = 0; b < Dr; ++b) {
        out = cadd(out, cjmul(A0[x_ * 8 + b], Y[y_ * 8 + b]));
        out = cadd(out, csc(cjmul(A1[x_ * 8 + b], Y[64 + y_ * 8 + b]), zsign1));
      }
    }
  };

  // ---------------- right sweep: Rp_{q+1} for every column (stored), and RO_{q+1} for the readout cuts
  if (lane == 0) R[0] = make_float2(1.f, 0.f);
  wave_lds();
  for (int q = n - 1; q >= 0; --q) {
    const int Dl = q == 0 ? 1 : D, Dr = q == n - 1 ? 1 : D;
    rp[(size_t)q * 64 + lane] = R[lane];   // Rp_{q+1} (entries past Dr x Dr unused)
    Col c;
    build_col(g, th, xs[q], q, x_, y_, c);
    put_col(c, Dl, Dr);
    env_right(R, Dl, Dr, U1[wave][0]);
    float2 o;
    env_right_fin(U1[wave][0], Dl, Dr, 1.f, o);
    wave_lds();
    R[lane] = o;
    wave_lds();
  }
  // <psi|psi> = Rp_0 (1 x 1): the readout is divided by it (exactly 1 up to fp32 rounding, as the torch MPS backend
  // normalises), the gradients too (first order)
  const float inv_norm = 1.f / R[0].x;
  // ---------------- readout <Z_c>: left sweep up to the last readout qubit
  float2* Lp = E1[wave];
  float2* LO = E2[wave];
  float2* Rq = E3[wave];
  float2* ROq = E4[wave];
  // RO_{q+1} of the readout cuts (gradient mode), written by the RO sweep below
  float2* ros = reinterpret_cast<float2*>(g.ro) + (size_t)s * (g.qmax + 1) * 64;
  float zc[RMAX];
  // left sweep over columns [0, qend): <Z> of the readout qubits into zc, and with gm the gradient terms
  auto left = [&](int qend, bool gm) {
#pragma unroll
  for (int i = 0; i < RMAX; ++i) zc[i] = 0.f;
  if (lane == 0) {
      Lp[0] = make_float2(1.f, 0.f);
      LO[0] = make_float2(0.f, 0.f);
    }
    wave_lds();
    float* gout = grad ? g.grad + (size_t)s * 2 * n * g.L : nullptr;
    for (int q = 0; q < qend; ++q) {
      const int Dl = q == 0 ? 1 : D, Dr = q == n - 1 ? 1 : D;
      Col c;
      build_col(g, th, xs[q], q, x_, y_, c);
      put_col(c, Dl, Dr);
      Rq[lane] = rp[(size_t)q * 64 + lane];
      ROq[lane] = (gm && q <= g.qmax) ? ros[(size_t)q * 64 + lane] : make_float2(0.f, 0.f);
      // U1[a'][s][b] = sum_a conj(A[a,s,b]) Lp[a][a'],  U2 the same with LO   (lane (a', b))
      float2* u1 = U1[wave][0];
      float2* u2 = U2[wave][0];
      if (x_ < Dl && y_ < Dr) {
        float2 p0 = make_float2(0.f, 0.f), p1 = p0, o0 = p0, o1 = p0;
        for (int a = 0; a < Dl; ++a) {
          const float2 l = Lp[a * 8 + x_], lo = LO[a * 8 + x_];
          const float2 a0 = A0[a * 8 + y_], a1 = A1[a * 8 + y_];
          p0 = cadd(p0, cjmul(a0, l));
          p1 = cadd(p1, cjmul(a1, l));
          o0 = cadd(o0, cjmul(a0, lo));
          o1 = cadd(o1, cjmul(a1, lo));
        }
        u1[x_ * 8 + y_] = p0;
        u1[64 + x_ * 8 + y_] = p1;
        u2[x_ * 8 + y_] = o0;
        u2[64 + x_ * 8 + y_] = o1;
      }
      wave_lds();
      const float wz = wof(q);
      // readout: <Z_q> = sum_{a',s,b,b'} z_s U1[a',s,b] A[a',s,b'] Rp[b][b']
      bool isro = false;
  #pragma unroll
      for (int i = 0; i < RMAX; ++i) isro |= rq[i] == q;
      if (isro) {
        float t = 0.f;
        if (x_ < Dl && y_ < Dr) {
          float2 y0 = make_float2(0.f, 0.f), y1 = y0;
          for (int bp = 0; bp < Dr; ++bp) {
            const float2 r = Rq[y_ * 8 + bp];
            y0 = cadd(y0, cmul(A0[x_ * 8 + bp], r));
            y1 = cadd(y1, cmul(A1[x_ * 8 + bp], r));
          }
          t = cmul(u1[x_ * 8 + y_], y0).x - cmul(u1[64 + x_ * 8 + y_], y1).x;
        }
        t = wave_sum(t);
  #pragma unroll
        for (int i = 0; i < RMAX; ++i)
          if (rq[i] == q) zc[i] = t;
      }
      if (gm) {
        // Ybar[a'][s][b'] = sum_b U1[a',s,b] (RO[b][b'] + wz z_s Rp[b][b']) + U2[a',s,b] Rp[b][b']   (lane (a', b'))
        float2 g0 = make_float2(0.f, 0.f), g1 = g0;
        if (x_ < Dl && y_ < Dr) {
          for (int b = 0; b < Dr; ++b) {
            const float2 r = Rq[b * 8 + y_], ro = ROq[b * 8 + y_];
            const float2 k0 = cadd(ro, csc(r, wz)), k1 = cadd(ro, csc(r, -wz));
            g0 = cadd(g0, cadd(cmul(u1[x_ * 8 + b], k0), cmul(u2[x_ * 8 + b], r)));
            g1 = cadd(g1, cadd(cmul(u1[64 + x_ * 8 + b], k1), cmul(u2[64 + x_ * 8 + b], r)));
          }
        }
        float part[6] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
        if (x_ < Dl && y_ < Dr) reverse_col(g, c, q, x_, y_, g0, g1, part);
  #pragma unroll
        for (int l = 0; l < 3; ++l) {
          if (l >= g.L) break;
          const float dt = wave_sum(part[2 * l]), dp = wave_sum(part[2 * l + 1]);
          if (lane == 0) {
            gout[2 * (l * n + q)] = dt * inv_norm;      // (reverse_col already returns 2 Re)
            gout[2 * (l * n + q) + 1] = dp * inv_norm;
          }
        }
      }
      // Lp_{q+1}[b][b'] = sum_{a',s} U1[a',s,b] A[a',s,b'];  LO_{q+1} = sum (U2 + wz z_s U1) A   (lane (b, b'))
      float2 nl = make_float2(0.f, 0.f), no = nl;
      if (x_ < Dr && y_ < Dr) {
        for (int ap = 0; ap < Dl; ++ap) {
          const float2 a0 = A0[ap * 8 + y_], a1 = A1[ap * 8 + y_];
          const float2 p0 = u1[ap * 8 + x_], p1 = u1[64 + ap * 8 + x_];
          nl = cadd(nl, cadd(cmul(p0, a0), cmul(p1, a1)));
          if (gm) {
            const float2 o0 = cadd(u2[ap * 8 + x_], csc(p0, wz)), o1 = cadd(u2[64 + ap * 8 + x_], csc(p1, -wz));
            no = cadd(no, cadd(cmul(o0, a0), cmul(o1, a1)));
          }
        }
      }
      wave_lds();
      Lp[lane] = nl;
      LO[lane] = no;
      wave_lds();
    }
  };
  if (fused) {
    // <Z> first (left sweep up to the last readout qubit), then the sample's logits a <Z> + b, softmax cross
    // entropy (qfx_readout.h, the HEA engine's fused readout) and dL/d<Z>_c = a_c dl_c for the gradient sweeps
    left(g.qmax + 1, false);
    float* wsh = reinterpret_cast<float*>(E3[wave]);
    if (lane == 0) {
      const float* prm = g.theta + (size_t)(s / g.spc) * g.t_stride + g.ro_off;
      float zz[qfx_ro::RO_CMAX], dl[qfx_ro::RO_CMAX], loss, hit;
#pragma unroll
      for (int i = 0; i < qfx_ro::RO_CMAX; ++i) zz[i] = i < g.C ? zc[i] * inv_norm : 0.f;
      qfx_ro::ce_sample(zz, prm, prm + g.C, g.C, (int)g.y[s], g.wts[s], dl, loss, hit);
      for (int i = 0; i < g.C; ++i) {
        g.z[(size_t)s * g.C + i] = zz[i];
        g.dl[(size_t)s * g.C + i] = dl[i];
        wsh[i] = prm[i] * dl[i];
      }
      g.lossv[s] = loss;
      g.hitv[s] = hit;
    }
    wave_lds();
#pragma unroll
    for (int i = 0; i < RMAX; ++i) wq[i] = i < g.C ? wsh[i] : 0.f;
    wave_lds();
  }
  if (grad) {
    ROq[lane] = make_float2(0.f, 0.f);
    wave_lds();
    for (int q = g.qmax; q >= 0; --q) {
      const int Dl = q == 0 ? 1 : D, Dr = q == n - 1 ? 1 : D;
      ros[(size_t)q * 64 + lane] = ROq[lane];
      Rq[lane] = rp[(size_t)q * 64 + lane];
      Col c;
      build_col(g, th, xs[q], q, x_, y_, c);
      put_col(c, Dl, Dr);
      const float wz = wof(q);
      env_right(ROq, Dl, Dr, U1[wave][0]);
      env_right(Rq, Dl, Dr, U2[wave][0]);
      float2 o1, o2;
      env_right_fin(U1[wave][0], Dl, Dr, 1.f, o1);
      env_right_fin(U2[wave][0], Dl, Dr, -1.f, o2);
      wave_lds();
      ROq[lane] = cadd(o1, csc(o2, wz));
      wave_lds();
    }
  }
  left(grad ? n : g.qmax + 1, grad);
  if (lane == 0 && !fused) {
#pragma unroll
    for (int i = 0; i < RMAX; ++i)
      if (i < g.C) g.z[(size_t)s * g.C + i] = zc[i] * inv_norm;
  }
}

}  // namespace qfx_mps

extern "C" int qfx_mps_chain(const qfx_mps::MpsArgs* args, hipStream_t st) {
  const qfx_mps::MpsArgs& g = *args;
  if (g.L < 1 || g.L > 3 || g.n < 2 || g.C < 1 || g.C > qfx_mps::RMAX || g.qmax >= g.n) return -2;
  if (g.S == 0) return 0;
  const unsigned grid = (unsigned)((g.S + qfx_mps::WPB - 1) / qfx_mps::WPB);
  hipLaunchKernelGGL(qfx_mps::mps_chain_kernel, dim3(grid), dim3(64 * qfx_mps::WPB), 0, st, g);
  return (int)hipGetLastError();
}

extern "C" int qfx_mps_args_size() { return (int)sizeof(qfx_mps::MpsArgs); }
