// Device-side building blocks of the statevector pass kernels, shared by the ahead-of-time
// interpreter kernel (statevec.hip) and the circuit-specialised kernels that jit.cpp generates and
// compiles with hiprtc at plan time.  Header-only, no <stdint.h> (hiprtc has no libc headers).
#pragma once
#include <hip/hip_runtime.h>

#include "qfx_plan.h"

typedef unsigned int uint32_t;

namespace qfx {

// the plan blob is read-only for the whole launch: reading it through the constant address space
// lets hipcc use scalar (SMEM) loads even though the adjoint kernel stores gradient partials to
// global memory inside the op loop (a generic pointer could alias those stores)
typedef const __attribute__((address_space(4))) int* cint_p;

struct M2 { float2 a, b, c, d; };   // [[a, b], [c, d]]

__device__ __forceinline__ float2 mk(float x, float y) { return make_float2(x, y); }
__device__ __forceinline__ float2 cmul(float2 a, float2 b) {
  return make_float2(fmaf(a.x, b.x, -a.y * b.y), fmaf(a.x, b.y, a.y * b.x));
}
__device__ __forceinline__ float2 cfma(float2 a, float2 b, float2 c) {  // a*b + c
  return make_float2(fmaf(a.x, b.x, fmaf(-a.y, b.y, c.x)), fmaf(a.x, b.y, fmaf(a.y, b.x, c.y)));
}
__device__ __forceinline__ float2 conjf2(float2 a) { return make_float2(a.x, -a.y); }
__device__ __forceinline__ float imcl(float2 l, float2 p) { return l.x * p.y - l.y * p.x; }  // Im(conj(l) p)
__device__ __forceinline__ float recl(float2 l, float2 p) { return l.x * p.x + l.y * p.y; }  // Re(conj(l) p)

__device__ __forceinline__ bool kind_is_diag(int k) {
  return k == K_RZ || k == K_P || k == K_Z || k == K_S || k == K_SDG || k == K_T || k == K_TDG;
}

__device__ __forceinline__ float gate_angle(cint_p gt, int gi, const float* prow,
                                            const float* xrow, int n_theta) {
  cint_p e = gt + gi * GATE_WORDS;
  const int slot = e[3];
  float v = 0.f;
  if (slot >= 0) v = slot < n_theta ? prow[slot] : xrow[slot - n_theta];
  return fmaf(__int_as_float(e[4]), v, __int_as_float(e[5]));
}

// (c, s) = (cos, sin) of the half angle for RX/RY/RZ, of the full angle for P
__device__ __forceinline__ float2 gate_cs(cint_p gt, int gi, const float* prow,
                                          const float* xrow, int n_theta) {
  const float ang = gate_angle(gt, gi, prow, xrow, n_theta);
  const float x = gt[gi * GATE_WORDS] == K_P ? ang : 0.5f * ang;
  float s, c;
  sincosf(x, &s, &c);
  return mk(c, s);
}

// full 2x2 (diagonal kinds too); inverse = conjugate transpose
__device__ __forceinline__ M2 gate_m2(int kind, float2 cs, bool inv) {
  const float r2 = 0.70710678118654752f, t = 0.70710678118654752f;
  const float c = cs.x, s = cs.y;
  M2 m;
  const float2 z = mk(0.f, 0.f), one = mk(1.f, 0.f);
  switch (kind) {
    case K_RX: m = {mk(c, 0.f), mk(0.f, -s), mk(0.f, -s), mk(c, 0.f)}; break;
    case K_RY: m = {mk(c, 0.f), mk(-s, 0.f), mk(s, 0.f), mk(c, 0.f)}; break;
    case K_RZ: m = {mk(c, -s), z, z, mk(c, s)}; break;
    case K_P: m = {one, z, z, cs}; break;
    case K_H: m = {mk(r2, 0.f), mk(r2, 0.f), mk(r2, 0.f), mk(-r2, 0.f)}; break;
    case K_X: m = {z, one, one, z}; break;
    case K_Y: m = {z, mk(0.f, -1.f), mk(0.f, 1.f), z}; break;
    case K_Z: m = {one, z, z, mk(-1.f, 0.f)}; break;
    case K_S: m = {one, z, z, mk(0.f, 1.f)}; break;
    case K_SDG: m = {one, z, z, mk(0.f, -1.f)}; break;
    case K_T: m = {one, z, z, mk(t, t)}; break;
    case K_TDG: m = {one, z, z, mk(t, -t)}; break;
    case K_SX: m = {mk(.5f, .5f), mk(.5f, -.5f), mk(.5f, -.5f), mk(.5f, .5f)}; break;
    default: m = {one, z, z, one}; break;
  }
  if (inv) m = {conjf2(m.a), conjf2(m.c), conjf2(m.b), conjf2(m.d)};
  return m;
}

__device__ __forceinline__ M2 m2mul(const M2& x, const M2& y) {  // x @ y
  return {cfma(x.b, y.c, cmul(x.a, y.a)), cfma(x.b, y.d, cmul(x.a, y.b)),
          cfma(x.d, y.c, cmul(x.c, y.a)), cfma(x.d, y.d, cmul(x.c, y.b))};
}

// value of physical bit p for register r of thread tl in the tile with non-tile base gbase
template <int RB>
__device__ __forceinline__ int pbit(int p, int r, int tl, uint32_t gbase) {
  if (p < RB) return (r >> p) & 1;
  if (p < PHYS_NONTILE) return (tl >> (p - RB)) & 1;
  return (gbase >> (p - PHYS_NONTILE)) & 1;
}

template <int R, int RBT>
__device__ __forceinline__ void m2_apply(float2 (&a)[R], const M2& m) {
#pragma unroll
  for (int r = 0; r < R; ++r) {
    if (r & (1 << RBT)) continue;
    const int r1 = r | (1 << RBT);
    const float2 x = a[r], y = a[r1];
    a[r] = cfma(m.b, y, cmul(m.a, x));
    a[r1] = cfma(m.d, y, cmul(m.c, x));
  }
}

// adjoint step for one gate on register bit RBT: gradient partial, then the inverse gate on psi
// and lambda.  CLS (compile time): 0 generic non-diagonal, 1 diagonal, 2 RX (grad X), 3 RY (grad Y),
// 4 RZ/P (grad Z, diagonal)
enum { CLS_GEN = 0, CLS_DIAG = 1, CLS_RX = 2, CLS_RY = 3, CLS_RZ = 4 };
template <int R, int RBT, int CLS>
__device__ __forceinline__ float adj_step(float2 (&a)[R], float2 (&l)[R], const M2& mi) {
  float acc = 0.f;
#pragma unroll
  for (int r = 0; r < R; ++r) {
    if (r & (1 << RBT)) continue;
    const int r1 = r | (1 << RBT);
    const float2 p0 = a[r], p1 = a[r1], l0 = l[r], l1 = l[r1];
    if constexpr (CLS == CLS_RX) acc += imcl(l0, p1) + imcl(l1, p0);
    if constexpr (CLS == CLS_RY) acc += recl(l1, p0) - recl(l0, p1);
    if constexpr (CLS == CLS_RZ) acc += imcl(l0, p0) - imcl(l1, p1);
    if constexpr (CLS == CLS_DIAG || CLS == CLS_RZ) {
      a[r] = cmul(mi.a, p0);
      a[r1] = cmul(mi.d, p1);
      l[r] = cmul(mi.a, l0);
      l[r1] = cmul(mi.d, l1);
    } else if constexpr (CLS == CLS_RX) {   // RX^dag = [[c, i s], [i s, c]]: real c, imaginary off-diagonal
      const float c = mi.a.x, s = mi.b.y;
      a[r] = mk(fmaf(c, p0.x, -s * p1.y), fmaf(c, p0.y, s * p1.x));
      a[r1] = mk(fmaf(c, p1.x, -s * p0.y), fmaf(c, p1.y, s * p0.x));
      l[r] = mk(fmaf(c, l0.x, -s * l1.y), fmaf(c, l0.y, s * l1.x));
      l[r1] = mk(fmaf(c, l1.x, -s * l0.y), fmaf(c, l1.y, s * l0.x));
    } else if constexpr (CLS == CLS_RY) {   // RY^dag = [[c, s], [-s, c]] real
      const float c = mi.a.x, s = mi.b.x;
      a[r] = mk(fmaf(c, p0.x, s * p1.x), fmaf(c, p0.y, s * p1.y));
      a[r1] = mk(fmaf(c, p1.x, mi.c.x * p0.x), fmaf(c, p1.y, mi.c.x * p0.y));
      l[r] = mk(fmaf(c, l0.x, s * l1.x), fmaf(c, l0.y, s * l1.y));
      l[r1] = mk(fmaf(c, l1.x, mi.c.x * l0.x), fmaf(c, l1.y, mi.c.x * l0.y));
    } else {
      a[r] = cfma(mi.b, p1, cmul(mi.a, p0));
      a[r1] = cfma(mi.d, p1, cmul(mi.c, p0));
      l[r] = cfma(mi.b, l1, cmul(mi.a, l0));
      l[r1] = cfma(mi.d, l1, cmul(mi.c, l0));
    }
  }
  return acc;
}

#define QFX_CLS_DISPATCH(cls, RBT_, OUT)                                   \
  switch (cls) {                                                         \
    case CLS_GEN: OUT = adj_step<R, RBT_, CLS_GEN>(a, l, mi); break;      \
    case CLS_DIAG: OUT = adj_step<R, RBT_, CLS_DIAG>(a, l, mi); break;    \
    case CLS_RX: OUT = adj_step<R, RBT_, CLS_RX>(a, l, mi); break;        \
    case CLS_RY: OUT = adj_step<R, RBT_, CLS_RY>(a, l, mi); break;        \
    default: OUT = adj_step<R, RBT_, CLS_RZ>(a, l, mi); break;            \
  }

template <int R, int RB, int TT, bool ADJ>
__device__ __forceinline__ void cx_apply(float2 (&a)[R], float2 (&l)[R], int ctl, int tl, uint32_t gbase) {
#pragma unroll
  for (int r = 0; r < R; ++r) {
    if (r & (1 << TT)) continue;
    const int r1 = r | (1 << TT);
    const bool c = pbit<RB>(ctl, r, tl, gbase);
    const float2 x = a[r], y = a[r1];
    a[r] = c ? y : x;
    a[r1] = c ? x : y;
    if constexpr (ADJ) {
      const float2 lx = l[r], ly = l[r1];
      l[r] = c ? ly : lx;
      l[r1] = c ? lx : ly;
    }
  }
}

// compile-time register-bit dispatch (explicit switch: keeps a[]/l[] in VGPRs - a lambda taking the
// arrays by reference is not force-inlined and demotes them to scratch)
#define QFX_RB_DISPATCH(rb, STMT)                                          \
  switch (rb) {                                                            \
    case 0: { constexpr int RBT = 0; STMT; } break;                        \
    case 1: { constexpr int RBT = 1; STMT; } break;                        \
    case 2: if constexpr (R >= 8) { constexpr int RBT = 2; STMT; } break;  \
    case 3: if constexpr (R >= 16) { constexpr int RBT = 3; STMT; } break; \
    case 4: if constexpr (R >= 32) { constexpr int RBT = 4; STMT; } break; \
    default: break;                                                        \
  }

// XOR of table entries selected by the bits of tl (thread-bit contributions)
__device__ __forceinline__ uint32_t xor_bits(cint_p tab, int tb, int tl) {
  uint32_t v = 0;
  for (int j = 0; j < tb; ++j) v ^= ((tl >> j) & 1) ? (uint32_t)tab[j] : 0u;
  return v;
}

template <int R>
__device__ __forceinline__ void do_remap(float2 (&a)[R], float2* __restrict__ xb, cint_p tab, int tb, int tl) {
  cint_p wr = tab;
  cint_p wt = tab + R;
  cint_p rr = tab + R + tb;
  cint_p rt = tab + 2 * R + tb;
  const uint32_t wthr = xor_bits(wt, tb, tl);
  const uint32_t rthr = xor_bits(rt, tb, tl);
  __syncthreads();  // WAR: previous readers of xb are done
#pragma unroll
  for (int r = 0; r < R; ++r) xb[(uint32_t)wr[r] ^ wthr] = a[r];
  __syncthreads();
#pragma unroll
  for (int r = 0; r < R; ++r) a[r] = xb[(uint32_t)rr[r] ^ rthr];
}

// wave-level sum over the T lanes of a tile group (T power of two <= 64)
__device__ __forceinline__ float group_sum(float v, int T) {
  for (int o = (T < 64 ? T : 64) >> 1; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// one-qubit prefix vector: (prefix gates of q) |0>
__device__ __forceinline__ float4 prefix_vec(cint_p blob, int q, const float* prow, const float* xrow,
                                             int n_theta) {
  cint_p gt = blob + blob[HF_GATES];
  cint_p pl = blob + blob[blob[HF_PREFIX] + q];
  const int cnt = pl[0];
  float2 v0 = mk(1.f, 0.f), v1 = mk(0.f, 0.f);
  for (int i = 0; i < cnt; ++i) {
    const int gi = pl[1 + i];
    const M2 m = gate_m2(gt[gi * GATE_WORDS], gate_cs(gt, gi, prow, xrow, n_theta), false);
    const float2 n0 = cfma(m.b, v1, cmul(m.a, v0));
    const float2 n1 = cfma(m.d, v1, cmul(m.c, v0));
    v0 = n0;
    v1 = n1;
  }
  return make_float4(v0.x, v0.y, v1.x, v1.y);
}

struct PassArgs {
  const int* blob;
  int pass_off;
  float2* psi;           // [n_samples, 2^n]
  float2* lam;           // adjoint only
  const float* params;   // [n_clients, p_stride]
  int p_stride;
  int spc;               // samples per client (sample s uses params row s / spc)
  const float* xang;     // [n_samples, x_stride]
  int x_stride;
  const float* w_read;   // [n_samples, C] dL/d<Z_c> (adjoint lambda init)
  float* out_read;       // [tiles_total, C] readout partials
  float* gslab;          // [tiles_total, n_gates] gradient partials
  int n_samples;
  int n_grad;            // grad partial slots (max over passes) reserved in LDS
};

}  // namespace qfx
