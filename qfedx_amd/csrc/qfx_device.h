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

// Complex amplitudes are native 2-wide float vectors: every complex op below is written so that the
// gfx950 backend emits packed fp32 math (v_pk_mul_f32 / v_pk_fma_f32, two lanes of math per issue)
// with the re/im swap and sign flips folded into op_sel / neg modifiers - a complex multiply is 2
// packed instructions, an Im(conj(l) p) accumulation 1.
typedef float v2f __attribute__((ext_vector_type(2)));

struct M2 { v2f a, b, c, d; };   // [[a, b], [c, d]]

__device__ __forceinline__ v2f mk(float x, float y) { return v2f{x, y}; }
__device__ __forceinline__ v2f splat(float x) { return v2f{x, x}; }
__device__ __forceinline__ v2f sw(v2f v) { return __builtin_shufflevector(v, v, 1, 0); }
__device__ __forceinline__ v2f pfma(v2f a, v2f b, v2f c) { return __builtin_elementwise_fma(a, b, c); }
// a * b  (put the gate-uniform factor in `a`: its splat / sign vector is hoisted out of loops)
// (the re/im swap is applied to a fresh product, never to a state register: swaps of state registers
// get CSE'd across gates and then materialised with v_pk_mov instead of folding into op_sel)
__device__ __forceinline__ v2f cmul(v2f a, v2f b) { return pfma(splat(a.x), b, sw(b * mk(a.y, -a.y))); }
// a * b + c
__device__ __forceinline__ v2f cfma(v2f a, v2f b, v2f c) { return pfma(splat(a.x), b, sw(pfma(b, mk(a.y, -a.y), sw(c)))); }
// bf16 statevector storage (state_dtype=bf16): one amplitude = bf16 re | bf16 im << 16 in 32 bits;
// compute stays fp32, stores round to nearest even
__device__ __forceinline__ v2f unpack_bf16x2(uint32_t u) {
  return mk(__uint_as_float(u << 16), __uint_as_float(u & 0xffff0000u));
}
__device__ __forceinline__ uint32_t bf16_rne(float f) {
  uint32_t u = __float_as_uint(f);
  u += 0x7fffu + ((u >> 16) & 1u);
  return u >> 16;
}
__device__ __forceinline__ uint32_t pack_bf16x2(v2f v) { return bf16_rne(v.x) | (bf16_rne(v.y) << 16); }
__device__ __forceinline__ v2f conjf2(v2f a) { return mk(a.x, -a.y); }
__device__ __forceinline__ float imcl(v2f l, v2f p) { return l.x * p.y - l.y * p.x; }  // Im(conj(l) p)
__device__ __forceinline__ float recl(v2f l, v2f p) { return l.x * p.x + l.y * p.y; }  // Re(conj(l) p)
// packed accumulators: Im(conj(l) p) = acc.x - acc.y after acc = pfma(l, sw(p), acc);
//                      Re(conj(l) p) = acc.x + acc.y after acc = pfma(l, p, acc)
__device__ __forceinline__ v2f acc_im(v2f acc, v2f l, v2f p) { return pfma(l, sw(p), acc); }
__device__ __forceinline__ v2f acc_re(v2f acc, v2f l, v2f p) { return pfma(l, p, acc); }

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
__device__ __forceinline__ v2f gate_cs(cint_p gt, int gi, const float* prow,
                                          const float* xrow, int n_theta) {
  const float ang = gate_angle(gt, gi, prow, xrow, n_theta);
  if (gt[gi * GATE_WORDS] == K_PAULI) return mk(ang, 0.f);   // Pauli index, no trig
  const float x = gt[gi * GATE_WORDS] == K_P ? ang : 0.5f * ang;
  float s, c;
  sincosf(x, &s, &c);
  return mk(c, s);
}

// full 2x2 (diagonal kinds too); inverse = conjugate transpose
__device__ __forceinline__ M2 gate_m2(int kind, v2f cs, bool inv) {
  const float r2 = 0.70710678118654752f, t = 0.70710678118654752f;
  const float c = cs.x, s = cs.y;
  M2 m;
  const v2f z = mk(0.f, 0.f), one = mk(1.f, 0.f);
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
    case K_PAULI: {   // trajectory Pauli: 0 I, 1 X, 2 Y, 3 Z (Hermitian: its own inverse)
      const int pc = (int)(c + 0.5f);
      if (pc == 1) m = {z, one, one, z};
      else if (pc == 2) m = {z, mk(0.f, -1.f), mk(0.f, 1.f), z};
      else if (pc == 3) m = {one, z, z, mk(-1.f, 0.f)};
      else m = {one, z, z, one};
    } break;
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

// 2x2 complex matvec row:  m0 * x + m1 * y  in 4 packed instructions.  cmul(a, x) = a.x*x + sw(x*(a.y,-a.y)),
// so the single re/im swap lands on a one-use temporary and folds into op_sel (a swap of x or y
// itself would be shared by both output rows and materialised with v_pk_mov).
__device__ __forceinline__ v2f mrow(v2f m0, v2f m1, v2f x, v2f y) {
  const v2f t = pfma(x, mk(m0.y, -m0.y), mk(m1.y, -m1.y) * y);
  return pfma(splat(m0.x), x, pfma(splat(m1.x), y, sw(t)));
}

template <int R, int RBT>
__device__ __forceinline__ void m2_apply(v2f (&a)[R], const M2& m) {
#pragma unroll
  for (int r = 0; r < R; ++r) {
    if (r & (1 << RBT)) continue;
    const int r1 = r | (1 << RBT);
    const v2f x = a[r], y = a[r1];
    a[r] = mrow(m.a, m.b, x, y);
    a[r1] = mrow(m.c, m.d, x, y);
  }
}

// adjoint step for one gate on register bit RBT: the inverse gate on psi and lambda, then the
// gradient partial.  The generator (X, Y or Z) commutes with its own rotation, so
// Im<lambda|P|psi> is the same before and after un-applying the gate; taking it from the new values
// keeps every swapped operand single-use (foldable).  CLS (compile time): 0 generic non-diagonal,
// 1 diagonal, 2 RX (grad X), 3 RY (grad Y), 4 RZ/P (grad Z, diagonal)
enum { CLS_GEN = 0, CLS_DIAG = 1, CLS_RX = 2, CLS_RY = 3, CLS_RZ = 4 };
template <int R, int RBT, int CLS>
__device__ __forceinline__ float adj_step(v2f (&a)[R], v2f (&l)[R], const M2& mi) {
  v2f acc = mk(0.f, 0.f);
  // gate-uniform factors, hoisted out of the register loop
  const v2f c2 = splat(mi.a.x);
  const v2f rxs = mk(mi.b.y, -mi.b.y);      // RX^dag off-diagonal: i*s*p = sw(p * (s, -s))
  const v2f rys = splat(mi.b.x), rysn = splat(mi.c.x);
#pragma unroll
  for (int r = 0; r < R; ++r) {
    if (r & (1 << RBT)) continue;
    const int r1 = r | (1 << RBT);
    const v2f p0 = a[r], p1 = a[r1], l0 = l[r], l1 = l[r1];
    v2f q0, q1, m0, m1;
    if constexpr (CLS == CLS_DIAG || CLS == CLS_RZ) {
      q0 = cmul(mi.a, p0);
      q1 = cmul(mi.d, p1);
      m0 = cmul(mi.a, l0);
      m1 = cmul(mi.d, l1);
    } else if constexpr (CLS == CLS_RX) {   // RX^dag = [[c, i s], [i s, c]]
      q0 = pfma(c2, p0, sw(p1 * rxs));
      q1 = pfma(c2, p1, sw(p0 * rxs));
      m0 = pfma(c2, l0, sw(l1 * rxs));
      m1 = pfma(c2, l1, sw(l0 * rxs));
    } else if constexpr (CLS == CLS_RY) {   // RY^dag = [[c, s], [-s, c]] real
      q0 = pfma(c2, p0, rys * p1);
      q1 = pfma(c2, p1, rysn * p0);
      m0 = pfma(c2, l0, rys * l1);
      m1 = pfma(c2, l1, rysn * l0);
    } else {
      q0 = mrow(mi.a, mi.b, p0, p1);
      q1 = mrow(mi.c, mi.d, p0, p1);
      m0 = mrow(mi.a, mi.b, l0, l1);
      m1 = mrow(mi.c, mi.d, l0, l1);
    }
    a[r] = q0;
    a[r1] = q1;
    l[r] = m0;
    l[r1] = m1;
    if constexpr (CLS == CLS_RX) { acc = acc_im(acc, m0, q1); acc = acc_im(acc, m1, q0); }
    if constexpr (CLS == CLS_RY) { acc = acc_re(acc, m1, q0); acc = acc_re(acc, -m0, q1); }
    if constexpr (CLS == CLS_RZ) { acc = acc_im(acc, m0, q0); acc = acc_im(acc, -m1, q1); }
  }
  if constexpr (CLS == CLS_RY) return acc.x + acc.y;
  return acc.x - acc.y;
}

// gradient only (the gate's inverse is not needed by anything processed later): Im<lambda|P|psi> on
// the current values - equal to the post-inverse value because the generator commutes with its gate
template <int R, int RBT, int CLS>
__device__ __forceinline__ float adj_grad_only(const v2f (&a)[R], const v2f (&l)[R]) {
  v2f acc = mk(0.f, 0.f);
#pragma unroll
  for (int r = 0; r < R; ++r) {
    if (r & (1 << RBT)) continue;
    const int r1 = r | (1 << RBT);
    const v2f p0 = a[r], p1 = a[r1], l0 = l[r], l1 = l[r1];
    if constexpr (CLS == CLS_RX) { acc = acc_im(acc, l0, p1); acc = acc_im(acc, l1, p0); }
    if constexpr (CLS == CLS_RY) { acc = acc_re(acc, l1, p0); acc = acc_re(acc, -l0, p1); }
    if constexpr (CLS == CLS_RZ) { acc = acc_im(acc, l0, p0); acc = acc_im(acc, -l1, p1); }
  }
  if constexpr (CLS == CLS_RY) return acc.x + acc.y;
  return acc.x - acc.y;
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
__device__ __forceinline__ void cx_apply(v2f (&a)[R], v2f (&l)[R], int ctl, int tl, uint32_t gbase) {
#pragma unroll
  for (int r = 0; r < R; ++r) {
    if (r & (1 << TT)) continue;
    const int r1 = r | (1 << TT);
    const bool c = pbit<RB>(ctl, r, tl, gbase);
    const v2f x = a[r], y = a[r1];
    a[r] = c ? y : x;
    a[r1] = c ? x : y;
    if constexpr (ADJ) {
      const v2f lx = l[r], ly = l[r1];
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
__device__ __forceinline__ void do_remap(v2f (&a)[R], v2f* __restrict__ xb, cint_p tab, int tb, int tl) {
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

// DPP lane permutation inside a 16-lane row (VALU, no LDS round trip)
template <int CTRL>
__device__ __forceinline__ float dppf(float v) {
  return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), CTRL, 0xF, 0xF, false));
}

// sum over aligned groups of G <= 16 lanes with row-local DPP: xor 1, xor 2 (quad_perm), then the
// half-row and row mirrors (every lane of a quad / half-row already holds the same partial sum)
template <int G>
__device__ __forceinline__ float row_sum(float v) {
  if constexpr (G >= 2) v += dppf<0xB1>(v);    // quad_perm [1,0,3,2]
  if constexpr (G >= 4) v += dppf<0x4E>(v);    // quad_perm [2,3,0,1]
  if constexpr (G >= 8) v += dppf<0x141>(v);   // row_half_mirror
  if constexpr (G >= 16) v += dppf<0x140>(v);  // row_mirror
  return v;
}

// wave-level sum over the T lanes of a tile group (T power of two <= 64), runtime T
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
  v2f v0 = mk(1.f, 0.f), v1 = mk(0.f, 0.f);
  for (int i = 0; i < cnt; ++i) {
    const int gi = pl[1 + i];
    const M2 m = gate_m2(gt[gi * GATE_WORDS], gate_cs(gt, gi, prow, xrow, n_theta), false);
    const v2f n0 = cfma(m.b, v1, cmul(m.a, v0));
    const v2f n1 = cfma(m.d, v1, cmul(m.c, v0));
    v0 = n0;
    v1 = n1;
  }
  return make_float4(v0.x, v0.y, v1.x, v1.y);
}

struct PassArgs {
  const int* blob;
  int pass_off;
  v2f* psi;           // [n_samples, 2^n]
  v2f* lam;           // adjoint only
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
