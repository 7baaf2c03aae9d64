// gfx950 (MI355X / CDNA4) statevector pass kernels: forward, readout, adjoint gradients.
//
// Replaces the reference's CPU Qiskit simulation (src/QFed/qAmplitude.py:44-46) and implements the
// ROADMAP VQC (ROADMAP.md:20-23,125-135) - SURVEY kernels K9/K11 (state init), K12 (gates),
// K13/K14 (<Z> readout), K16 (adjoint differentiation).
//
// Execution model (see qfx_plan.h): one launch = one pass over every 2^k-amplitude tile of every
// sample.  A 256-thread workgroup (4 wave64s) holds 256*R amplitudes in REGISTERS (R per lane);
// gates on register bits are VALU-only, gates on thread bits are reached through LDS "remaps"
// (one 16*R-byte write + read per lane per remap, XOR-swizzled slots), which also apply fused
// CNOT-chain permutations for free.  Small states (n <= 12) fit one tile -> the whole circuit is
// one launch with zero HBM traffic for the state; 16-24 qubit states stream once per pass with
// 128-byte coalesced rows.  Adjoint mode carries psi and lambda together and reduces every
// parameter's Im<lambda|P|psi> deterministically (wave64 xor-tree, fixed-order cross-wave sum).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <type_traits>

#include "qfx_plan.h"

namespace qfx {

struct M2 { float2 a, b, c, d; };   // [[a, b], [c, d]]
struct D2 { float2 d0, d1; };       // diag(d0, d1)

__device__ __forceinline__ float2 cmul(float2 a, float2 b) {
  return make_float2(a.x * b.x - a.y * b.y, a.x * b.y + a.y * b.x);
}
__device__ __forceinline__ float2 cfma(float2 a, float2 b, float2 c) {  // a*b + c
  return make_float2(fmaf(a.x, b.x, fmaf(-a.y, b.y, c.x)), fmaf(a.x, b.y, fmaf(a.y, b.x, c.y)));
}
__device__ __forceinline__ float2 mk(float x, float y) { return make_float2(x, y); }
__device__ __forceinline__ float2 conjf2(float2 a) { return make_float2(a.x, -a.y); }

__device__ __forceinline__ bool kind_is_diag(int k) {
  return k == K_RZ || k == K_P || k == K_Z || k == K_S || k == K_SDG || k == K_T || k == K_TDG;
}

__device__ __forceinline__ float gate_angle(const int* __restrict__ gt, int gi, const float* prow,
                                            const float* xrow, int n_theta) {
  const int* e = gt + gi * GATE_WORDS;
  const int slot = e[3];
  float v = 0.f;
  if (slot >= 0) v = slot < n_theta ? prow[slot] : xrow[slot - n_theta];
  return fmaf(__int_as_float(e[4]), v, __int_as_float(e[5]));
}

__device__ __forceinline__ M2 gate_m2(int kind, float ang, bool inv) {
  const float r2 = 0.70710678118654752f;
  float s, c;
  sincosf(0.5f * ang, &s, &c);
  if (inv) s = -s;
  switch (kind) {
    case K_RX: return {mk(c, 0.f), mk(0.f, -s), mk(0.f, -s), mk(c, 0.f)};
    case K_RY: return {mk(c, 0.f), mk(-s, 0.f), mk(s, 0.f), mk(c, 0.f)};
    case K_H: return {mk(r2, 0.f), mk(r2, 0.f), mk(r2, 0.f), mk(-r2, 0.f)};
    case K_X: return {mk(0.f, 0.f), mk(1.f, 0.f), mk(1.f, 0.f), mk(0.f, 0.f)};
    case K_Y: return {mk(0.f, 0.f), mk(0.f, -1.f), mk(0.f, 1.f), mk(0.f, 0.f)};
    case K_SX:
      if (!inv) return {mk(.5f, .5f), mk(.5f, -.5f), mk(.5f, -.5f), mk(.5f, .5f)};
      return {mk(.5f, -.5f), mk(.5f, .5f), mk(.5f, .5f), mk(.5f, -.5f)};
    default: return {mk(1.f, 0.f), mk(0.f, 0.f), mk(0.f, 0.f), mk(1.f, 0.f)};
  }
}

__device__ __forceinline__ D2 gate_d2(int kind, float ang, bool inv) {
  float2 d0 = mk(1.f, 0.f), d1 = mk(1.f, 0.f);
  const float t = 0.70710678118654752f;
  switch (kind) {
    case K_RZ: {
      float s, c;
      sincosf(0.5f * ang, &s, &c);
      d0 = mk(c, -s);
      d1 = mk(c, s);
      break;
    }
    case K_P: {
      float s, c;
      sincosf(ang, &s, &c);
      d1 = mk(c, s);
      break;
    }
    case K_Z: d1 = mk(-1.f, 0.f); break;
    case K_S: d1 = mk(0.f, 1.f); break;
    case K_SDG: d1 = mk(0.f, -1.f); break;
    case K_T: d1 = mk(t, t); break;
    case K_TDG: d1 = mk(t, -t); break;
    default: break;
  }
  if (inv) { d0 = conjf2(d0); d1 = conjf2(d1); }
  return {d0, d1};
}

// value of physical bit p for register r of thread tl in the tile with non-tile base gbase
template <int RB>
__device__ __forceinline__ int pbit(int p, int r, int tl, uint32_t gbase) {
  if (p < RB) return (r >> p) & 1;
  if (p < PHYS_NONTILE) return (tl >> (p - RB)) & 1;
  return (gbase >> (p - PHYS_NONTILE)) & 1;
}

template <int R, int RBT>
__device__ __forceinline__ void u1_apply(float2 (&a)[R], const M2& m) {
#pragma unroll
  for (int r = 0; r < R; ++r) {
    if (r & (1 << RBT)) continue;
    const int r1 = r | (1 << RBT);
    const float2 x = a[r], y = a[r1];
    a[r] = cfma(m.b, y, cmul(m.a, x));
    a[r1] = cfma(m.d, y, cmul(m.c, x));
  }
}

// Im<l|G|p> over this lane's pairs on register bit RBT; G = X (gen 0) or Y (gen 1)
template <int R, int RBT>
__device__ __forceinline__ float u1_grad(const float2 (&p)[R], const float2 (&l)[R], int gen) {
  float acc = 0.f;
#pragma unroll
  for (int r = 0; r < R; ++r) {
    if (r & (1 << RBT)) continue;
    const int r1 = r | (1 << RBT);
    const float2 p0 = p[r], p1 = p[r1], l0 = l[r], l1 = l[r1];
    if (gen == 0) {   // Im(conj(l0) p1 + conj(l1) p0)
      acc += l0.x * p1.y - l0.y * p1.x + l1.x * p0.y - l1.y * p0.x;
    } else {          // -Re(conj(l0) p1) + Re(conj(l1) p0)
      acc += -(l0.x * p1.x + l0.y * p1.y) + (l1.x * p0.x + l1.y * p0.y);
    }
  }
  return acc;
}

template <int R, typename F>
__device__ __forceinline__ void with_rbit(int rb, F&& f) {
  switch (rb) {
    case 0: f(std::integral_constant<int, 0>{}); break;
    case 1: f(std::integral_constant<int, 1>{}); break;
    case 2:
      if constexpr (R >= 8) f(std::integral_constant<int, 2>{});
      break;
    case 3:
      if constexpr (R >= 16) f(std::integral_constant<int, 3>{});
      break;
    case 4:
      if constexpr (R >= 32) f(std::integral_constant<int, 4>{});
      break;
    default: break;
  }
}

__device__ __forceinline__ uint32_t apply_map(uint32_t x, const int* __restrict__ rows, int k) {
  uint32_t y = 0;
  for (int j = 0; j < k; ++j) y |= (uint32_t)(__popc(x & (uint32_t)rows[j]) & 1) << j;
  return y;
}

__device__ __forceinline__ uint32_t swz(uint32_t s, int k) {
  // spread high tile bits over the low 5 bits: lanes that differ only in high tile bits then hit
  // different LDS banks (ds_write_b64: 16-lane groups mod 16 slots; ds_read_b64: 32-lane mod 32)
  return k >= 10 ? (s ^ ((s >> 5) & 31u)) : (k >= 6 ? (s ^ ((s >> 5) & 15u)) : s);
}

// wave-level sum over the T lanes of a tile group (T power of two <= 64)
__device__ __forceinline__ float group_sum(float v, int T) {
  for (int o = (T < 64 ? T : 64) >> 1; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

template <int R, int RB>
__device__ __forceinline__ void do_remap(float2 (&a)[R], float2* __restrict__ xb,
                                         const int* __restrict__ blob, int old_lay, int new_lay,
                                         int map_off, int k, int tl) {
  uint32_t tthr = 0;
  for (int p = RB; p < k; ++p) tthr |= (uint32_t)((tl >> (p - RB)) & 1) << blob[old_lay + p];
  if (map_off >= 0) tthr = apply_map(tthr, blob + map_off, k);
  __syncthreads();  // WAR: previous readers of xb are done
#pragma unroll
  for (int r = 0; r < R; ++r) {
    uint32_t treg = 0;
#pragma unroll
    for (int p = 0; p < RB; ++p)
      if ((r >> p) & 1) treg |= 1u << blob[old_lay + p];
    if (map_off >= 0) treg = apply_map(treg, blob + map_off, k);
    xb[swz(treg ^ tthr, k)] = a[r];
  }
  __syncthreads();
  uint32_t nthr = 0;
  for (int p = RB; p < k; ++p) nthr |= (uint32_t)((tl >> (p - RB)) & 1) << blob[new_lay + p];
#pragma unroll
  for (int r = 0; r < R; ++r) {
    uint32_t treg = 0;
#pragma unroll
    for (int p = 0; p < RB; ++p)
      if ((r >> p) & 1) treg |= 1u << blob[new_lay + p];
    a[r] = xb[swz(treg ^ nthr, k)];
  }
}

// global amplitude offset (within a sample) of register r, thread tl, under layout `lay`
template <int RB>
__device__ __forceinline__ uint32_t goff_thr(const int* __restrict__ blob, const int* __restrict__ pd,
                                             int lay, int k, int tl) {
  uint32_t g = 0;
  for (int p = RB; p < k; ++p)
    g |= (uint32_t)((tl >> (p - RB)) & 1) << pd[PF_TILEQ + blob[lay + p]];
  return g;
}
template <int RB>
__device__ __forceinline__ uint32_t goff_reg(const int* __restrict__ blob, const int* __restrict__ pd,
                                             int lay, int r) {
  uint32_t g = 0;
#pragma unroll
  for (int p = 0; p < RB; ++p)
    if ((r >> p) & 1) g |= 1u << pd[PF_TILEQ + blob[lay + p]];
  return g;
}

// one-qubit prefix vector: (prefix gates of q) |0>
__device__ __forceinline__ void prefix_vec(const int* __restrict__ blob, int q, const float* prow,
                                           const float* xrow, int n_theta, float2& v0, float2& v1) {
  const int* gt = blob + blob[HF_GATES];
  const int* pl = blob + blob[blob[HF_PREFIX] + q];
  const int cnt = pl[0];
  v0 = mk(1.f, 0.f);
  v1 = mk(0.f, 0.f);
  for (int i = 0; i < cnt; ++i) {
    const int gi = pl[1 + i];
    const int kind = gt[gi * GATE_WORDS];
    const float ang = gate_angle(gt, gi, prow, xrow, n_theta);
    if (kind_is_diag(kind)) {
      const D2 d = gate_d2(kind, ang, false);
      v0 = cmul(d.d0, v0);
      v1 = cmul(d.d1, v1);
    } else {
      const M2 m = gate_m2(kind, ang, false);
      const float2 n0 = cfma(m.b, v1, cmul(m.a, v0));
      const float2 n1 = cfma(m.d, v1, cmul(m.c, v0));
      v0 = n0;
      v1 = n1;
    }
  }
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
};

template <int R, bool ADJ>
__global__ void __launch_bounds__(256) qfx_pass_kernel(PassArgs A) {
  constexpr int RB = (R == 4) ? 2 : (R == 8) ? 3 : (R == 16) ? 4 : 5;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int* __restrict__ blob = A.blob;
  const int* __restrict__ pd = blob + A.pass_off;
  const int* __restrict__ gt = blob + blob[HF_GATES];
  const int n = blob[HF_N];
  const int n_theta = blob[HF_NTHETA];
  const int G = blob[HF_NGATES];
  const int k = pd[PF_K];
  const int tb = pd[PF_TB];
  const int T = 1 << tb;                     // threads per tile
  const int tid = threadIdx.x;
  const int tib = tid >> tb;                 // tile within block
  const int tl = tid & (T - 1);
  const int tiles_pb = 256 >> tb;
  const long tile = (long)blockIdx.x * tiles_pb + tib;
  const int ltps = n - k;
  const long sample = tile >> ltps;
  const uint32_t tau = (uint32_t)(tile & ((1L << ltps) - 1));
  const bool valid = sample < A.n_samples;
  const long s_eff = valid ? sample : 0;
  const size_t sbase = (size_t)s_eff << n;
  const float* prow = A.params + (size_t)(s_eff / A.spc) * A.p_stride;
  const float* xrow = A.xang + (size_t)s_eff * A.x_stride;
  const int wave = tid >> 6;
  const int lane = tid & 63;

  uint32_t gbase = 0;
  {
    const int nn = pd[PF_NNONTILE];
    for (int j = 0; j < nn; ++j) gbase |= ((tau >> j) & 1u) << pd[PF_NONTILE + j];
  }
  float2* xb = reinterpret_cast<float2*>(smem) + (size_t)tib * (1u << k);
  float* red = reinterpret_cast<float*>(smem + 256 * R * sizeof(float2));   // [64] readout scratch
  float* gacc = red + 64;                                                    // [n_grad][5]

  float2 a[R];
  float2 l[R];
#pragma unroll
  for (int r = 0; r < R; ++r) l[r] = mk(0.f, 0.f);
  int lay = pd[PF_LAYOUT0];
  const int init = pd[PF_INIT];

  // ------------------------------------------------------------------ init
  if (init == INIT_PRODUCT) {
    float2 base = mk(1.f, 0.f);
    const int nn = pd[PF_NNONTILE];
    for (int j = 0; j < nn; ++j) {
      const int q = pd[PF_NONTILE + j];
      float2 v0, v1;
      prefix_vec(blob, q, prow, xrow, n_theta, v0, v1);
      base = cmul(base, ((gbase >> q) & 1u) ? v1 : v0);
    }
    for (int p = RB; p < k; ++p) {
      const int q = pd[PF_TILEQ + blob[lay + p]];
      float2 v0, v1;
      prefix_vec(blob, q, prow, xrow, n_theta, v0, v1);
      base = cmul(base, ((tl >> (p - RB)) & 1) ? v1 : v0);
    }
    a[0] = base;
#pragma unroll
    for (int p = 0; p < RB; ++p) {
      const int q = pd[PF_TILEQ + blob[lay + p]];
      float2 v0, v1;
      prefix_vec(blob, q, prow, xrow, n_theta, v0, v1);
#pragma unroll
      for (int r = 0; r < (1 << p); ++r) {
        a[r | (1 << p)] = cmul(a[r], v1);
        a[r] = cmul(a[r], v0);
      }
    }
  } else {
    const uint32_t gthr = goff_thr<RB>(blob, pd, lay, k, tl);
#pragma unroll
    for (int r = 0; r < R; ++r) {
      const size_t off = sbase + gbase + gthr + goff_reg<RB>(blob, pd, lay, r);
      a[r] = valid ? A.psi[off] : mk(0.f, 0.f);
      if constexpr (ADJ) {
        if (init == INIT_LOAD_BOTH) l[r] = valid ? A.lam[off] : mk(0.f, 0.f);
      }
    }
    if constexpr (ADJ) {
      if (init == INIT_PSI_LAMBDA) {
        const int C = pd[PF_NREAD];
#pragma unroll
        for (int r = 0; r < R; ++r) {
          float s = 0.f;
          for (int c = 0; c < C; ++c) {
            const float w = valid ? A.w_read[(size_t)s_eff * C + c] : 0.f;
            s += pbit<RB>(pd[PF_LAM_PHYS + c], r, tl, gbase) ? -w : w;
          }
          l[r] = mk(a[r].x * s, a[r].y * s);
        }
      }
    }
  }

  // ------------------------------------------------------------------ micro-ops
  const int nops = pd[PF_NOPS];
  const int* __restrict__ ops = blob + pd[PF_OPS];
  int gcount = 0;
  for (int i = 0; i < nops; ++i) {
    const int code = ops[i * OP_WORDS + 0];
    const int oa = ops[i * OP_WORDS + 1];
    const int ob = ops[i * OP_WORDS + 2];
    const int oc = ops[i * OP_WORDS + 3];
    if (code == OP_REMAP) {
      do_remap<R, RB>(a, xb, blob, lay, oa, ob, k, tl);
      if constexpr (ADJ) do_remap<R, RB>(l, xb, blob, lay, oa, ob, k, tl);
      lay = oa;
      continue;
    }
    const int kind = gt[oc * GATE_WORDS];
    const int slot = gt[oc * GATE_WORDS + 3];
    if (code == OP_U1) {
      const float ang = gate_angle(gt, oc, prow, xrow, n_theta);
      const M2 m = gate_m2(kind, ang, ADJ);
      if constexpr (ADJ) {
        if (slot >= 0 && slot < n_theta && (kind == K_RX || kind == K_RY)) {
          float part = 0.f;
          with_rbit<R>(oa, [&](auto RBT) { part = u1_grad<R, decltype(RBT)::value>(a, l, kind == K_RX ? 0 : 1); });
          part = group_sum(part, T);
          if (T <= 64) {
            if (tl == 0 && valid) A.gslab[(size_t)tile * G + oc] = part;
          } else if (lane == 0) {
            gacc[gcount * 5 + wave] = part;
            if (wave == 0) gacc[gcount * 5 + 4] = __int_as_float(oc);
          }
          ++gcount;
        }
        with_rbit<R>(oa, [&](auto RBT) {
          u1_apply<R, decltype(RBT)::value>(a, m);
          u1_apply<R, decltype(RBT)::value>(l, m);
        });
      } else {
        with_rbit<R>(oa, [&](auto RBT) { u1_apply<R, decltype(RBT)::value>(a, m); });
      }
    } else if (code == OP_D1) {
      const float ang = gate_angle(gt, oc, prow, xrow, n_theta);
      const D2 d = gate_d2(kind, ang, ADJ);
      if constexpr (ADJ) {
        if (slot >= 0 && slot < n_theta && (kind == K_RZ || kind == K_P)) {
          float part = 0.f;
#pragma unroll
          for (int r = 0; r < R; ++r) {
            const float im = l[r].x * a[r].y - l[r].y * a[r].x;
            part += pbit<RB>(oa, r, tl, gbase) ? -im : im;
          }
          part = group_sum(part, T);
          if (T <= 64) {
            if (tl == 0 && valid) A.gslab[(size_t)tile * G + oc] = part;
          } else if (lane == 0) {
            gacc[gcount * 5 + wave] = part;
            if (wave == 0) gacc[gcount * 5 + 4] = __int_as_float(oc);
          }
          ++gcount;
        }
      }
#pragma unroll
      for (int r = 0; r < R; ++r) {
        const float2 ph = pbit<RB>(oa, r, tl, gbase) ? d.d1 : d.d0;
        a[r] = cmul(a[r], ph);
        if constexpr (ADJ) l[r] = cmul(l[r], ph);
      }
    } else if (code == OP_CX) {
      with_rbit<R>(ob, [&](auto RBT) {
        constexpr int TT = decltype(RBT)::value;
#pragma unroll
        for (int r = 0; r < R; ++r) {
          if (r & (1 << TT)) continue;
          const int r1 = r | (1 << TT);
          const bool c = pbit<RB>(oa, r, tl, gbase);
          const float2 x = a[r], y = a[r1];
          a[r] = c ? y : x;
          a[r1] = c ? x : y;
          if constexpr (ADJ) {
            const float2 lx = l[r], ly = l[r1];
            l[r] = c ? ly : lx;
            l[r1] = c ? lx : ly;
          }
        }
      });
    } else if (code == OP_CZ) {
#pragma unroll
      for (int r = 0; r < R; ++r) {
        const bool neg = pbit<RB>(oa, r, tl, gbase) & pbit<RB>(ob, r, tl, gbase);
        if (neg) {
          a[r] = mk(-a[r].x, -a[r].y);
          if constexpr (ADJ) l[r] = mk(-l[r].x, -l[r].y);
        }
      }
    }
  }

  // ------------------------------------------------------------------ finalize
  const int fin = pd[PF_FINAL];
  if constexpr (ADJ) {
    if (T > 64) {
      __syncthreads();
      for (int g = tid; g < gcount; g += 256) {
        const float sum = gacc[g * 5 + 0] + gacc[g * 5 + 1] + gacc[g * 5 + 2] + gacc[g * 5 + 3];
        if (valid) A.gslab[(size_t)tile * G + __float_as_int(gacc[g * 5 + 4])] = sum;
      }
    }
  }
  if (fin & FIN_READOUT) {
    const int C = pd[PF_NREAD];
    for (int c = 0; c < C; ++c) {
      const int ph = pd[PF_READ_PHYS + c];
      float acc = 0.f;
#pragma unroll
      for (int r = 0; r < R; ++r) {
        const float pr = a[r].x * a[r].x + a[r].y * a[r].y;
        acc += pbit<RB>(ph, r, tl, gbase) ? -pr : pr;
      }
      acc = group_sum(acc, T);
      if (T <= 64) {
        if (tl == 0 && valid) A.out_read[(size_t)tile * C + c] = acc;
      } else {
        if (lane == 0) red[c * 4 + wave] = acc;
      }
    }
    if (T > 64) {
      __syncthreads();
      if (tid < C && valid)
        A.out_read[(size_t)tile * C + tid] = red[tid * 4 + 0] + red[tid * 4 + 1] + red[tid * 4 + 2] + red[tid * 4 + 3];
    }
  }
  if (fin & FIN_STORE) {
    const uint32_t gthr = goff_thr<RB>(blob, pd, lay, k, tl);
    if (valid) {
#pragma unroll
      for (int r = 0; r < R; ++r) {
        const size_t off = sbase + gbase + gthr + goff_reg<RB>(blob, pd, lay, r);
        A.psi[off] = a[r];
        if constexpr (ADJ) A.lam[off] = l[r];
      }
    }
  }
}

}  // namespace qfx

// ----------------------------------------------------------------------------------- launchers
extern "C" int qfx_launch_pass(int R, int adjoint, const int* blob, int pass_off, int k, int n,
                               float2* psi, float2* lam, const float* params, int p_stride, int spc,
                               const float* xang, int x_stride, const float* w_read, float* out_read,
                               float* gslab, int n_samples, int n_grad_ops, hipStream_t stream) {
  using namespace qfx;
  const int tb = k - (R == 4 ? 2 : R == 8 ? 3 : R == 16 ? 4 : 5);
  const int tiles_pb = 256 >> tb;
  const long tiles_total = (long)n_samples << (n - k);
  const long blocks = (tiles_total + tiles_pb - 1) / tiles_pb;
  if (blocks <= 0) return 0;
  PassArgs A{blob, pass_off, psi, lam, params, p_stride, spc, xang, x_stride, w_read, out_read, gslab, n_samples};
  const size_t lds = 256 * (size_t)R * sizeof(float2) + 64 * sizeof(float) +
                     (size_t)n_grad_ops * 5 * sizeof(float);
  dim3 grid((unsigned)blocks), block(256);
#define QFX_L(RR, AA)                                                                     \
  hipLaunchKernelGGL((qfx_pass_kernel<RR, AA>), grid, block, lds, stream, A)
  if (R == 4) { if (adjoint) QFX_L(4, true); else QFX_L(4, false); }
  else if (R == 16) { if (adjoint) QFX_L(16, true); else QFX_L(16, false); }
  else return -1;
#undef QFX_L
  return (int)hipGetLastError();
}
