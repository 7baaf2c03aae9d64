// Exact matrix-product-state contraction of ANY lowered circuit (1-qubit gates of every IR kind, CX / CZ at any
// distance) whose two-qubit gates put at most 4 bond bits on every cut (bond <= 16): the generic MPS backend's HIP
// path (tables and torch emulator: qfedx_amd/quantum/mps_mpo.py; the einsum network it replaces: quantum/mps.py).
//
// A two-qubit gate applied as the bond-2 MPO |0><0| (x) I + |1><1| (x) U adds one bit k_g to every cut between its
// qubits, and with no recompression the final MPS is known column by column: bit i of the word on cut c is the i-th
// two-qubit gate (program order) crossing c, and qubit q's tensor for left / right words (a, b) is
//     A_q[a, :, b] = E_m ... E_1 |0>
// over q's own events in program order - its 1-qubit gates, the projector P_{k_g} where q controls g, X^{k_g} /
// Z^{k_g} where q is g's target - and zero unless every gate passing over q (crossing both of its cuts) has the same
// bit in a and b.  One 256-thread workgroup per sample; thread (x, y) of the 16 x 16 grid builds the column (a, b) =
// (x, y) and owns entry (x, y) of every D x D transfer environment:
//   right sweep   R_q = sum_s conj(A_q[s]) R_{q+1} A_q[s]^T        (stored per cut)
//   <Z_c>         L_c, conj(A_c) Z A_c and R_{c+1}                  (left sweep up to the last readout qubit)
//   gradients     RO (O = sum_c w_c Z_c right of a cut) for the readout cuts, then a left sweep carrying L and LO:
//                 Ybar = d<O>/dA_q per column, pulled back through the column's events; each rotation's derivative
//                 2 Re(u . dG v) is summed over the 256 columns (fixed order: per-wave sums, then the four waves).
// Cost O(n D^3) per sample.  The torch network launches ~10 small batched GEMMs per gate.
#include <hip/hip_runtime.h>

#include <cstdint>

#include "mps_args.h"

namespace qfx_mpo {

constexpr int DM = QFX_MPO_DMAX, NT = DM * DM, NW = NT / 64;
constexpr int MAXPG = QFX_MPO_MAXPG, RMAX = QFX_MPS_RMAX;
enum { EV_GATE = 0, EV_CTRL = 1, EV_X = 2, EV_Z = 3 };
enum { K_RX = 0, K_RY, K_RZ, K_P, K_H, K_X, K_Y, K_Z, K_S, K_SDG, K_T, K_TDG, K_SX, K_PAULI = 18 };

__device__ __forceinline__ float2 mk(float a, float b) { return make_float2(a, b); }
__device__ __forceinline__ float2 cmul(float2 a, float2 b) { return mk(a.x * b.x - a.y * b.y, a.x * b.y + a.y * b.x); }
__device__ __forceinline__ float2 cjmul(float2 a, float2 b) { return mk(a.x * b.x + a.y * b.y, a.x * b.y - a.y * b.x); }
__device__ __forceinline__ float2 cadd(float2 a, float2 b) { return mk(a.x + b.x, a.y + b.y); }
__device__ __forceinline__ float2 csc(float2 a, float s) { return mk(a.x * s, a.y * s); }
__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

struct M2 {
  float2 a, b, c, d;   // [[a, b], [c, d]]
};

// 2 x 2 matrix of a 1-qubit gate (statevec_torch._u1): kind is uniform over the workgroup
__device__ M2 gate_mat(int kind, float th) {
  const float r2 = 0.70710678118654752f;
  const float2 o = mk(1.f, 0.f), z = mk(0.f, 0.f);
  float s, c;
  switch (kind) {
    case K_RX: sincosf(0.5f * th, &s, &c); return {mk(c, 0.f), mk(0.f, -s), mk(0.f, -s), mk(c, 0.f)};
    case K_RY: sincosf(0.5f * th, &s, &c); return {mk(c, 0.f), mk(-s, 0.f), mk(s, 0.f), mk(c, 0.f)};
    case K_RZ: sincosf(0.5f * th, &s, &c); return {mk(c, -s), z, z, mk(c, s)};
    case K_P: sincosf(th, &s, &c); return {o, z, z, mk(c, s)};
    case K_H: return {mk(r2, 0.f), mk(r2, 0.f), mk(r2, 0.f), mk(-r2, 0.f)};
    case K_X: return {z, o, o, z};
    case K_Y: return {z, mk(0.f, -1.f), mk(0.f, 1.f), z};
    case K_Z: return {o, z, z, mk(-1.f, 0.f)};
    case K_S: return {o, z, z, mk(0.f, 1.f)};
    case K_SDG: return {o, z, z, mk(0.f, -1.f)};
    case K_T: return {o, z, z, mk(r2, r2)};
    case K_TDG: return {o, z, z, mk(r2, -r2)};
    case K_SX: return {mk(.5f, .5f), mk(.5f, -.5f), mk(.5f, -.5f), mk(.5f, .5f)};
    default: {   // K_PAULI: per-sample trajectory Pauli, round(angle) = 0 / 1 / 2 / 3 = I / X / Y / Z
      const int ch = (int)rintf(th);
      const float i_ = ch == 0, x_ = ch == 1, y_ = ch == 2, z_ = ch == 3;
      return {mk(i_ + z_, 0.f), mk(x_, -y_), mk(x_, y_), mk(i_ - z_, 0.f)};
    }
  }
}

__device__ __forceinline__ bool rotation(int kind) { return kind <= K_P; }

// event e = type | side << 2 | bit << 3 | gate << 8 (side 0: bit of the left word a, 1: of the right word b)
__device__ __forceinline__ int ev_bit(int e, int a, int b) { return ((((e >> 2) & 1) ? b : a) >> ((e >> 3) & 3)) & 1; }

// forward: v <- E_e v (transpose = false) or pull-back u <- E_e^T u (transpose = true); projector, X and Z are
// symmetric
template <bool TR>
__device__ __forceinline__ void apply_ev(int e, const M2* m, int a, int b, float2& v0, float2& v1) {
  const int type = e & 3;
  if (type == EV_GATE) {
    const float2 n0 = TR ? cadd(cmul(m->a, v0), cmul(m->c, v1)) : cadd(cmul(m->a, v0), cmul(m->b, v1));
    const float2 n1 = TR ? cadd(cmul(m->b, v0), cmul(m->d, v1)) : cadd(cmul(m->c, v0), cmul(m->d, v1));
    v0 = n0;
    v1 = n1;
    return;
  }
  const int k = ev_bit(e, a, b);
  if (type == EV_CTRL) {
    if (k) v0 = mk(0.f, 0.f);
    else v1 = mk(0.f, 0.f);
  } else if (type == EV_X) {
    if (k) {
      const float2 t = v0;
      v0 = v1;
      v1 = t;
    }
  } else if (k) {
    v1 = mk(-v1.x, -v1.y);
  }
}

struct Site {
  const int* ev;
  int cnt, pt, npt, npg, Dl, Dr;
};

__device__ __forceinline__ Site site_of(const QfxMpoArgs& g, int q) {
  const int* si = g.sinfo + 8 * q;
  Site t;
  t.ev = g.events + si[0];
  t.cnt = si[1];
  t.pt = si[2];
  t.npt = si[3];
  t.npg = si[4];
  t.Dl = q == 0 ? 1 : 1 << g.nbits[q - 1];
  t.Dr = q == g.n - 1 ? 1 : 1 << g.nbits[q];
  return t;
}

// column (a, b) is nonzero only if every gate passing over the qubit carries the same bit on both cuts
__device__ __forceinline__ bool col_valid(const Site& t, int a, int b) {
  if (a >= t.Dl || b >= t.Dr) return false;
  for (int p = 0; p < t.npt; ++p) {
    const int i = (t.pt >> (4 * p)) & 3, j = (t.pt >> (4 * p + 2)) & 3;
    if (((a >> i) ^ (b >> j)) & 1) return false;
  }
  return true;
}

// E_{upto-1} ... E_0 |0> for column (a, b)
__device__ __forceinline__ void build_col(const Site& t, const float* ang, const int* gk, int a, int b, int upto,
                                          float2& v0, float2& v1) {
  v0 = mk(1.f, 0.f);
  v1 = mk(0.f, 0.f);
  for (int i = 0; i < upto; ++i) {
    const int e = t.ev[i];
    M2 m;
    if ((e & 3) == EV_GATE) m = gate_mat(gk[e >> 8], ang[e >> 8]);
    apply_ev<false>(e, &m, a, b, v0, v1);
  }
}

__global__ void __launch_bounds__(NT) mps_mpo_kernel(QfxMpoArgs g) {
  __shared__ float2 A0[NT], A1[NT];              // A[s][a * 16 + b]
  __shared__ float2 U1[2][NT], U2[2][NT];
  __shared__ float2 E1[NT], E2[NT], E3[NT], E4[NT];
  __shared__ float red[NW][MAXPG + RMAX];
  __shared__ int pg_s[MAXPG];
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int x = tid >> 4, y = tid & 15;
  const int s = blockIdx.x, n = g.n;
  const float* ang = g.ang + (size_t)s * g.G;
  float2* rp = reinterpret_cast<float2*>(g.rp) + (size_t)s * n * NT;
  const bool grad = g.w != nullptr;
  float wq[RMAX];
  int rq[RMAX];
#pragma unroll
  for (int i = 0; i < RMAX; ++i) {
    rq[i] = i < g.C ? g.readout[i] : -1;
    wq[i] = (grad && i < g.C) ? g.w[(size_t)s * g.C + i] : 0.f;
  }
  auto wof = [&](int q) {                        // weight of Z_q in O (0 off the readout)
    float v = 0.f;
#pragma unroll
    for (int i = 0; i < RMAX; ++i) v += rq[i] == q ? wq[i] : 0.f;
    return v;
  };
  auto put_col = [&](const Site& t) {            // A_q into LDS (zero outside the valid columns)
    float2 v0 = mk(0.f, 0.f), v1 = v0;
    if (col_valid(t, x, y)) build_col(t, ang, g.gkind, x, y, t.cnt, v0, v1);
    A0[tid] = v0;
    A1[tid] = v1;
  };
  // Y[a'][s][b] = sum_b' A[a',s,b'] Rin[b][b']      (thread (a', b))
  auto env_y = [&](const float2* Rin, const Site& t, float2* Y) {
    float2 y0 = mk(0.f, 0.f), y1 = y0;
    if (x < t.Dl && y < t.Dr) {
      for (int bp = 0; bp < t.Dr; ++bp) {
        const float2 r = Rin[y * DM + bp];
        y0 = cadd(y0, cmul(A0[x * DM + bp], r));
        y1 = cadd(y1, cmul(A1[x * DM + bp], r));
      }
    }
    Y[tid] = y0;
    Y[NT + tid] = y1;
  };
  // out[a][a'] = sum_{s, b} zs conj(A[a,s,b]) Y[a'][s][b]     (thread (a, a'))
  auto env_fin = [&](const float2* Y, const Site& t, float zsign1) {
    float2 o = mk(0.f, 0.f);
    if (x < t.Dl && y < t.Dl) {
      for (int b = 0; b < t.Dr; ++b) {
        o = cadd(o, cjmul(A0[x * DM + b], Y[y * DM + b]));
        o = cadd(o, csc(cjmul(A1[x * DM + b], Y[NT + y * DM + b]), zsign1));
      }
    }
    return o;
  };

  // ---------------- right sweep: R_{q+1} for every qubit (stored)
  float2* R = E1;
  R[tid] = tid == 0 ? mk(1.f, 0.f) : mk(0.f, 0.f);
  __syncthreads();
  for (int q = n - 1; q >= 0; --q) {
    const Site t = site_of(g, q);
    rp[(size_t)q * NT + tid] = R[tid];
    put_col(t);
    __syncthreads();
    env_y(R, t, U1[0]);
    __syncthreads();
    const float2 o = env_fin(U1[0], t, 1.f);
    __syncthreads();
    R[tid] = o;
    __syncthreads();
  }
  // <psi|psi> = R_0 (exactly 1 up to rounding): readout and gradients are divided by it, as the torch MPS does
  const float inv_norm = 1.f / R[0].x;
  __syncthreads();

  float2* Lp = E1;
  float2* LO = E2;
  float2* Rq = E3;
  float2* ROq = E4;
  float2* ros = reinterpret_cast<float2*>(g.ro) + (size_t)s * (g.qmax + 1) * NT;
  // ---------------- RO sweep (gradient mode): RO_{q+1} for q <= qmax, from RO_{qmax+1} = 0
  if (grad) {
    ROq[tid] = mk(0.f, 0.f);
    __syncthreads();
    for (int q = g.qmax; q >= 0; --q) {
      const Site t = site_of(g, q);
      ros[(size_t)q * NT + tid] = ROq[tid];
      Rq[tid] = rp[(size_t)q * NT + tid];
      put_col(t);
      __syncthreads();
      env_y(ROq, t, U1[0]);
      env_y(Rq, t, U2[0]);
      __syncthreads();
      const float2 o1 = env_fin(U1[0], t, 1.f), o2 = env_fin(U2[0], t, -1.f);
      __syncthreads();
      ROq[tid] = cadd(o1, csc(o2, wof(q)));
      __syncthreads();
    }
  }

  // ---------------- left sweep: readout up to qmax, gradients over every qubit
  Lp[tid] = tid == 0 ? mk(1.f, 0.f) : mk(0.f, 0.f);
  LO[tid] = mk(0.f, 0.f);
  __syncthreads();
  const int qend = grad ? n : g.qmax + 1;
  for (int q = 0; q < qend; ++q) {
    const Site t = site_of(g, q);
    put_col(t);
    Rq[tid] = rp[(size_t)q * NT + tid];
    ROq[tid] = (grad && q <= g.qmax) ? ros[(size_t)q * NT + tid] : mk(0.f, 0.f);
    __syncthreads();
    // U1[a'][s][b] = sum_a conj(A[a,s,b]) Lp[a][a'],  U2 the same with LO      (thread (a', b))
    {
      float2 p0 = mk(0.f, 0.f), p1 = p0, o0 = p0, o1 = p0;
      if (x < t.Dl && y < t.Dr) {
        for (int a = 0; a < t.Dl; ++a) {
          const float2 l = Lp[a * DM + x], lo = LO[a * DM + x];
          const float2 a0 = A0[a * DM + y], a1 = A1[a * DM + y];
          p0 = cadd(p0, cjmul(a0, l));
          p1 = cadd(p1, cjmul(a1, l));
          o0 = cadd(o0, cjmul(a0, lo));
          o1 = cadd(o1, cjmul(a1, lo));
        }
      }
      U1[0][tid] = p0;
      U1[1][tid] = p1;
      U2[0][tid] = o0;
      U2[1][tid] = o1;
    }
    __syncthreads();
    const float wz = wof(q);
    bool isro = false;
#pragma unroll
    for (int i = 0; i < RMAX; ++i) isro |= rq[i] == q;
    if (isro) {   // <Z_q> = sum_{a',s,b,b'} z_s U1[a',s,b] A[a',s,b'] Rq[b][b']
      float tz = 0.f;
      if (x < t.Dl && y < t.Dr) {
        float2 y0 = mk(0.f, 0.f), y1 = y0;
        for (int bp = 0; bp < t.Dr; ++bp) {
          const float2 r = Rq[y * DM + bp];
          y0 = cadd(y0, cmul(A0[x * DM + bp], r));
          y1 = cadd(y1, cmul(A1[x * DM + bp], r));
        }
        tz = cmul(U1[0][tid], y0).x - cmul(U1[1][tid], y1).x;
      }
      tz = wave_sum(tz);
      if (lane == 0) {
#pragma unroll
        for (int i = 0; i < RMAX; ++i)
          if (rq[i] == q) red[wave][MAXPG + i] = tz;
      }
    }
    if (grad && t.npg > 0) {
      // Ybar[a'][s][b'] = sum_b U1[a',s,b] (RO[b][b'] + wz z_s Rq[b][b']) + U2[a',s,b] Rq[b][b']   (thread (a', b'))
      float2 u0 = mk(0.f, 0.f), u1 = u0;
      if (col_valid(t, x, y)) {
        for (int b = 0; b < t.Dr; ++b) {
          const float2 r = Rq[b * DM + y], ro = ROq[b * DM + y];
          const float2 k0 = cadd(ro, csc(r, wz)), k1 = cadd(ro, csc(r, -wz));
          u0 = cadd(u0, cadd(cmul(U1[0][x * DM + b], k0), cmul(U2[0][x * DM + b], r)));
          u1 = cadd(u1, cadd(cmul(U1[1][x * DM + b], k1), cmul(U2[1][x * DM + b], r)));
        }
      }
      // pull u back through the column's events; at each rotation G (input v, output r = G v):
      // d<O>/d angle += 2 Re(u . dG v), dG v = (-i/2) X r (RX), (-i/2) Y r (RY), (-i/2) Z r (RZ), (0, i r1) (P)
      int p = t.npg;
      for (int i = t.cnt - 1; i >= 0; --i) {
        const int e = t.ev[i];
        M2 m;
        if ((e & 3) == EV_GATE) {
          const int gi = e >> 8, kind = g.gkind[gi];
          m = gate_mat(kind, ang[gi]);
          if (rotation(kind)) {
            float2 v0, v1;
            build_col(t, ang, g.gkind, x, y, i, v0, v1);
            const float2 r0 = cadd(cmul(m.a, v0), cmul(m.b, v1)), r1 = cadd(cmul(m.c, v0), cmul(m.d, v1));
            float2 d0, d1;
            if (kind == K_RX) {
              d0 = mk(0.5f * r1.y, -0.5f * r1.x);
              d1 = mk(0.5f * r0.y, -0.5f * r0.x);
            } else if (kind == K_RY) {
              d0 = mk(-0.5f * r1.x, -0.5f * r1.y);
              d1 = mk(0.5f * r0.x, 0.5f * r0.y);
            } else if (kind == K_RZ) {
              d0 = mk(0.5f * r0.y, -0.5f * r0.x);
              d1 = mk(-0.5f * r1.y, 0.5f * r1.x);
            } else {
              d0 = mk(0.f, 0.f);
              d1 = mk(-r1.y, r1.x);
            }
            const float c = 2.f * (cmul(u0, d0).x + cmul(u1, d1).x);
            const float sum = wave_sum(c);
            --p;
            if (lane == 0) red[wave][p] = sum;
            if (tid == 0) pg_s[p] = gi;
          }
        }
        apply_ev<true>(e, &m, x, y, u0, u1);
      }
    }
    // Lp_{q+1}[b][b'] = sum_{a',s} U1[a',s,b] A[a',s,b'];  LO_{q+1} = sum (U2 + wz z_s U1) A      (thread (b, b'))
    float2 nl = mk(0.f, 0.f), no = nl;
    if (x < t.Dr && y < t.Dr) {
      for (int ap = 0; ap < t.Dl; ++ap) {
        const float2 a0 = A0[ap * DM + y], a1 = A1[ap * DM + y];
        const float2 p0 = U1[0][ap * DM + x], p1 = U1[1][ap * DM + x];
        nl = cadd(nl, cadd(cmul(p0, a0), cmul(p1, a1)));
        if (grad) {
          const float2 o0 = cadd(U2[0][ap * DM + x], csc(p0, wz)), o1 = cadd(U2[1][ap * DM + x], csc(p1, -wz));
          no = cadd(no, cadd(cmul(o0, a0), cmul(o1, a1)));
        }
      }
    }
    __syncthreads();
    Lp[tid] = nl;
    LO[tid] = no;
    if (grad && tid < t.npg) {                   // the site's rotations, summed over the four waves in order
      float v = 0.f;
#pragma unroll
      for (int w_ = 0; w_ < NW; ++w_) v += red[w_][tid];
      g.dang[(size_t)s * g.G + pg_s[tid]] = v * inv_norm;
    }
    __syncthreads();
  }
  if (tid < g.C) {
    float v = 0.f;
#pragma unroll
    for (int w_ = 0; w_ < NW; ++w_) v += red[w_][MAXPG + tid];
    g.z[(size_t)s * g.C + tid] = v * inv_norm;
  }
}

}  // namespace qfx_mpo

extern "C" int qfx_mps_mpo(const QfxMpoArgs* args, hipStream_t st) {
  const QfxMpoArgs& g = *args;
  if (g.n < 2 || g.C < 1 || g.C > QFX_MPS_RMAX || g.qmax >= g.n || g.G < 1) return -2;
  if (g.S == 0) return 0;
  hipLaunchKernelGGL(qfx_mpo::mps_mpo_kernel, dim3((unsigned)g.S), dim3(qfx_mpo::NT), 0, st, g);
  return (int)hipGetLastError();
}
