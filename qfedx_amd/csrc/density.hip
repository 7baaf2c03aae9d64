// Exact density-matrix simulation of small noisy circuits (ROADMAP.md:64-73: depolarizing p, amplitude damping
// gamma as their exact Kraus channels; the statevector engines only realise Pauli channels, as trajectories).
//
// rho (2^n x 2^n, complex64) is a vector over 2n index bits: bit q of a row index is bit q, bit q of a column
// index is bit q + n (i = r + c 2^n).  A one-qubit gate U on qubit q followed by the gate-noise channel {K_i}
// on q is ONE 4 x 4 superoperator on the bit pair (q, q + n):
//     T = S (U (x) U*),   S[(a, b)][(a', b')] = sum_i K_i[a][a'] conj(K_i[b][b'])   (quad element a + 2 b)
// applied to every quad of rho in one pass.  Two-qubit gates (cx, cz, swap) are permutations / signs of rows and
// columns (in-place pair swaps), followed by S on each qubit they touch.  <Z_c> = sum_r rho_rr (1 - 2 r_c).
// The channel is trace preserving, so nothing renormalises.
//
// One workgroup runs one circuit instance (one sample row of slot values) through the whole program: rho lives
// in LDS up to n = 6 (32 KB) and in a global scratch slab beyond (n <= 10; 512 KB at n = 8 stays in the XCD's
// L2).  Passes are separated by workgroup barriers (the L1 is shared by a workgroup's waves, so a workgroup-scope
// fence orders the global slab too).  ops/density.py lowers the program; quantum/noise.py is the float64 oracle.
#include <hip/hip_runtime.h>

#include <cstdint>

namespace dm {

constexpr int NT = 256;
constexpr int LDS_QUBITS = 6;
constexpr int MAXQ = 10;
constexpr int CMAX = 16;

enum { K_RX = 0, K_RY = 1, K_RZ = 2, K_P = 3, K_CX = 13, K_CZ = 14, K_SWAP = 15 };

struct Gate {          // one lowered gate (ops/density.py)
  int kind, q0, q1, slot;
  float scale, off;
  float m[8];          // fixed one-qubit matrix (re, im) x 4, row-major; unused for rx / ry / rz / p
};

struct Args {
  const Gate* gates;
  int G, n;
  const float* rows;   // [S][W] slot values (theta | x)
  int W;
  const int* readout;
  int C;
  const float* S;      // [32] noise superoperator (re, im) x 16, row-major over quad index a + 2 b; null = none
  float2* scratch;     // [S][4^n] when n > LDS_QUBITS
  float* expz;         // [S][C]
};

__device__ __forceinline__ float2 cmul(float2 a, float2 b) {
  return make_float2(a.x * b.x - a.y * b.y, a.x * b.y + a.y * b.x);
}
__device__ __forceinline__ float2 cadd(float2 a, float2 b) { return make_float2(a.x + b.x, a.y + b.y); }
__device__ __forceinline__ float2 conj2(float2 a) { return make_float2(a.x, -a.y); }

// the gate's 2 x 2 matrix (Qiskit conventions, quantum/circuit.py gate_matrix)
__device__ void gate_matrix(const Gate& g, const float* row, float2 u[4]) {
  if (g.kind <= K_P) {
    const float ang = g.scale * (g.slot >= 0 ? row[g.slot] : 0.f) + g.off;
    float s, c;
    sincosf(0.5f * ang, &s, &c);
    if (g.kind == K_RX) {
      u[0] = make_float2(c, 0.f); u[1] = make_float2(0.f, -s); u[2] = make_float2(0.f, -s); u[3] = make_float2(c, 0.f);
    } else if (g.kind == K_RY) {
      u[0] = make_float2(c, 0.f); u[1] = make_float2(-s, 0.f); u[2] = make_float2(s, 0.f); u[3] = make_float2(c, 0.f);
    } else if (g.kind == K_RZ) {
      u[0] = make_float2(c, -s); u[1] = make_float2(0.f, 0.f); u[2] = make_float2(0.f, 0.f); u[3] = make_float2(c, s);
    } else {                                   // p(phi) = diag(1, e^{i phi})
      float sp, cp;
      sincosf(ang, &sp, &cp);
      u[0] = make_float2(1.f, 0.f); u[1] = make_float2(0.f, 0.f); u[2] = make_float2(0.f, 0.f); u[3] = make_float2(cp, sp);
    }
    return;
  }
  for (int e = 0; e < 4; ++e) u[e] = make_float2(g.m[2 * e], g.m[2 * e + 1]);
}

// T = S (U (x) U*) into LDS (16 entries, threads 0..15); U = identity gives T = S
__device__ void build_superop(const float2 u[4], const float* S, float2* T) {
  const int t = threadIdx.x;
  if (t < 16) {
    const int r = t >> 2, c = t & 3;
    float2 acc = make_float2(0.f, 0.f);
    for (int m = 0; m < 4; ++m) {
      // (U (x) U*)[m][c] with m = a + 2 b, c = a' + 2 b': U[a][a'] conj(U[b][b'])
      const float2 uu = cmul(u[(m & 1) * 2 + (c & 1)], conj2(u[(m >> 1) * 2 + (c >> 1)]));
      const float2 s = S ? make_float2(S[2 * (r * 4 + m)], S[2 * (r * 4 + m) + 1])
                         : make_float2(r == m ? 1.f : 0.f, 0.f);
      acc = cadd(acc, cmul(s, uu));
    }
    T[t] = acc;
  }
}

// rho <- T on every quad of bits (q, q + n)
__device__ void apply_superop(float2* rho, int n, int q, const float2* T) {
  const int nb = 2 * n;
  const long nq = 1L << (nb - 2);
  const long lo_a = (1L << q) - 1, lo_b = (1L << (q + n)) - 1;   // insert zero bits at q, then at q + n
  float2 t[16];
#pragma unroll
  for (int e = 0; e < 16; ++e) t[e] = T[e];
  for (long j = threadIdx.x; j < nq; j += NT) {
    long x = ((j & ~lo_a) << 1) | (j & lo_a);                       // bit q = 0
    x = ((x & ~lo_b) << 1) | (x & lo_b);                            // bit q + n = 0
    const long i0 = x, i1 = x | (1L << q), i2 = x | (1L << (q + n)), i3 = i1 | (1L << (q + n));
    const float2 v0 = rho[i0], v1 = rho[i1], v2 = rho[i2], v3 = rho[i3];
    float2 o[4];
#pragma unroll
    for (int r = 0; r < 4; ++r)
      o[r] = cadd(cadd(cmul(t[4 * r], v0), cmul(t[4 * r + 1], v1)), cadd(cmul(t[4 * r + 2], v2), cmul(t[4 * r + 3], v3)));
    rho[i0] = o[0];
    rho[i1] = o[1];
    rho[i2] = o[2];
    rho[i3] = o[3];
  }
}

// conditional pair swaps on one side (off = 0 rows, n columns): for cx(q0 -> q1) swap bit q1 where q0 is set;
// for swap(q0, q1) exchange entries whose two bits differ
__device__ void permute_side(float2* rho, int n, int kind, int q0, int q1, int off) {
  const long N = 1L << (2 * n);
  const long m0 = 1L << (q0 + off), m1 = 1L << (q1 + off);
  for (long i = threadIdx.x; i < N; i += NT) {
    long j;
    if (kind == K_CX) {
      if (!(i & m0) || (i & m1)) continue;
      j = i | m1;
    } else {                                   // swap: (q0 = 1, q1 = 0) <-> (q0 = 0, q1 = 1)
      if (!(i & m0) || (i & m1)) continue;
      j = (i & ~m0) | m1;
    }
    const float2 a = rho[i], b = rho[j];
    rho[i] = b;
    rho[j] = a;
  }
}

__device__ void apply_cz(float2* rho, int n, int q0, int q1) {
  const long N = 1L << (2 * n);
  for (long i = threadIdx.x; i < N; i += NT) {
    const int zr = ((i >> q0) & (i >> q1) & 1), zc = ((i >> (q0 + n)) & (i >> (q1 + n)) & 1);
    if (zr ^ zc) rho[i] = make_float2(-rho[i].x, -rho[i].y);
  }
}

__global__ void __launch_bounds__(NT) dm_kernel(Args a) {
  __shared__ float2 rho_s[1 << (2 * LDS_QUBITS)];
  __shared__ float2 T[16];
  __shared__ float red[NT / 64][CMAX];
  const int s = blockIdx.x, n = a.n;
  const long N = 1L << (2 * n);
  float2* rho = n <= LDS_QUBITS ? rho_s : a.scratch + (size_t)s * N;
  const float* row = a.rows + (size_t)s * a.W;
  for (long i = threadIdx.x; i < N; i += NT) rho[i] = make_float2(i == 0 ? 1.f : 0.f, 0.f);
  __syncthreads();
  for (int gi = 0; gi < a.G; ++gi) {
    const Gate g = a.gates[gi];
    if (g.kind == K_CX || g.kind == K_CZ || g.kind == K_SWAP) {
      if (g.kind == K_CZ) {
        apply_cz(rho, n, g.q0, g.q1);
      } else {
        permute_side(rho, n, g.kind, g.q0, g.q1, 0);
        __syncthreads();
        permute_side(rho, n, g.kind, g.q0, g.q1, n);
      }
      if (a.S) {                               // the channel on both qubits
        const float2 id[4] = {make_float2(1.f, 0.f), make_float2(0.f, 0.f), make_float2(0.f, 0.f), make_float2(1.f, 0.f)};
        __syncthreads();
        build_superop(id, a.S, T);
        __syncthreads();
        apply_superop(rho, n, g.q0, T);
        __syncthreads();
        apply_superop(rho, n, g.q1, T);
      }
    } else {
      float2 u[4];
      gate_matrix(g, row, u);
      build_superop(u, a.S, T);
      __syncthreads();
      apply_superop(rho, n, g.q0, T);
    }
    __syncthreads();
  }
  // <Z_c> from the diagonal, fixed-order block reduction
  const long D = 1L << n;
  float acc[CMAX];
  for (int c = 0; c < a.C; ++c) acc[c] = 0.f;
  for (long r = threadIdx.x; r < D; r += NT) {
    const float p = rho[r + (r << n)].x;
    for (int c = 0; c < a.C; ++c) acc[c] += ((r >> a.readout[c]) & 1) ? -p : p;
  }
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  for (int c = 0; c < a.C; ++c) {
    float v = acc[c];
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    if (lane == 0) red[wave][c] = v;
  }
  __syncthreads();
  if (threadIdx.x < a.C) {
    float v = 0.f;
    for (int w = 0; w < NT / 64; ++w) v += red[w][threadIdx.x];
    a.expz[(size_t)s * a.C + threadIdx.x] = v;
  }
}

}  // namespace dm

extern "C" int qfx_dm_gate_bytes() { return (int)sizeof(dm::Gate); }

extern "C" int qfx_dm_run(const void* gates, int G, int n, const float* rows, int W, long S, const int* readout, int C,
                          const float* superop, void* scratch, float* expz, hipStream_t st) {
  if (n < 1 || n > dm::MAXQ || C < 1 || C > dm::CMAX || S <= 0) return (int)hipErrorInvalidValue;
  if (n > dm::LDS_QUBITS && !scratch) return (int)hipErrorInvalidValue;
  dm::Args a{(const dm::Gate*)gates, G, n, rows, W, readout, C, superop, (float2*)scratch, expz};
  hipLaunchKernelGGL(dm::dm_kernel, dim3((unsigned)S), dim3(dm::NT), 0, st, a);
  return (int)hipGetLastError();
}

extern "C" int qfx_dm_lds_qubits() { return dm::LDS_QUBITS; }
