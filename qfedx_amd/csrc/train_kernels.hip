// gfx950 kernels around the statevector passes: readout + cross-entropy (K14), adjoint gradient
// reduction, fused client-batched Adam / SGD-momentum (K6), and the fused FedAvg local reduce with
// angle wrap + DP clip + Philox Gaussian noise (K8 + K17 + K20).
//
// Reference equivalents: CrossEntropyLoss + optimizer.step in client_update
// (src/CFed/Classical_FL.py:53-62), federated_averaging (:66-81); ROADMAP.md:36-37 (delta + wrap),
// :50-51 (clip + Gaussian noise), :38 (Adam).
//
// All reductions are deterministic: fixed-order per-thread loops + LDS tree, no float atomics, so
// results do not depend on timing or on how clients are sharded across GPUs.
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>

#include "philox.h"
#include "qfx_adam.h"
#include "qfx_plan.h"
#include "qfx_readout.h"
#include "hea_frag.h"
#include "qfx_fedavg.h"

namespace qfx {

constexpr int CMAX = 8;

// readout noise model (K19): confusion probabilities + shot count + per-client Philox keys
struct ReadoutNoise {
  float p01, p10;            // P(read 1 | 0), P(read 0 | 1)
  int shots;                 // 0 = exact expectation
  const long long* keys;     // [K, 2] per-client Philox key words (shots > 0)
  unsigned stream;           // Philox stream (local step)
};

// deterministic block reduction of NV values per thread (blockDim = 256)
template <int NV>
__device__ __forceinline__ void block_sum(float (&v)[NV], float* sm) {
#pragma unroll
  for (int i = 0; i < NV; ++i) {
    float x = v[i];
    for (int o = 32; o > 0; o >>= 1) x += __shfl_xor(x, o, 64);
    v[i] = x;
  }
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  __syncthreads();
  if (lane == 0) {
#pragma unroll
    for (int i = 0; i < NV; ++i) sm[i * 4 + w] = v[i];
  }
  __syncthreads();
#pragma unroll
  for (int i = 0; i < NV; ++i) v[i] = sm[i * 4 + 0] + sm[i * 4 + 1] + sm[i * 4 + 2] + sm[i * 4 + 3];
}

// one block per client: <Z_c> = sum of tile partials; logits a<Z>+b; CE; dL/d<Z>; grads of a, b
__global__ void __launch_bounds__(256) qfx_readout_ce_kernel(
    const float* __restrict__ part, int tps, int C, int spc, const long long* __restrict__ y,
    const float* __restrict__ wts, const float* __restrict__ params, int p_stride, int n_theta,
    float* __restrict__ expz, float* __restrict__ w_out, float* __restrict__ loss,
    float* __restrict__ correct, float* __restrict__ grad, int write_grad, ReadoutNoise nz) {
  __shared__ float sm[(2 * CMAX + 2) * 4];
  const int k = blockIdx.x;
  const bool noisy = nz.p01 != 0.f || nz.p10 != 0.f || nz.shots > 0;
  const uint32_t k0 = nz.keys ? (uint32_t)nz.keys[2 * k] : 0u, k1 = nz.keys ? (uint32_t)nz.keys[2 * k + 1] : 0u;
  const float gscale = 1.f - nz.p01 - nz.p10;   // straight-through d<Z>_noisy / d<Z>
  const float* a = params + (size_t)k * p_stride + n_theta;
  const float* b = a + C;
  float acc[2 * CMAX + 2];
#pragma unroll
  for (int i = 0; i < 2 * CMAX + 2; ++i) acc[i] = 0.f;
  for (int j = threadIdx.x; j < spc; j += 256) {
    const long s = (long)k * spc + j;
    float z[CMAX], zs[CMAX];
    qfx_ro::tile_sums(part, s, tps, C, zs);
#pragma unroll
    for (int c = 0; c < CMAX; ++c) {
      float t = c < C ? zs[c] : 0.f;
      if (noisy && c < C) t = noisy_z(t, nz.p01, nz.p10, nz.shots, k0, k1, nz.stream, ((uint64_t)j * C + c) * (uint64_t)nz.shots);
      z[c] = t;
    }
    const int yy = (int)y[s];
    const float ws = wts[s];
    float dl[CMAX], lterm, hit;
    qfx_ro::ce_sample(z, a, b, C, yy, ws, dl, lterm, hit);
#pragma unroll
    for (int c = 0; c < CMAX; ++c) {
      if (c >= C) break;
      expz[(size_t)s * C + c] = z[c];
      w_out[(size_t)s * C + c] = dl[c] * a[c] * gscale;
      acc[c] += dl[c] * z[c];
      acc[CMAX + c] += dl[c];
    }
    acc[2 * CMAX] += lterm;
    acc[2 * CMAX + 1] += hit;
  }
  block_sum<2 * CMAX + 2>(acc, sm);
  if (threadIdx.x == 0) {
    loss[k] = acc[2 * CMAX];
    correct[k] = acc[2 * CMAX + 1];
    if (write_grad) {
      float* g = grad + (size_t)k * p_stride + n_theta;
      for (int c = 0; c < C; ++c) {
        g[c] = acc[c];
        g[C + c] = acc[CMAX + c];
      }
    }
  }
}

// readout noise on exact expectations expz [K * spc, C] in place (evaluation path)
__global__ void qfx_readout_noise_kernel(float* __restrict__ expz, int C, int spc, long n_samples, ReadoutNoise nz) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n_samples * C) return;
  const long s = i / C;
  const int c = (int)(i % C);
  const long k = s / spc, j = s - k * spc;
  const uint32_t k0 = nz.keys ? (uint32_t)nz.keys[2 * k] : 0u, k1 = nz.keys ? (uint32_t)nz.keys[2 * k + 1] : 0u;
  expz[i] = noisy_z(expz[i], nz.p01, nz.p10, nz.shots, k0, k1, nz.stream, ((uint64_t)j * C + c) * (uint64_t)nz.shots);
}

// Philox uniforms (0,1]: out[k][e] for e < n from key keys[k] and the given stream (noise trajectories)
__global__ void qfx_philox_uniform_kernel(const long long* __restrict__ keys, long n, unsigned stream,
                                          float* __restrict__ out) {
  const int k = blockIdx.y;
  const long e = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= n) return;
  out[(size_t)k * n + e] = philox_uniform_at((uint64_t)e, (uint32_t)keys[2 * k], (uint32_t)keys[2 * k + 1], stream);
}

// sum of tile partials only (evaluation): expz[s][c]
__global__ void qfx_readout_sum_kernel(const float* __restrict__ part, int tps, int C, long n_samples,
                                       float* __restrict__ expz) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n_samples * C) return;
  const long s = i / C;
  const int c = (int)(i % C);
  const float* base = part + (size_t)s * tps * C + c;
  float t = 0.f;
  for (int u0 = 0; u0 < tps; u0 += 8) {   // 8 loads in flight, summed in tile order
    float v[8];
#pragma unroll
    for (int du = 0; du < 8; ++du) v[du] = u0 + du < tps ? base[(size_t)(u0 + du) * C] : 0.f;
#pragma unroll
    for (int du = 0; du < 8; ++du) t += v[du];
  }
  expz[i] = t;
}

// gradient reduction, stage 1: gpart[k][rs][g] = sum of slab rows of client k in row-split rs, for 64
// gates per block (threads: 64 gates x 4 row lanes, coalesced over gates), fixed-order LDS combine
constexpr int GR_SPLIT_MAX = 16;
__global__ void __launch_bounds__(256) qfx_grad_partial_kernel(const float* __restrict__ slab, long rows, int G,
                                                               int RS, float* __restrict__ gpart) {
  __shared__ float sm[256];
  const int k = blockIdx.x, rs = blockIdx.z;
  const int gl = threadIdx.x & 63, rl = threadIdx.x >> 6;
  const int g = blockIdx.y * 64 + gl;
  const long chunk = (rows + RS - 1) / RS;
  const long r0 = (long)rs * chunk, r1 = min(rows, r0 + chunk);
  float acc = 0.f;
  if (g < G) {   // rows r0+rl, +4, +8, ...: four loads in flight per iteration, summed in row order
    const float* base = slab + (size_t)k * rows * G + g;
    for (long r = r0 + rl; r < r1; r += 16) {
      const float v0 = base[(size_t)r * G];
      const float v1 = r + 4 < r1 ? base[(size_t)(r + 4) * G] : 0.f;
      const float v2 = r + 8 < r1 ? base[(size_t)(r + 8) * G] : 0.f;
      const float v3 = r + 12 < r1 ? base[(size_t)(r + 12) * G] : 0.f;
      acc += v0;
      acc += v1;
      acc += v2;
      acc += v3;
    }
  }
  sm[threadIdx.x] = acc;
  __syncthreads();
  if (rl == 0 && g < G) gpart[((size_t)k * RS + rs) * G + g] = sm[gl] + sm[64 + gl] + sm[128 + gl] + sm[192 + gl];
}

// stage 2, one block per client: gsum[g] = sum_rs gpart (fixed order) for gradient gates, then
// grad[k][slot] = sum_{gates g of slot} scale_g * gsum[g] in gate order, walking the host-built slot -> gate
// CSR (csr[0..n_theta] offsets, then gate ids) so each slot touches only its own gates.
__global__ void __launch_bounds__(256) qfx_grad_slots_kernel(const float* __restrict__ gpart, int RS,
                                                             const int* __restrict__ blob,
                                                             const int* __restrict__ csr, float* __restrict__ grad,
                                                             int p_stride) {
  extern __shared__ float gsh[];
  const int k = blockIdx.x;
  const int G = blob[HF_NGATES];
  const int n_theta = blob[HF_NTHETA];
  const int* gt = blob + blob[HF_GATES];
  float* gsum = gsh;
  float* gscale = gsh + G;
  for (int g = threadIdx.x; g < G; g += 256) {
    const int kind = gt[g * GATE_WORDS];
    const int slot = gt[g * GATE_WORDS + 3];
    const bool use = slot >= 0 && slot < n_theta && kind <= K_P;
    float v[GR_SPLIT_MAX];
#pragma unroll
    for (int r = 0; r < GR_SPLIT_MAX; ++r) v[r] = (use && r < RS) ? gpart[((size_t)k * RS + r) * G + g] : 0.f;
    float s = 0.f;
#pragma unroll
    for (int r = 0; r < GR_SPLIT_MAX; ++r) s += v[r];
    gsum[g] = s;
    gscale[g] = __int_as_float(gt[g * GATE_WORDS + 4]);
  }
  __syncthreads();
  for (int slot = threadIdx.x; slot < n_theta; slot += 256) {
    float s = 0.f;
    const int e1 = csr[slot + 1];
    for (int e = csr[slot]; e < e1; ++e) {
      const int g = csr[n_theta + 1 + e];
      s = fmaf(gscale[g], gsum[g], s);
    }
    grad[(size_t)k * p_stride + slot] = s;
  }
}

// fused client-batched Adam: rows with active[k]==0 untouched
// The per-client step counter ping-pongs between two buffers (t_in read by the whole row, t_out = t_in +
// active written by the row's first element), so no separate counter launch is needed.
__global__ void qfx_adam_kernel(float* __restrict__ p, const float* __restrict__ g, float* __restrict__ m,
                                float* __restrict__ v, const float* __restrict__ t_in, float* __restrict__ t_out,
                                const float* __restrict__ active, int K, int P, float lr, float b1, float b2,
                                float eps) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (long)K * P) return;
  const int k = (int)(i / P);
  qfx_adam_elem(p, g[i], m, v, t_in, t_out, active, k, i, i == (long)k * P, lr, b1, b2, eps);
}

// torch.optim.SGD(momentum) semantics: buf = g on the first step, else mu*buf + g; p -= lr*buf
// grid (chunks of SG_E parameters, clients): no per-element client division; SG_U elements per thread in flight
constexpr int SG_U = 4, SG_E = 256 * SG_U;
__global__ void __launch_bounds__(256) qfx_sgdm_kernel(float* __restrict__ p, const float* __restrict__ g,
                                                       float* __restrict__ buf, const float* __restrict__ t_in,
                                                       float* __restrict__ t_out, const float* __restrict__ active,
                                                       int K, int P, float lr, float mu, int keep) {
  const int k = blockIdx.y;
  const float act = active[k];
  if (blockIdx.x == 0 && threadIdx.x == 0) t_out[k] = t_in[k] + act;
  if (act == 0.f) return;
  const bool first = t_in[k] == 0.f;   // torch SGD: the buffer is the gradient on the first step (never read)
  const size_t row = (size_t)k * P;
  const int e0 = blockIdx.x * SG_E + threadIdx.x;
  float gv[SG_U], bv[SG_U];
#pragma unroll
  for (int u = 0; u < SG_U; ++u) {
    const int e = e0 + u * 256;
    if (e < P) {
      gv[u] = g[row + e];
      bv[u] = first ? 0.f : buf[row + e];
    }
  }
#pragma unroll
  for (int u = 0; u < SG_U; ++u) {
    const int e = e0 + u * 256;
    if (e < P) {
      const float b = first ? gv[u] : fmaf(mu, bv[u], gv[u]);
      if (keep) buf[row + e] = b;
      p[row + e] -= lr * b;
    }
  }
}

// per-client l2 norm of the (wrapped) update for DP clipping: stage 1, grid (client, chunk of
// NORM_CHUNK params) -> partial sums of squares in double (fixed-order wave + LDS combine)
constexpr int NORM_CHUNK = 8192;
__global__ void __launch_bounds__(256) qfx_delta_norm_partial_kernel(
    const float* __restrict__ theta_k, const float* __restrict__ theta_g,
    const unsigned char* __restrict__ angle_mask, int P, int wrap, double* __restrict__ partial) {
  __shared__ double sm[4];
  const int k = blockIdx.x, c = blockIdx.y;
  const int e0 = c * NORM_CHUNK, e1 = min(P, e0 + NORM_CHUNK);
  double acc = 0.0;
  for (int e = e0 + threadIdx.x; e < e1; e += 256) {
    double d = (double)theta_k[(size_t)k * P + e] - (double)theta_g[e];
    if (wrap && angle_mask[e]) d = wrap_pi(d);
    acc += d * d;
  }
  for (int o = 32; o > 0; o >>= 1) acc += __shfl_xor(acc, o, 64);
  if ((threadIdx.x & 63) == 0) sm[threadIdx.x >> 6] = acc;
  __syncthreads();
  if (threadIdx.x == 0) partial[(size_t)k * gridDim.y + c] = sm[0] + sm[1] + sm[2] + sm[3];
}

// stage 2: norms[k] = sqrt(sum_c partial[k][c]) in chunk order
__global__ void qfx_delta_norm_final_kernel(const double* __restrict__ partial, int nc, int K, double* __restrict__ norms) {
  const int k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= K) return;
  double s = 0.0;
  for (int c = 0; c < nc; ++c) s += partial[(size_t)k * nc + c];
  norms[k] = sqrt(s);
}

// out[e] = sum_k round(2^32 * w_k * priv(wrap(theta_k[e] - theta_g[e]))), out[P] = sum_k round(2^32 w_k)
// Each client's term is rounded to fixed point BEFORE the sum: integer addition is associative, so the
// aggregate is bitwise identical for any sharding of clients over GPUs (and equal to the CPU path).
constexpr int FA_E = 64, FA_G = 16;  // fedavg reduce: parameters per block (one wave row) x client groups per block
// (16 groups: a 64-client round has every client row in flight at once; 4 left the launch latency-bound)
constexpr int FA_U = 4;              // client rows in flight per thread

// Pairwise-mask secure aggregation inside the reduce (privacy/secure_agg.py is the host protocol and
// oracle).  Client row k's masked term of element e (e < P: weighted update, e == P: the weight) in Z_2^bits:
//   encode(x) = round(x * scale) mod 2^bits,  + sum_j sign[k][j] * PRG(seed[k][j], round)[e]  mod 2^bits
// with PRG = Philox4x32-10 keyed by the 64-bit pair seed, counter (e / 2, 0, round, 0x5EC), element e the 48-bit
// value of words 2 (e & 1), 2 (e & 1) + 1 (prg_mask's exact layout).  sign is +1 toward peers j > k, -1 toward
// j < k, 0 for non-participants, the client itself and padding rows; the orphan-mask correction of a dropped peer
// d (the survivor reveals seed[k][d], the server removes that mask) cancels the survivor's mask toward d exactly
// mod 2^bits, so the host folds it into sign[k][d] = 0.  Sums run in wrapping int64 (2^bits divides 2^64); the
// decode (round_apply) reduces mod 2^bits.
struct SecAgg {
  const uint32_t* seeds;     // [K][N][2] pair-seed key words (lo, hi); nullptr = plain exact aggregation
  const int* sign;           // [K][N]
  const int* round;          // [1] (a device word: the reduce is captured in the round graph)
  int N;
  double scale;
  long long mask;            // 2^bits - 1
  long long* masks;          // [K][P + 1] each client's total pair mask per element (qfx_secagg_mask_kernel)
  int epb;                   // mask elements per Philox block: 2 (bits > 32, two words each) or 4 (bits <= 32)
};

// Every client's total pair mask, one thread per (client, Philox block): one block per peer yields the values of
// elements epb b .. epb b + epb - 1 in prg_mask's layout (bits > 32: two words per element, 2 elements; bits <= 32:
// one word per element, 4 elements), so the K x N x (P + 1) / epb generator calls - the work each client would do on
// its own device - spread over the whole GPU.
__global__ void __launch_bounds__(256) qfx_secagg_mask_kernel(SecAgg sa, int P) {
  const int k = blockIdx.y;
  const long b = (long)blockIdx.x * 256 + threadIdx.x;      // Philox block
  const long e0 = (long)sa.epb * b;
  if (e0 > P) return;
  const uint32_t rnd = (uint32_t)sa.round[0];
  long long a[4] = {0, 0, 0, 0};
  for (int j = 0; j < sa.N; ++j) {
    const int sg = sa.sign[(size_t)k * sa.N + j];
    if (sg == 0) continue;
    const uint32_t* key = sa.seeds + ((size_t)k * sa.N + j) * 2;
    const u32x4 o = philox4x32_10({(uint32_t)b, (uint32_t)((uint64_t)b >> 32), rnd, 0x5ECu}, key[0], key[1]);
    long long m[4];
    if (sa.epb == 2) {
      m[0] = (long long)(((uint64_t)o.y << 32 | o.x) & (uint64_t)sa.mask);
      m[1] = (long long)(((uint64_t)o.w << 32 | o.z) & (uint64_t)sa.mask);
      m[2] = m[3] = 0;
    } else {
      m[0] = (long long)((uint64_t)o.x & (uint64_t)sa.mask);
      m[1] = (long long)((uint64_t)o.y & (uint64_t)sa.mask);
      m[2] = (long long)((uint64_t)o.z & (uint64_t)sa.mask);
      m[3] = (long long)((uint64_t)o.w & (uint64_t)sa.mask);
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) a[i] += sg > 0 ? m[i] : -m[i];
  }
  long long* row = sa.masks + (size_t)k * (P + 1);
  for (int i = 0; i < sa.epb; ++i)
    if (e0 + i <= P) row[e0 + i] = a[i];
}

// The same masks when the table is square (full graph, row k = client k, every client local: one rank): a pair's
// stream is the same Philox stream for both of its clients (one shared seed, opposite signs), so it is generated
// once and added to both rows - half the generator calls of the per-client kernel, bitwise the same integer sums.
// A workgroup (4 waves) owns SaPs<EPB>::NB consecutive Philox blocks; wave w owns blocks w + 4 t (t < NT) of every
// row.  Its lanes walk the pairs in round-robin order (circle method: the K/2 pairs of a round are disjoint), so
// within a wave no two lanes touch one accumulator and no other wave touches it at all: plain LDS adds, no atomics.
// Each (block, row) keeps a + and a - accumulator ([NB][2][EPB][K] int64, K x 512 bytes; rows innermost, so the
// lanes' distinct rows spread over the banks): a lane adds its mask words to the one its sign selects (one 64-bit
// add per word; the difference is taken at the end).  A lane's pair (rows, signs, key words - per lane, so the key
// schedule is VALU work here) serves NT generator calls, run as NT interleaved Philox chains (one round key per
// round for all of them: the ILP that 2 waves per SIMD need), with the next pair's table loads in flight and its
// LDS slots read before the generator runs (profiles/r6_secagg_pairsym_ab.txt: each of these steps measured).
template <int EPB> struct SaPs {
  static constexpr int NT = 8 / EPB;                   // generator calls per lane and pair
  static constexpr int NB = 4 * NT;                    // Philox blocks per workgroup
};
template <int NT>
__device__ __forceinline__ void philox_multi(u32x4 (&c)[NT], uint32_t k0, uint32_t k1) {
#pragma unroll
  for (int i = 0; i < 10; ++i) {
#pragma unroll
    for (int t = 0; t < NT; ++t) {
      uint32_t hi0, lo0, hi1, lo1;
      mulhilo32(0xD2511F53u, c[t].x, hi0, lo0);
      mulhilo32(0xCD9E8D57u, c[t].z, hi1, lo1);
      c[t] = {hi1 ^ c[t].y ^ k0, lo1, hi0 ^ c[t].w ^ k1, lo0};
    }
    k0 += 0x9E3779B9u;
    k1 += 0xBB67AE85u;
  }
}
template <int EPB>
__global__ void __launch_bounds__(256) qfx_secagg_pairsym_kernel(SecAgg sa, int K, int P) {
  constexpr int NT = SaPs<EPB>::NT, NB = SaPs<EPB>::NB;
  extern __shared__ long long sacc[];                  // [NB][2][EPB][K]
  const int tid = threadIdx.x, slot = tid & 63, bl = tid >> 6;
  const long base = (long)blockIdx.x * NB;             // first Philox block of the workgroup
  for (int e = tid; e < NB * K * 2 * EPB; e += 256) sacc[e] = 0;
  __syncthreads();
  const int Kp = K + (K & 1), R = Kp - 1, half = Kp >> 1;
  const int nq = (half + 63) >> 6, nit = R * nq;       // lane iterations: (round, pair slot + 64 q)
  const uint32_t rnd = (uint32_t)sa.round[0];
  int nlive = 0;                                       // this wave's blocks that hold elements <= P (a prefix)
#pragma unroll
  for (int t = 0; t < NT; ++t) nlive += (long)EPB * (base + bl + 4 * t) <= P;
  struct Pair { int k, j, sk, sj; uint32_t k0, k1; };
  auto fetch = [&](int it) {
    Pair q{0, 0, 0, 0, 0u, 0u};
    if (it >= nit) return q;
    const int r = it / nq, i = slot + 64 * (it - r * nq);
    if (i >= half) return q;
    int a = r, b = Kp - 1;                             // i == 0: the fixed player
    if (i > 0) {
      a = r + i;
      if (a >= R) a -= R;
      b = r - i;
      if (b < 0) b += R;
    }
    if (a >= K || b >= K) return q;                    // the odd-K bye
    q.k = min(a, b);
    q.j = max(a, b);
    q.sk = sa.sign[(size_t)q.k * sa.N + q.j];
    q.sj = sa.sign[(size_t)q.j * sa.N + q.k];
    const uint32_t* key = sa.seeds + ((size_t)q.k * sa.N + q.j) * 2;
    q.k0 = key[0];
    q.k1 = key[1];
    return q;
  };
  const uint64_t wm = (uint64_t)sa.mask;
  Pair nx = fetch(0);
  for (int it = 0; it < nit; ++it) {
    const Pair cu = nx;
    nx = fetch(it + 1);
    if ((cu.sk | cu.sj) == 0) continue;
    // accumulator slots: element index of (row, sign half) within a block's [2][EPB][K] plane.  Every slot this
    // lane updates is read before the generator runs (the LDS latency hides behind it) and written after, a zero
    // sign adding 0 (the slot is this lane's in this round either way)
    const int ok = (cu.sk < 0) * EPB * K + cu.k, oj = (cu.sj < 0) * EPB * K + cu.j;
    const uint64_t zk = cu.sk ? ~0ull : 0ull, zj = cu.sj ? ~0ull : 0ull;
    long long vk[NT][EPB], vj[NT][EPB];
#pragma unroll
    for (int t = 0; t < NT; ++t) {
      const long long* row = sacc + (size_t)(bl + 4 * t) * K * 2 * EPB;
#pragma unroll
      for (int e = 0; e < EPB; ++e) {
        vk[t][e] = row[ok + e * K];
        vj[t][e] = row[oj + e * K];
      }
    }
    u32x4 o[NT];
#pragma unroll
    for (int t = 0; t < NT; ++t) {
      const long blk = base + bl + 4 * t;
      o[t] = {(uint32_t)blk, (uint32_t)((uint64_t)blk >> 32), rnd, 0x5ECu};
    }
    philox_multi<NT>(o, cu.k0, cu.k1);
#pragma unroll
    for (int t = 0; t < NT; ++t) {
      if (t >= nlive) break;
      uint64_t m[EPB];
      if constexpr (EPB == 2) {
        m[0] = ((uint64_t)o[t].y << 32 | o[t].x) & wm;
        m[1] = ((uint64_t)o[t].w << 32 | o[t].z) & wm;
      } else {
        m[0] = o[t].x & wm;
        m[1] = o[t].y & wm;
        m[2] = o[t].z & wm;
        m[3] = o[t].w & wm;
      }
      long long* row = sacc + (size_t)(bl + 4 * t) * K * 2 * EPB;
#pragma unroll
      for (int e = 0; e < EPB; ++e) {
        row[ok + e * K] = vk[t][e] + (long long)(m[e] & zk);
        row[oj + e * K] = vj[t][e] + (long long)(m[e] & zj);
      }
    }
  }
  __syncthreads();
  for (int idx = tid; idx < K * NB * EPB; idx += 256) {   // row k: NB EPB consecutive elements
    const int k = idx / (NB * EPB), rest = idx % (NB * EPB);
    const long el = (long)EPB * base + rest;
    const long long* a = sacc + ((size_t)(rest / EPB) * 2 * EPB + rest % EPB) * K + k;
    if (el <= P) sa.masks[(size_t)k * (P + 1) + el] = a[0] - a[(size_t)EPB * K];
  }
}

__device__ __forceinline__ long long secagg_masks(const SecAgg& sa, int k, long e, int P) {
  return sa.masks[(size_t)k * (P + 1) + e];
}

template <bool PLAIN>
__device__ __forceinline__ long long fedavg_term(float x, double tg, bool wr, int k, long e, const double* weights,
                                                 const double* norms, const uint32_t* keys, const float* dps, int dp,
                                                 float clip, float sigma, int& nsat, const SecAgg& sa, int sa_P) {
  const double SC = 4294967296.0;
  double d = (double)x - tg;
  if (wr) d = wrap_pi(d);
  if constexpr (PLAIN) return fixed_term(weights[k] * d * SC, nsat);
  if (dp) {
    const double n = norms[k];
    const double sc = fmin(1.0, (double)clip / fmax(n, 1e-12));
    d = d * sc;
    // dps: per-client noise scale of the round (distributed DP: 1 / sqrt(live participants)), else 1
    if (sigma > 0.f)
      d += (double)sigma * (dps ? (double)dps[k] : 1.0) * (double)clip *
           (double)philox_normal_at((uint64_t)e, keys[2 * k], keys[2 * k + 1], 0u);
  }
  if (sa.seeds) {                      // SecAgg ring element: held to +-2^(bits - 1) before it wraps
    double v = weights[k] * d * sa.scale;
    const double lim = (double)(sa.mask >> 1);
    if (!(fabs(v) <= lim)) {
      ++nsat;
      v = v > 0.0 ? lim : (v < 0.0 ? -lim : 0.0);
    }
    return ((long long)llrint(v) & sa.mask) + secagg_masks(sa, k, e, sa_P);
  }
  return fixed_term(weights[k] * d * SC, nsat);
}

// A single-rank round has no collective between the reduce and the apply, so the reduce launch applies it too (one
// launch fewer per round): every parameter block knows the (exact, integer) weight sum - it is K loads - and applies
// its own entries right after forming them; the last arriving block reads out the metric / norm tail.  Under SecAgg
// the weight sum carries the masks, so only block 0 forms it and the last block applies every entry.
// theta == nullptr: not fused.
struct FusedApply {
  float* theta;
  double* out;
  unsigned* cnt;           // arrival counter, reset by the last block
  int bits, n_norms;
  double ring_scale, lr;
};

// Arrival of one block of a FusedApply launch; the last one applies entries [params_done ? P : 0, P + 6 + n_norms).
// ``release``: the block wrote what the last block reads (buffer entries, the metric pack, saturation counts) - its
// stores are in this XCD's L2 after the barrier and one agent-scope release publishes them before the arrival (the
// hea_grad_reduce Adam protocol).  A release is an L2 writeback on this chip, so blocks with nothing to publish (the
// parameter blocks that applied their own entries) skip it.  ``ws``: the weight sum when every block knows it.
__device__ __forceinline__ void fused_apply_tail(const FusedApply& fa, long long* buf, int P, bool params_done,
                                                 bool release, long long ws) {
  __shared__ int last_s;
  __syncthreads();
  if (threadIdx.x == 0) {
    if (release) __threadfence();
    const unsigned prev = atomicAdd(fa.cnt, 1u);
    last_s = prev == gridDim.x - 1;
    if (last_s) *fa.cnt = 0u;
  }
  __syncthreads();
  if (!last_s) return;
  // consumer side of the hand-off (every other block released its entries before its arrival): one agent-scope
  // acquire, drained, before any thread of the last block reads them (HIP / AMDGPU memory model)
  if (threadIdx.x == 0) {
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    __asm__ volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  __syncthreads();
  auto ld = [buf](long i) { return __hip_atomic_load(&buf[i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); };
  const double wsum = params_done ? (double)ws / 4294967296.0
                                  : (fa.bits ? ring_decode(ld(P), fa.bits, fa.ring_scale) : (double)ld(P) / 4294967296.0);
  for (long e = (params_done ? P : 0) + threadIdx.x; e < (long)P + 6 + fa.n_norms; e += blockDim.x)
    round_apply_elem(buf, P, fa.theta, fa.lr, fa.out, fa.bits, fa.ring_scale, fa.n_norms, e, wsum, ld);
}

// the weight sum (wave 0): lane-strided over the clients (one dependent global load per client made a serial loop
// the launch's long pole at 64 clients), then an integer wave sum - exact, so the split changes no bit.  Under
// SecAgg the weight is element P of each client's masked vector.
__device__ __forceinline__ long long weight_sum_wave(const double* __restrict__ weights, int K, int P,
                                                     const SecAgg& sa, int& wsat) {
  const double SC = 4294967296.0;
  long long ws = 0;
  wsat = 0;
  for (int k = threadIdx.x; k < K; k += 64) {
    if (sa.seeds) {
      const double v = weights[k] * sa.scale, lim = (double)(sa.mask >> 1);
      if (!(fabs(v) <= lim)) ++wsat;
      ws += ((long long)llrint(fmin(fmax(v, -lim), lim)) & sa.mask) + secagg_masks(sa, k, P, P);
      continue;
    }
    const double v = weights[k] * SC;
    if (!(fabs(v) <= FA_SAT)) ++wsat;
    ws += llrint(fmin(fmax(v, -FA_SAT), FA_SAT));
  }
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) {
    ws += __shfl_xor(ws, off, 64);
    wsat += __shfl_xor(wsat, off, 64);
  }
  return ws;
}

// PLAIN: no DP clip / noise and no SecAgg masks (the common round: the CFed and plain VQC reductions) - its own
// instantiation, since the general one's DP / SecAgg paths held it at 123 VGPRs, one 1024-thread block per CU
// (the CNN's 1,779 blocks then ran in seven rounds of latency-bound blocks: 34 us)
template <bool PLAIN>
__global__ void __launch_bounds__(FA_E * FA_G) qfx_fedavg_reduce_kernel(
    const float* __restrict__ theta_k, const float* theta_g,     // theta_g may be fa.theta (applied in place)
    const unsigned char* __restrict__ angle_mask, const double* __restrict__ weights,
    const double* __restrict__ norms, const uint32_t* __restrict__ keys, const float* __restrict__ dps, int K, int P,
    int wrap, int dp, float clip, float sigma, long long* __restrict__ out, RoundPack rp, long long* __restrict__ sat,
    SecAgg sa, FusedApply fa) {
  const bool own_apply = fa.theta && !sa.seeds;       // every parameter block applies its own entries (FusedApply)
  __shared__ long long ws_s;
  // the block past the parameter blocks (launched only with rp.buf) packs the round metrics into the tail of
  // the all-reduce buffer: the parameter blocks write out[0..P], the pack block out[P+1..P+4]
  if (blockIdx.x == gridDim.x - 1 && rp.buf != nullptr) {
    round_pack_block(rp, P);
    if (fa.theta) {
      if (own_apply && threadIdx.x < 64) {
        int wsat;
        const long long ws = weight_sum_wave(weights, K, P, sa, wsat);
        if (threadIdx.x == 0) ws_s = ws;
      }
      __syncthreads();
      fused_apply_tail(fa, rp.buf, P, own_apply, true, ws_s);
    }
    return;
  }
  // thread (group g, lane el): parameter e = block * FA_E + el (a wave reads 256 contiguous bytes of a client
  // row), clients k = g, g + FA_G, ... with FA_U rows loaded before their terms are formed; the FA_G integer
  // partials are combined in LDS (exact, so neither split changes a bit of the result)
  __shared__ long long part[FA_G][FA_E];
  const double SC = 4294967296.0;
  const int el = threadIdx.x % FA_E, grp = threadIdx.x / FA_E;
  const long e = (long)blockIdx.x * FA_E + el;
  int wsat = 0;
  if ((blockIdx.x == 0 || own_apply) && threadIdx.x < 64) {
    const long long ws = weight_sum_wave(weights, K, P, sa, wsat);
    if (threadIdx.x == 0) {
      ws_s = ws;
      if (blockIdx.x == 0) {
        out[P] = ws;
        if (wsat && sat) atomicAdd((unsigned long long*)sat, (unsigned long long)wsat);
      }
    }
    if (blockIdx.x != 0) wsat = 0;
  }
  long long acc = 0;
  int nsat = 0;
  if (e < P) {
    const double tg = (double)theta_g[e];
    const bool wr = wrap && angle_mask[e];
    int k = grp;
    for (; k + (FA_U - 1) * FA_G < K; k += FA_U * FA_G) {
      float x[FA_U];
#pragma unroll
      for (int u = 0; u < FA_U; ++u) x[u] = theta_k[(size_t)(k + u * FA_G) * P + e];
#pragma unroll
      for (int u = 0; u < FA_U; ++u)
        acc += fedavg_term<PLAIN>(x[u], tg, wr, k + u * FA_G, e, weights, norms, keys, dps, dp, clip, sigma, nsat, sa,
                                  P);
    }
    for (; k < K; k += FA_G)
      acc += fedavg_term<PLAIN>(theta_k[(size_t)k * P + e], tg, wr, k, e, weights, norms, keys, dps, dp, clip, sigma,
                                nsat, sa,
                         P);
  }
  // saturated terms are counted (an integer: the count is exact in any order); the host raises on a nonzero
  // count when it reads the round's metrics back (self-cleaning: round_apply zeroes it after the all-reduce)
  if (nsat && sat) atomicAdd((unsigned long long*)sat, (unsigned long long)nsat);
  part[grp][el] = acc;
  __syncthreads();
  if (grp == 0 && e < P) {
    long long v = 0;
    for (int j = 0; j < FA_G; ++j) v += part[j][el];
    out[e] = v;
    if (own_apply)        // ws_s was stored before the barrier above
      round_apply_elem(out, P, fa.theta, fa.lr, fa.out, 0, 1.0, 0, e, (double)ws_s / SC, [v](long) { return v; });
  }
  if (fa.theta) {
    // the last block reads this block's buffer entries only when it applies them (SecAgg); saturation counts it
    // always reads
    const bool counted = __syncthreads_or((nsat || wsat) ? 1 : 0);
    fused_apply_tail(fa, rp.buf, P, own_apply, !own_apply || counted, ws_s);
  }
}

// round epilogue 1 on its own (the HIP round path packs in the FedAvg launch's last block instead)
__global__ void __launch_bounds__(256) qfx_round_pack_kernel(RoundPack rp, int P) { round_pack_block(rp, P); }

// round epilogue 2 (after the all-reduce): round_apply_elem per entry
__global__ void qfx_round_apply_kernel(long long* __restrict__ buf, int P, float* __restrict__ theta, double lr,
                                       double* __restrict__ out, int bits, double ring_scale, int n_norms) {
  const long e = (long)blockIdx.x * blockDim.x + threadIdx.x;
  const double wsum = bits ? ring_decode(buf[P], bits, ring_scale) : (double)buf[P] / 4294967296.0;
  round_apply_elem(buf, P, theta, lr, out, bits, ring_scale, n_norms, e, wsum, [buf](long i) { return buf[i]; });
}

// Parameter-shift combine (ops/hea_mfma.py HeaMfmaProgram.param_shift): for client k and parameter j, the exact
// shifted expectations z+- = m +- f' (m = (f(theta) + f(theta + pi)) / 2, or 0 when only their difference counts),
// each confused / shot-sampled on the Philox stream of its (client, slot, sign) row exactly as the naive
// shifted-row path samples it (row key = client key mixed with row + 1), then dL/dtheta_j = 1/2 sum_(b, c)
// (z+ - z-) w[b][c].  One block per (j, k); per-thread partials and the block sum in fixed order (deterministic).
__global__ void __launch_bounds__(64) qfx_ps_combine_kernel(const float* __restrict__ f0, const float* __restrict__ fpi,
                                                            const float* __restrict__ jac, const float* __restrict__ w,
                                                            const long long* __restrict__ keys, float p01, float p10,
                                                            int shots, unsigned stream, int P, int B, int C,
                                                            int noisy, float* __restrict__ out) {
  const int j = blockIdx.x, k = blockIdx.y, tid = threadIdx.x;
  __shared__ double red[64];
  double acc = 0.0;
  for (int e = tid; e < 2 * B * C; e += 64) {
    const int sg = e / (B * C), bc = e - sg * B * C, b = bc / C, c = bc - b * C;
    const float jv = jac[(((size_t)k * B + b) * C + c) * P + j];
    const float m = fpi ? 0.5f * (f0[((size_t)k * B + b) * C + c] + fpi[(((size_t)k * P + j) * B + b) * C + c]) : 0.f;
    float z = sg ? m - jv : m + jv;
    if (noisy) {
      const uint32_t row = (uint32_t)(2 * j + sg) + 1u;
      const uint32_t k0 = keys ? ((uint32_t)keys[2 * k] ^ (row * 0x9E3779B9u)) : 0u;
      const uint32_t k1 = keys ? ((uint32_t)keys[2 * k + 1] + row * 0x85EBCA6Bu) : 0u;
      z = noisy_z(z, p01, p10, shots, k0, k1, stream, ((uint64_t)b * C + c) * (uint64_t)shots);
    }
    acc += (sg ? -0.5 : 0.5) * (double)z * (double)w[((size_t)k * B + b) * C + c];
  }
  red[tid] = acc;
  __syncthreads();
  for (int off = 32; off > 0; off >>= 1) {
    if (tid < off) red[tid] += red[tid + off];
    __syncthreads();
  }
  if (tid == 0) out[(size_t)k * P + j] = (float)red[0];
}

}  // namespace qfx

using namespace qfx;

extern "C" int qfx_launch_ps_combine(const float* f0, const float* fpi, const float* jac, const float* w,
                                     const long long* keys, float p01, float p10, int shots, unsigned stream, int K,
                                     int P, int B, int C, int noisy, float* out, hipStream_t st) {
  if (K <= 0 || P <= 0) return 0;
  hipLaunchKernelGGL(qfx_ps_combine_kernel, dim3((unsigned)P, (unsigned)K), dim3(64), 0, st, f0, fpi, jac, w, keys,
                     p01, p10, shots, stream, P, B, C, noisy, out);
  return (int)hipGetLastError();
}


extern "C" int qfx_fedavg_norm_scratch(int K, int P) { return K * (1 + (P + NORM_CHUNK - 1) / NORM_CHUNK); }

extern "C" int qfx_launch_round_pack(long long* buf, int P, const float* loss, const float* correct,
                                     const float* nvalid, const float* act, int n, hipStream_t st) {
  hipLaunchKernelGGL(qfx_round_pack_kernel, dim3(1), dim3(256), 0, st,
                     RoundPack{buf, loss, correct, nvalid, act, n, nullptr, nullptr, 0}, P);
  return (int)hipGetLastError();
}

extern "C" int qfx_launch_round_apply(long long* buf, int P, float* theta, double lr, double* out, int bits,
                                      double ring_scale, int n_norms, hipStream_t st) {
  if (bits < 0 || bits > 62 || n_norms < 0) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(qfx_round_apply_kernel, dim3((unsigned)((P + 6 + n_norms + 255) / 256)), dim3(256), 0, st, buf,
                     P, theta, lr, out, bits, ring_scale, n_norms);
  return (int)hipGetLastError();
}

extern "C" int qfx_launch_readout_ce(const float* part, int tps, int C, int spc, int K, const long long* y,
                                     const float* wts, const float* params, int p_stride, int n_theta,
                                     float* expz, float* w_out, float* loss, float* correct, float* grad,
                                     int write_grad, float p01, float p10, int shots, const long long* keys,
                                     unsigned stream, hipStream_t st) {
  if (C > CMAX) return -2;
  ReadoutNoise nz{p01, p10, shots, keys, stream};
  hipLaunchKernelGGL(qfx_readout_ce_kernel, dim3(K), dim3(256), 0, st, part, tps, C, spc, y, wts, params,
                     p_stride, n_theta, expz, w_out, loss, correct, grad, write_grad, nz);
  return (int)hipGetLastError();
}

extern "C" int qfx_launch_readout_noise(float* expz, int C, int spc, long n_samples, float p01, float p10,
                                        int shots, const long long* keys, unsigned stream, hipStream_t st) {
  const long tot = n_samples * C;
  if (tot <= 0) return 0;
  ReadoutNoise nz{p01, p10, shots, keys, stream};
  hipLaunchKernelGGL(qfx_readout_noise_kernel, dim3((unsigned)((tot + 255) / 256)), dim3(256), 0, st, expz, C, spc,
                     n_samples, nz);
  return (int)hipGetLastError();
}

extern "C" int qfx_launch_philox_uniform(const long long* keys, int K, long n, unsigned stream, float* out,
                                         hipStream_t st) {
  if (K <= 0 || n <= 0) return 0;
  hipLaunchKernelGGL(qfx_philox_uniform_kernel, dim3((unsigned)((n + 255) / 256), (unsigned)K), dim3(256), 0, st,
                     keys, n, stream, out);
  return (int)hipGetLastError();
}

extern "C" int qfx_launch_readout_sum(const float* part, int tps, int C, long n_samples, float* expz,
                                      hipStream_t st) {
  const long tot = n_samples * C;
  if (tot <= 0) return 0;
  hipLaunchKernelGGL(qfx_readout_sum_kernel, dim3((unsigned)((tot + 255) / 256)), dim3(256), 0, st, part,
                     tps, C, n_samples, expz);
  return (int)hipGetLastError();
}

// rows per client = spc * tps; the row split keeps >= ~64 rows per block and the grid >= a few hundred blocks
extern "C" int qfx_grad_split(int tps, int spc) {
  const long rows = (long)tps * spc;
  return (int)max(1L, min((long)GR_SPLIT_MAX, rows / 64));
}

extern "C" int qfx_launch_grad_reduce(const float* slab, int tps, int spc, int K, int G, const int* blob,
                                      const int* csr, float* grad, int p_stride, float* gpart, hipStream_t st) {
  const long rows = (long)tps * spc;
  const int RS = qfx_grad_split(tps, spc);
  if ((size_t)G * 8 > 64 * 1024) return -5;   // LDS gate sums + scales of the slot stage
  hipLaunchKernelGGL(qfx_grad_partial_kernel, dim3(K, (G + 63) / 64, RS), dim3(256), 0, st, slab, rows, G, RS, gpart);
  hipLaunchKernelGGL(qfx_grad_slots_kernel, dim3(K), dim3(256), (size_t)G * 8, st, gpart, RS, blob, csr, grad,
                     p_stride);
  return (int)hipGetLastError();
}

extern "C" int qfx_launch_adam(float* p, const float* g, float* m, float* v, const float* t_in, float* t_out,
                               const float* active, int K, int P, float lr, float b1, float b2, float eps,
                               hipStream_t st) {
  const long tot = (long)K * P;
  hipLaunchKernelGGL(qfx_adam_kernel, dim3((unsigned)((tot + 255) / 256)), dim3(256), 0, st, p, g, m, v, t_in,
                     t_out, active, K, P, lr, b1, b2, eps);
  return (int)hipGetLastError();
}

extern "C" int qfx_launch_sgdm(float* p, const float* g, float* buf, const float* t_in, float* t_out,
                               const float* active, int K, int P, float lr, float mu, int keep, hipStream_t st) {
  if (K <= 0 || P <= 0) return 0;
  hipLaunchKernelGGL(qfx_sgdm_kernel, dim3((unsigned)((P + SG_E - 1) / SG_E), (unsigned)K), dim3(256), 0, st, p, g, buf, t_in,
                     t_out, active, K, P, lr, mu, keep);
  return (int)hipGetLastError();
}

// ----------------------------------------------------------------------------------- round prologue
// local round start: every client row starts from the global params; optimizer moments / counters zeroed
// grid (chunks of SG_E parameters, clients): no per-element client modulo
struct RoundInit {
  const float* theta;
  int K, P;
  float *params, *m, *v, *t;   // params / m / v / t may be null (params: the first local step reads theta directly)
  int nt;
};

__device__ __forceinline__ void round_init_chunk(const RoundInit& ri, int k, int chunk) {
  const size_t row = (size_t)k * ri.P;
  const int e0 = chunk * SG_E + threadIdx.x;
#pragma unroll
  for (int u = 0; u < SG_U; ++u) {
    const int e = e0 + u * 256;
    if (e < ri.P) {
      if (ri.params) ri.params[row + e] = ri.theta[e];
      if (ri.m) ri.m[row + e] = 0.f;
      if (ri.v) ri.v[row + e] = 0.f;
    }
  }
  if (ri.t && chunk == 0 && k == 0)
    for (int i = threadIdx.x; i < ri.nt; i += 256) ri.t[i] = 0.f;
}

__global__ void __launch_bounds__(256) qfx_round_init_kernel(RoundInit ri) {
  round_init_chunk(ri, blockIdx.y, blockIdx.x);
}

extern "C" int qfx_launch_round_init(const float* theta, int K, int P, float* params, float* m, float* v, float* t,
                                     int nt, hipStream_t st) {
  if (K <= 0 || P <= 0) return 0;
  hipLaunchKernelGGL(qfx_round_init_kernel, dim3((unsigned)((P + SG_E - 1) / SG_E), (unsigned)K),
                     dim3(256), 0, st, RoundInit{theta, K, P, params, m, v, t, nt});
  return (int)hipGetLastError();
}

// ----------------------------------------------------------------------------------- host upload
// dst[0:n16) = src[0:n16) (16-byte words) where src is pinned host memory read by the kernel itself.  A kernel
// launch never waits on the stream, unlike a small hipMemcpyAsync issued behind a graph launch, which was seen
// to block the host until the queue drained (the GPU then idles while the host builds the next round).
//
// With a signal (ctr != nullptr) the kernel is also the captured round's completion signal for the pinned buffer
// it read: the last block to finish (arrival count in ctr[1], reset by that block for the next replay) bumps the
// round counter ctr[0] and publishes it to the coherent pinned word host_flag.  A block's loads from src have
// returned once its stores are issued, so the host may refill the buffer from then on; this replaces a separate
// one-thread signal node at the end of the round (one launch fewer per round).  The store is RELAXED at system
// scope: the host needs the count only, and a release would first write back the whole L2, dirty with the round's
// states.  (An event record between graph launches, the alternative, cost ~5 us of GPU idle each on this stack:
// scripts/graph_gap.py.)
__global__ void __launch_bounds__(256) qfx_host_upload_kernel(const uint4* __restrict__ src, uint4* __restrict__ dst,
                                                              long n16, long long* __restrict__ ctr,
                                                              long long* host_flag) {
  for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < n16; i += (long)gridDim.x * 256) dst[i] = src[i];
  if (!ctr) return;
  __syncthreads();
  if (threadIdx.x == 0) {
    const unsigned long long prev = atomicAdd((unsigned long long*)&ctr[1], 1ull);
    if (prev == (unsigned long long)gridDim.x - 1) {
      ctr[1] = 0;
      const long long c = ctr[0] + 1;
      ctr[0] = c;
      __hip_atomic_store(host_flag, c, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
  }
}

extern "C" int qfx_launch_host_upload(const void* host_src, void* dst, long nbytes, long long* ctr, long long* host_flag,
                                      hipStream_t st) {
  if (nbytes <= 0) return 0;
  if (nbytes % 16) return (int)hipErrorInvalidValue;
  void* dsrc = nullptr;
  hipError_t e = hipHostGetDevicePointer(&dsrc, const_cast<void*>(host_src), 0);
  if (e != hipSuccess) return (int)e;
  const long n16 = nbytes / 16;
  const long blocks = (n16 + 255) / 256;
  hipLaunchKernelGGL(qfx_host_upload_kernel, dim3((unsigned)(blocks < 1024 ? blocks : 1024)), dim3(256), 0, st,
                     (const uint4*)dsrc, (uint4*)dst, n16, ctr, host_flag);
  return (int)hipGetLastError();
}

// per-step minibatch gather + feature encoding, one block per sample row s = (step * K + k) * B + b:
//   x_out[s, 0:F] = enc(X[lid[k], idx[s], 0:F]),  y_out[s] = Y[lid[k], idx[s]]
// enc: 0 = alpha * x (ROADMAP RY(alpha x)), 1 = per-sample min-max -> pi * x^ (qAngle.py:36-41; constant
// rows -> 0), 2 = raw copy (amplitude encoding: normalised later by the state-load kernel)
struct BatchGather {
  const float* X;
  const long long *Y, *lid, *idx;
  int K, B;
  long nmax;
  int F, mode;
  float alpha;
  float* xo;
  int x_stride;
  long long* yo;
};

__device__ __forceinline__ void gather_row(const BatchGather& g, long s) {
  __shared__ float smn[4], smx[4];
  const long row = g.lid[(s / g.B) % g.K] * g.nmax + g.idx[s];
  const int F = g.F;
  const float* xr = g.X + row * F;
  float* out = g.xo + s * (long)g.x_stride;
  if (threadIdx.x == 0) g.yo[s] = g.Y[row];
  if (g.mode == 1) {
    float mn = INFINITY, mx = -INFINITY;
    for (int f = threadIdx.x; f < F; f += blockDim.x) {
      const float v = xr[f];
      mn = fminf(mn, v);
      mx = fmaxf(mx, v);
    }
    for (int o = 32; o > 0; o >>= 1) {
      mn = fminf(mn, __shfl_xor(mn, o, 64));
      mx = fmaxf(mx, __shfl_xor(mx, o, 64));
    }
    const int nw = blockDim.x >> 6;
    if ((threadIdx.x & 63) == 0) {
      smn[threadIdx.x >> 6] = mn;
      smx[threadIdx.x >> 6] = mx;
    }
    __syncthreads();
    mn = smn[0];
    mx = smx[0];
    for (int w = 1; w < nw; ++w) {
      mn = fminf(mn, smn[w]);
      mx = fmaxf(mx, smx[w]);
    }
    const float rng = mx - mn;
    const float pi_f = 3.14159265358979323846f;
    for (int f = threadIdx.x; f < F; f += blockDim.x) out[f] = rng > 0.f ? ((xr[f] - mn) / rng) * pi_f : 0.f;
  } else if (g.mode == 0) {
    for (int f = threadIdx.x; f < F; f += blockDim.x) out[f] = g.alpha * xr[f];
  } else if ((F & 3) == 0 && (g.x_stride & 3) == 0 && ((uintptr_t)g.X & 15) == 0 && ((uintptr_t)g.xo & 15) == 0) {
    // raw copy of 16-byte aligned rows (the CNN's 784-pixel images): one 16-byte load per lane
    const float4* src = (const float4*)xr;
    float4* dst = (float4*)out;
    for (int f = threadIdx.x; f < (F >> 2); f += blockDim.x) dst[f] = src[f];
  } else {
    for (int f = threadIdx.x; f < F; f += blockDim.x) out[f] = xr[f];
  }
}

__global__ void __launch_bounds__(256) qfx_batch_gather_kernel(BatchGather g) { gather_row(g, blockIdx.x); }

// Row s gathered and encoded by tps lanes (a power of two <= 64: an aligned lane group inside one wave; lane l of it),
// bitwise what gather_row computes (min / max are exact in any order).  The prologue packs 256 / tps rows into a block
// for short rows (the VQC's n-qubit features): one 256-thread block per 16-float row had made 2,048 gather blocks of a
// 64-client round.
__device__ __forceinline__ void gather_row_lanes(const BatchGather& g, long s, int l, int tps) {
  const long row = g.lid[(s / g.B) % g.K] * g.nmax + g.idx[s];
  const int F = g.F;
  const float* xr = g.X + row * F;
  float* out = g.xo + s * (long)g.x_stride;
  if (l == 0) g.yo[s] = g.Y[row];
  if (g.mode == 1) {
    float mn = INFINITY, mx = -INFINITY;
    for (int f = l; f < F; f += tps) {
      const float v = xr[f];
      mn = fminf(mn, v);
      mx = fmaxf(mx, v);
    }
    for (int o = tps >> 1; o > 0; o >>= 1) {
      mn = fminf(mn, __shfl_xor(mn, o, 64));
      mx = fmaxf(mx, __shfl_xor(mx, o, 64));
    }
    const float rng = mx - mn;
    const float pi_f = 3.14159265358979323846f;
    for (int f = l; f < F; f += tps) out[f] = rng > 0.f ? ((xr[f] - mn) / rng) * pi_f : 0.f;
  } else if (g.mode == 0) {
    for (int f = l; f < F; f += tps) out[f] = g.alpha * xr[f];
  } else {
    for (int f = l; f < F; f += tps) out[f] = xr[f];
  }
}

// Round prologue in ONE launch: blocks [0, K * chunks) initialise the client rows / optimizer state (as
// qfx_round_init_kernel), the rest gather and encode the minibatches of EVERY local step of the round (as
// qfx_batch_gather_kernel over steps * K * B rows).  Neither part reads what the other writes.
// The MFMA engine's fragments of the round's first local step (every client row starts as theta): one shared set,
// built from theta by n_slots extra blocks of the prologue launch (hea_frag.h) instead of a per-client frag launch.
struct FragJob {
  const int* slot_tab;    // [n_slots][9]
  int n_slots;            // 0: none
  uint4* frags;           // [n_slots][4][128]
  int bf16;
};

// The round's host upload folded into the prologue (otherwise the graph's first node, qfx_host_upload_kernel):
// ``blocks`` trailing blocks copy the pinned tables into the device pack for the later launches, the gather blocks
// read their slot and minibatch indices from the pinned copy itself (the launcher points BatchGather there), and the
// last block of the launch to finish is the round's completion signal for the pinned buffer (ctr / flag exactly as
// the upload kernel's).  Each gather block makes dependent host reads, so the trainer folds the upload only into
// small prologues (the 8-client share: 256 gather blocks, 9.7 -> 8.1 us and one launch fewer; at 64 clients, 2,048
// gather blocks, the merged launch took 35 us - profiles/r5_round_timelines_r5k.txt).
struct UploadJob {
  const uint4* src;        // device-mapped pinned buffer
  uint4* dst;
  long n16;
  long long* ctr;          // [round count, arrivals]
  long long* flag;         // coherent pinned word
  int blocks;              // 0: no upload in this launch
};

__device__ __forceinline__ void prologue_block(const RoundInit& ri, int chunks, const BatchGather& g, const FragJob& fj,
                                               long gather_blocks, long gather_rows, int tps, long long* zero,
                                               int nzero, long blk) {
  const int init_blocks = ri.K * chunks;
  if (blk < init_blocks) {
    round_init_chunk(ri, (int)(blk / chunks), (int)(blk % chunks));
    return;
  }
  const long b = blk - init_blocks;
  if (b < gather_blocks) {
    if (tps == 0) {
      gather_row(g, b);
    } else {
      const long s = b * (256 / tps) + threadIdx.x / tps;
      if (s < gather_rows) gather_row_lanes(g, s, threadIdx.x % tps, tps);
    }
    return;
  }
  if (b == gather_blocks + fj.n_slots) {   // the all-reduce buffer head the FedAvg tail (hea_grad_reduce) adds into
    for (int e = threadIdx.x; e < nzero; e += 256) zero[e] = 0;
    return;
  }
  const int slot = (int)(b - gather_blocks);
  uint4* out = fj.frags + (size_t)slot * 4 * 128;
  if (fj.bf16)
    hea_frag::build<__bf16>(ri.theta, fj.slot_tab + slot * 9, threadIdx.x, out);
  else
    hea_frag::build<_Float16>(ri.theta, fj.slot_tab + slot * 9, threadIdx.x, out);
}

__global__ void __launch_bounds__(256) qfx_round_prologue_kernel(RoundInit ri, int chunks, BatchGather g, FragJob fj,
                                                                 long gather_blocks, long gather_rows, int tps,
                                                                 long long* zero, int nzero, UploadJob up) {
  const long work = (long)gridDim.x - up.blocks;
  if ((long)blockIdx.x < work) {
    prologue_block(ri, chunks, g, fj, gather_blocks, gather_rows, tps, zero, nzero, blockIdx.x);
  } else {
    for (long i = ((long)blockIdx.x - work) * 256 + threadIdx.x; i < up.n16; i += (long)up.blocks * 256)
      up.dst[i] = up.src[i];
  }
  if (!up.ctr) return;
  // a block's pinned loads have returned once the stores they feed are issued (the copy, the gather rows)
  __syncthreads();
  if (threadIdx.x == 0) {
    const unsigned long long prev = atomicAdd((unsigned long long*)&up.ctr[1], 1ull);
    if (prev == (unsigned long long)gridDim.x - 1) {
      up.ctr[1] = 0;
      const long long c = up.ctr[0] + 1;
      up.ctr[0] = c;
      __hip_atomic_store(up.flag, c, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
  }
}

extern "C" int qfx_prologue_gather_lanes(int F);

extern "C" int qfx_launch_round_prologue(const float* theta, int K, int P, float* params, float* m, float* v, float* t,
                                         int nt, const float* X, const long long* Y, const long long* lid,
                                         const long long* idx, int steps, int B, long nmax, int F, int mode,
                                         float alpha, float* xo, int x_stride, long long* yo, const int* slot_tab,
                                         int n_slots, void* frags, int bf16, long long* zero, int nzero,
                                         const void* up_host, void* up_dst, long up_nbytes, long long* up_ctr,
                                         long long* up_flag, hipStream_t st) {
  if (K <= 0 || P <= 0) return 0;
  if (n_slots < 0 || (n_slots > 0 && (!slot_tab || !frags))) return (int)hipErrorInvalidValue;
  UploadJob up{nullptr, nullptr, 0, nullptr, nullptr, 0};
  if (up_nbytes > 0) {
    if (up_nbytes % 16 || !up_dst || !up_host || (up_ctr == nullptr) != (up_flag == nullptr))
      return (int)hipErrorInvalidValue;
    void* dsrc = nullptr;
    const hipError_t e = hipHostGetDevicePointer(&dsrc, const_cast<void*>(up_host), 0);
    if (e != hipSuccess) return (int)e;
    // the gather reads lid / idx from the pinned copy: both must lie inside the uploaded range
    const char *d0 = (const char*)up_dst, *d1 = d0 + up_nbytes;
    const char *l0 = (const char*)lid, *i0 = (const char*)idx;
    const long lb = (long)K * 8, ib = (long)steps * K * B * 8;
    if (l0 < d0 || l0 + lb > d1 || i0 < d0 || i0 + ib > d1) return (int)hipErrorInvalidValue;
    lid = (const long long*)((const char*)dsrc + (l0 - d0));
    idx = (const long long*)((const char*)dsrc + (i0 - d0));
    const long n16 = up_nbytes / 16, ub = (n16 + 255) / 256;
    up = UploadJob{(const uint4*)dsrc, (uint4*)up_dst, n16, up_ctr, up_flag, (int)(ub < 256 ? ub : 256)};
  }
  // without client rows or moments to set, only the step counters need a block (chunk 0 of row 0)
  const bool rows = params || m || v;
  const int chunks = rows ? (P + SG_E - 1) / SG_E : (t ? 1 : 0);
  const int kinit = rows ? K : (t ? 1 : 0);
  const long gather_rows = (long)steps * K * B;
  // short rows: tps lanes per row, 256 / tps rows per block (prologue_gather_lanes, shared with the trainer's gate)
  const int tps = qfx_prologue_gather_lanes(F);
  const long gather = tps ? (gather_rows + 256 / tps - 1) / (256 / tps) : gather_rows;
  if (nzero < 0 || (nzero > 0 && !zero)) return (int)hipErrorInvalidValue;
  const long blocks = (long)kinit * chunks + gather + n_slots + (nzero > 0 ? 1 : 0) + up.blocks;
  if (blocks > 0x7fffffffL) return (int)hipErrorInvalidValue;
  if (blocks == 0) return 0;
  hipLaunchKernelGGL(qfx_round_prologue_kernel, dim3((unsigned)blocks), dim3(256), 0, st,
                     RoundInit{theta, kinit, P, params, m, v, t, nt}, chunks,
                     BatchGather{X, Y, lid, idx, K, B, nmax, F, mode, alpha, xo, x_stride, yo},
                     FragJob{slot_tab, n_slots, (uint4*)frags, bf16}, gather, gather_rows, tps, zero, nzero, up);
  return (int)hipGetLastError();
}

extern "C" int qfx_prologue_gather_lanes(int F) {
  if (F <= 0 || F > 64) return 0;
  int t = 8;
  while (t < F) t <<= 1;
  return t;
}

extern "C" int qfx_launch_batch_gather(const float* X, const long long* Y, const long long* lid, const long long* idx,
                                       int K, int B, long nmax, int F, int mode, float alpha, float* xo, int x_stride,
                                       long long* yo, hipStream_t st) {
  if (K <= 0 || B <= 0) return 0;
  const int threads = F > 64 ? 256 : 64;
  hipLaunchKernelGGL(qfx_batch_gather_kernel, dim3((unsigned)((long)K * B)), dim3(threads), 0, st,
                     BatchGather{X, Y, lid, idx, K, B, nmax, F, mode, alpha, xo, x_stride, yo});
  return (int)hipGetLastError();
}

extern "C" int qfx_launch_fedavg(const float* theta_k, const float* theta_g, const unsigned char* angle_mask,
                                 const double* weights, double* norms, const uint32_t* keys, int K, int P,
                                 int wrap, int dp, float clip, float sigma, long long* out, long long* pack_buf,
                                 const float* loss, const float* correct, const float* nvalid, const float* act,
                                 int n_metrics, long long* sat, const uint32_t* sa_seeds, const int* sa_sign,
                                 const int* sa_round, int sa_n, double sa_scale, int sa_bits, long long* sa_masks,
                                 const int* norm_cid, float* fa_theta, double* fa_out, unsigned* fa_cnt,
                                 int fa_bits, double fa_ring_scale, int fa_n_norms, const float* dp_scale,
                                 int sa_pairsym, hipStream_t st) {
  if (dp) {   // clipping needs the per-client norms; without DP they are not computed
    const int nc = (P + NORM_CHUNK - 1) / NORM_CHUNK;
    double* partial = norms + K;   // scratch tail of the norms buffer: K * nc doubles
    hipLaunchKernelGGL(qfx_delta_norm_partial_kernel, dim3(K, nc), dim3(256), 0, st, theta_k, theta_g, angle_mask, P,
                       wrap, partial);
    hipLaunchKernelGGL(qfx_delta_norm_final_kernel, dim3((K + 63) / 64), dim3(64), 0, st, partial, nc, K, norms);
  }
  const RoundPack rp{pack_buf, loss, correct, nvalid, act, n_metrics, (dp && norm_cid) ? norms : nullptr, norm_cid, K};
  const int epb = sa_bits <= 32 ? 4 : 2;
  const SecAgg sa{sa_seeds, sa_sign, sa_round, sa_n, sa_scale, sa_seeds ? (1LL << sa_bits) - 1 : 0, sa_masks, epb};
  if (sa_seeds) {
    if (!sa_masks) return (int)hipErrorInvalidValue;
    const long nblk = (P + 1 + epb - 1) / epb;
    if (sa_pairsym) {   // square table (host-checked: N == K <= 128, row k = client k)
      const size_t lds = (size_t)K * 512;             // [NB][2][EPB][K] int64 (NB x EPB = 32)
      if (K > 128) return (int)hipErrorInvalidValue;
      if (epb == 2)
        hipLaunchKernelGGL(qfx_secagg_pairsym_kernel<2>, dim3((unsigned)((nblk + SaPs<2>::NB - 1) / SaPs<2>::NB)),
                           dim3(256), lds, st, sa, K, P);
      else
        hipLaunchKernelGGL(qfx_secagg_pairsym_kernel<4>, dim3((unsigned)((nblk + SaPs<4>::NB - 1) / SaPs<4>::NB)),
                           dim3(256), lds, st, sa, K, P);
    } else {
      hipLaunchKernelGGL(qfx_secagg_mask_kernel, dim3((unsigned)((nblk + 255) / 256), (unsigned)K), dim3(256), 0,
                         st, sa, P);
    }
  }
  const unsigned blocks = (unsigned)((P + FA_E - 1) / FA_E) + (pack_buf ? 1u : 0u);
  // the fused apply reads the whole [P + 6 + n_norms] buffer this launch writes: it needs the pack block and the
  // buffer head to be this launch's output
  if (fa_theta && (!pack_buf || !fa_out || !fa_cnt || out != pack_buf || fa_bits < 0 || fa_bits > 62 ||
                   fa_n_norms < 0 || (fa_bits != 0) != (sa_seeds != nullptr)))
    return (int)hipErrorInvalidValue;
  const FusedApply fa{fa_theta, fa_out, fa_cnt, fa_bits, fa_n_norms, fa_ring_scale, 1.0};
  if (!dp && !sa_seeds)
    hipLaunchKernelGGL(qfx_fedavg_reduce_kernel<true>, dim3(blocks), dim3(FA_E * FA_G), 0, st, theta_k, theta_g,
                       angle_mask, weights, norms, keys, nullptr, K, P, wrap, 0, clip, sigma, out, rp, sat, sa, fa);
  else
    hipLaunchKernelGGL(qfx_fedavg_reduce_kernel<false>, dim3(blocks), dim3(FA_E * FA_G), 0, st, theta_k, theta_g,
                       angle_mask, weights, norms, keys, dp ? dp_scale : nullptr, K, P, wrap, dp, clip, sigma, out, rp,
                       sat, sa, fa);
  return (int)hipGetLastError();
}
