// Client-batched TinyCNN (CFed path) on gfx950: fused conv + bias + ReLU + 2x2 max-pool forward, the
// conv backward (unpool, conv2 weight + input gradients, conv1 weight gradient), the fc head
// (ReLU + dropout + fc2 + cross-entropy + their backward) and the deterministic gradient reduction.
//
// Reference: TinyCNN / client_update (src/CFed/Classical_FL.py:21-64); SURVEY §2.3 K1-K5, K7.
// The reference trains K clients one after another with separate cuDNN-style library calls; here all
// K clients x B samples run as one launch, every client with its own weights (row k of the flat
// [K, P] parameter buffer, reference key order).
//
// Matrix work uses fp32 MFMA, v_mfma_f32_16x16x4_f32 (wave64): lane l supplies A[l%16][l/16] and
// B[l/16][l%16] and holds D[4*(l/16)+r][l%16] (r = 0..3).  Convolutions are implicit GEMMs over
// LDS-staged, zero-padded feature maps with precomputed im2col offset tables.  For the forward
// convs the GEMM rows are ordered (pool window, position in window), so the 4 accumulator
// registers of a lane are exactly one 2x2 pooling window of one channel: bias + ReLU + max-pool +
// argmax happen in registers, and the pre-pool activation never exists in memory.
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>

#include "cnn_args.h"
#include "philox.h"

namespace qfx {
namespace cnn {

typedef float f4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ f4 mfma(float a, float b, f4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}

constexpr int NT = 512;            // threads per workgroup (8 waves)
constexpr int NW = NT / 64;
constexpr int IMG = 28, IMGP = 32; // conv1 input, zero-padded by 2
constexpr int C1 = 16, H1 = 28, Q1 = 14;   // conv1 channels, output size, pooled size
constexpr int C2 = 32, H2 = 14, Q2 = 7;    // conv2 channels, output size, pooled size
constexpr int P1P = 18;            // pooled1 zero-padded by 2 (conv2 input)
constexpr int K1 = 25, K1P = 28;   // conv1 reduction (dy,dx), padded to the MFMA k-step
constexpr int K2 = 400;            // conv2 reduction (ci,dy,dx)

struct CnnOff {                    // float offsets of the tensors inside one client's parameter row
  int w1, b1, w2, b2;
};

// One gradient entry of client k (row stride P) into its sink (cnn_args.h): the gradient row, or the fused SGD step.
__device__ __forceinline__ void sink_put(const CnnSgd& sg, int P, int k, long e, float g) {
  if (!sg.pout) {
    sg.grad[(size_t)k * P + e] = g;
    return;
  }
  const float pin = sg.pin[(size_t)k * sg.pstride + e];
  float out = pin;
  if (sg.act[k] != 0.f) {
    const bool first = sg.t_in[k] == 0.f;   // the momentum buffer is the gradient on the first step (never read)
    const float b = first ? g : fmaf(sg.mu, sg.buf[(size_t)k * P + e], g);
    if (sg.keep) sg.buf[(size_t)k * P + e] = b;
    out = pin - sg.lr * b;
  }
  sg.pout[(size_t)k * P + e] = out;
}

// Four consecutive entries e .. e + 3 of client k's row (rows are only 4-byte aligned: dword-aligned 16-byte accesses),
// the same element math as sink_put
typedef float f4a __attribute__((ext_vector_type(4), aligned(4)));
__device__ __forceinline__ void sink_put4(const CnnSgd& sg, int P, int k, long e, f4 g) {
  if (!sg.pout) {
    *(f4a*)(sg.grad + (size_t)k * P + e) = g;
    return;
  }
  const f4a pin = *(const f4a*)(sg.pin + (size_t)k * sg.pstride + e);
  f4a out = pin;
  if (sg.act[k] != 0.f) {
    const bool first = sg.t_in[k] == 0.f;
    f4a b = g;
    if (!first) {
      const f4a m = *(const f4a*)(sg.buf + (size_t)k * P + e);
#pragma unroll
      for (int j = 0; j < 4; ++j) b[j] = fmaf(sg.mu, m[j], g[j]);
    }
    if (sg.keep) *(f4a*)(sg.buf + (size_t)k * P + e) = b;
#pragma unroll
    for (int j = 0; j < 4; ++j) out[j] = pin[j] - sg.lr * b[j];
  }
  *(f4a*)(sg.pout + (size_t)k * P + e) = out;
}

// --------------------------------------------------------------------------------------------
// layout probe: D[16x16] = A[16xK] B[Kx16] with one wave (tests pin the MFMA operand layout)
// --------------------------------------------------------------------------------------------
__global__ void mfma_probe(const float* A, const float* B, float* D, int K) {
  const int l = threadIdx.x;
  f4 acc = {0.f, 0.f, 0.f, 0.f};
  for (int k0 = 0; k0 < K; k0 += 4) acc = mfma(A[(l % 16) * K + k0 + l / 16], B[(k0 + l / 16) * 16 + l % 16], acc);
  for (int r = 0; r < 4; ++r) D[(4 * (l / 16) + r) * 16 + l % 16] = acc[r];
}

// --------------------------------------------------------------------------------------------
// shared helpers
// --------------------------------------------------------------------------------------------
__device__ __forceinline__ int q14(int p) { return p + 4 * (p / H2); }   // (y, x) of a 14x14 map -> 18*y + x
__device__ __forceinline__ int tap_off(int r) { return (r / 5) * P1P + r % 5; }   // 5x5 tap -> padded 18-wide map

// Software-pipelined loop over k-chunks [c0, c1): chunk c+1's operands are read into the other register
// set before chunk c's MFMAs issue (the sched barriers keep the compiler from sinking the reads below
// the MFMAs), so LDS latency overlaps matrix work even with two waves per SIMD.
template <class Set, class Load, class Mma>
__device__ __forceinline__ void pipelined(int c0, int c1, Load&& load, Mma&& mma) {
  Set s0, s1;
  load(c0, s0);
  int c = c0;
#pragma unroll 1
  for (; c + 2 < c1; c += 2) {
    load(c + 1, s1);
    __builtin_amdgcn_sched_barrier(0);
    mma(s0);
    __builtin_amdgcn_sched_barrier(0);
    load(c + 2, s0);
    __builtin_amdgcn_sched_barrier(0);
    mma(s1);
    __builtin_amdgcn_sched_barrier(0);
  }
  if (c + 1 < c1) {
    load(c + 1, s1);
    __builtin_amdgcn_sched_barrier(0);
    mma(s0);
    mma(s1);
  } else {
    mma(s0);
  }
}

// bias + ReLU + 2x2 max-pool (+ argmax 0..3, first maximum wins) of one window held in 4 registers
__device__ __forceinline__ float relu_pool(f4 acc, float bias, int& arg) {
  float best = fmaxf(acc[0] + bias, 0.f);
  arg = 0;
#pragma unroll
  for (int r = 1; r < 4; ++r) {
    const float v = fmaxf(acc[r] + bias, 0.f);
    if (v > best) { best = v; arg = r; }
  }
  return best;
}

// --------------------------------------------------------------------------------------------
// forward: conv1 -> ReLU -> pool -> conv2 -> ReLU -> pool for FSG samples of one client
//   outputs per sample: pool1 [16][196], am1 [16][196] (argmax 0..3), pool2 [32][49], am2 [32][49]
//
//   conv1  M = 196 windows x 4 (49 m-tiles), N = 16, K = 28: B (W1) stays in 7 registers for the whole
//          phase, each lane's 7 tap offsets are registers; two m-tiles per step (two MFMA chains)
//   conv2  M = 48 windows x 4 (12 full m-tiles) + window 48, N = 32, K ordered (tap, ci) = 25 x 16:
//          A[row][(r, ci)] = p1pad[ci][q(row) + off(r)], B = w2f[o][r*16 + ci]; the tap offset is
//          wave-uniform and ci runs over immediate offsets.  Wave w owns 6 full (sample, m-tile)
//          units as two groups of 3 m-tiles (6 accumulator chains) and half the taps of sample
//          w/2's last m-tile (window 48); the two halves are summed in fixed order afterwards.
// --------------------------------------------------------------------------------------------
constexpr int FSG = 4;             // samples per forward workgroup
constexpr int IRF = 46;            // LDS row stride of a padded forward image (32 used): conv1's A reads of 4
                                   // windows x 2 rows x 2 taps average 1.19-way vs 2.24-way at stride 32
static_assert(FSG * 2 == NW, "conv2 partial m-tile: one (sample, half) per wave");

// conv2 runs on the fp16 matrix pipe at fp32-grade accuracy: every fp32 operand x is split into fp16 halves
// hi = fp16(x), lo = fp16(x - hi) (22 significant bits) and each K = 32 slab takes three v_mfma_f32_16x16x32_f16
// (hi.hi + hi.lo + lo.hi; lo.lo is below the split's own 2^-22) with fp32 accumulation - 48 MFMA cycles where the
// fp32 pipe (v_mfma_f32_16x16x4_f32) needed 256.  W2 is scaled by 2^8 before the split (its 0.05-scale lo halves
// would sit in fp16's subnormal range) and the accumulators by 2^-8 after (exact).  CPU emulation of the split on
// TinyCNN conv2 (max |err| / max |y| against float64): 1.30e-6 vs 0.97e-6 for fp32 (3 x bf16: 6.9e-6).
//   K ordered (tap, ci), 13 slabs of 2 taps x 16 channels (tap 25 is zero): lane group g = lane / 16 supplies
//   k = 8 g .. 8 g + 7 = tap 2 slab + g / 2, channels 8 (g & 1) .. + 7 - one 16-byte chunk of a position record.
constexpr int NPOS = P1P * P1P;    // positions of the zero-padded 18 x 18 pool1 map
constexpr int PRQ = 4;             // 16-byte chunks per position record: hi ci 0-7 | hi ci 8-15 | lo ci 0-7 | lo 8-15
constexpr int W2T = 5;             // chunks per tap record of the split W2 image (4 + 1 pad: the staging stores of a
                                   // wave's consecutive taps spread over 8 bank groups instead of 2 - 6.5-way, not 12-way)
constexpr int W2Q = 130;           // chunks per output channel of the split W2 image (26 taps x 5: the 16
                                   // lanes of a ds_read_b128 group land on distinct 16-byte bank slots)
constexpr int NSL = 13;            // K slabs
constexpr float SW2 = 256.f;       // W2 scale before the split (power of two, undone on the accumulators)

// pool1 record chunk c of position pos sits at chunk c ^ h(pos): with the fwd_win row order the 16 rows of an
// m-tile have distinct pos mod 16, and this XOR puts each 16-lane ds_read_b128 group on distinct bank slots
// (exhaustive check over tiles, taps and lane groups: 1.08-way on average, from 2-way unswizzled)
__device__ __forceinline__ int p1_chunk(int pos, int c) { return c ^ ((pos ^ (pos >> 1)) & 3); }

typedef _Float16 h8 __attribute__((ext_vector_type(8)));
__device__ __forceinline__ f4 mfma_h(uint4 a, uint4 b, f4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(h8, a), __builtin_bit_cast(h8, b), c, 0, 0, 0);
}

// conv2 (forward) m-tile slot (tile * 4 + j, slot 48 = the partial tile) -> pooled window wy * 7 + wx.  A 32-lane
// half of an A read touches 4 windows x 4 positions of two channels CSF apart: with window origins o = 36 wy + 2 wx,
// positions {0, 1, 18, 19} and CSF == 16 (mod 32) its 32 banks are distinct iff the 4 windows share the parity of wx
// and have distinct (2 wy + wx) mod 8.  Tiles 0-6 are the even-wx windows of one row, tiles 7-11 the odd-wx triple
// of rows 0-4 plus one odd window of rows 5 / 6 (packed 6-bit ids), window 43 = (6, 1) is left for the partial
// tile.  In plain row order two windows of a tile collide and every A read of the round-4 kernel was 2-way
// (PMC: 44% of the kernel's LDS cycles were conflict cycles).
__device__ __forceinline__ int fwd_win(int slot) {
  const int t = slot >> 2, j = slot & 3;
  if (slot >= Q2 * Q2 - 1) return 43;
  if (t < 7) return t * Q2 + 2 * j;
  if (j < 3) return (t - 7) * Q2 + 2 * j + 1;
  return (0x2D9A4BE8u >> (6 * (t - 7))) & 63;   // 40, 47, 36, 38, 45
}

// conv2 (forward) GEMM row -> offset of its 5x5 window origin in the padded 18-wide map
__device__ __forceinline__ int fwd_q2(int row) {
  const int w = fwd_win(min(row >> 2, Q2 * Q2 - 1)), pos = row & 3;   // rows past slot 48 clamp (dropped later)
  return (2 * (w / Q2) + (pos >> 1)) * P1P + 2 * (w % Q2) + (pos & 1);
}

template <int NM>
struct Fwd2Set {
  uint4 ah[NM], al[NM], bh[2], bl[2];
};

// conv2 over slabs [c0, c1) for NM m-tiles of one sample: apos = each m-tile row's window position (lane row i),
// p1 = the sample's position records, w2 = lane column i's W2 chunks (+ 16 W2Q for the second n-tile)
template <int NM>
__device__ __forceinline__ void fwd_conv2(const uint4* p1, const int (&apos)[NM], const uint4* w2, int g, int c0,
                                          int c1, f4 (&acc)[NM][2]) {
  const int tpar = g >> 1, ch = g & 1;
  pipelined<Fwd2Set<NM>>(
      c0, c1,
      [&](int sl, Fwd2Set<NM>& st) {
        const int tap = 2 * sl + tpar;
        const uint4* bp = w2 + tap * W2T + ch;
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          st.bh[h] = bp[h * 16 * W2Q];
          st.bl[h] = bp[h * 16 * W2Q + 2];
        }
        const int ro = tap_off(min(tap, K1 - 1));   // tap 25 has zero weights: any in-range position
#pragma unroll
        for (int m = 0; m < NM; ++m) {
          const int pos = apos[m] + ro;
          const uint4* rec = p1 + pos * PRQ;
          st.ah[m] = rec[p1_chunk(pos, ch)];
          st.al[m] = rec[p1_chunk(pos, 2 + ch)];
        }
      },
      [&](const Fwd2Set<NM>& st) {
#pragma unroll
        for (int m = 0; m < NM; ++m)
#pragma unroll
          for (int h = 0; h < 2; ++h) {
            acc[m][h] = mfma_h(st.ah[m], st.bh[h], acc[m][h]);
            acc[m][h] = mfma_h(st.ah[m], st.bl[h], acc[m][h]);
            acc[m][h] = mfma_h(st.al[m], st.bh[h], acc[m][h]);
          }
      });
}

// LDS of cnn_fwd (bytes, 16-byte aligned pieces): pool1 records | (images during conv1, then the split W2) | W1 |
// b1 | b2 | window-48 partials
constexpr int FWD_P1_B = FSG * NPOS * PRQ * 16;
constexpr int FWD_U_B = (C2 * W2Q * 16 > FSG * IMGP * IRF * 4) ? C2 * W2Q * 16 : FSG * IMGP * IRF * 4;
constexpr int FWD_LDS = FWD_P1_B + FWD_U_B + (C1 * K1P + C1 + C2 + FSG * 2 * C2 * 4) * 4;
static_assert(FWD_LDS <= 160 * 1024, "cnn_fwd LDS");

__global__ void __launch_bounds__(NT) cnn_fwd(const float* __restrict__ X, const float* __restrict__ params,
                                              int P, int B, int G, CnnOff off, float* __restrict__ pool1,
                                              uint8_t* __restrict__ am1, float* __restrict__ pool2,
                                              uint8_t* __restrict__ am2) {
  extern __shared__ __attribute__((aligned(16))) float sm[];
  uint4* p1q = reinterpret_cast<uint4*>(sm);                          // [FSG][324][4] split pool1 records
  char* ub = reinterpret_cast<char*>(sm) + FWD_P1_B;
  float* img = reinterpret_cast<float*>(ub);                          // [FSG][32][46] zero-padded images (conv1)
  uint4* w2q = reinterpret_cast<uint4*>(ub);                          // [32][106] split W2 chunks (conv2)
  float* w1s = reinterpret_cast<float*>(ub + FWD_U_B);                // [16][28]  (tap >= 25 zero)
  float* b1s = w1s + C1 * K1P;                                        // [16]
  float* b2s = b1s + C1;                                              // [32]
  float* red = b2s + C2;                                              // [FSG][2 halves][32 o][4]: window-48 partials

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int k = blockIdx.x / G, g = blockIdx.x - k * G;
  const int s0 = g * FSG;
  const int ns = min(FSG, B - s0);
  const float* prow = params + (size_t)k * P;
  const int i = lane & 15, kq = lane >> 4;

  // W2 loads are issued now and land in registers behind conv1; they are split into the image region once conv1
  // has consumed the images
  constexpr int NU2 = (C2 * K2 + NT - 1) / NT;
  float w2v[NU2];
#pragma unroll
  for (int u = 0; u < NU2; ++u) {
    const int e = tid + u * NT;
    if (e < C2 * K2) w2v[u] = prow[off.w2 + e];
  }
  for (int e = tid; e < C1 * K1P; e += NT) {
    const int o = e / K1P, kk = e - o * K1P;
    w1s[e] = kk < K1 ? prow[off.w1 + o * K1 + kk] : 0.f;
  }
  if (tid < C1) b1s[tid] = prow[off.b1 + tid];
  if (tid < C2) b2s[tid] = prow[off.b2 + tid];
  {
    constexpr int NU = FSG * IMGP * IMGP / NT;
    static_assert(NU * NT == FSG * IMGP * IMGP && IMGP == 32, "whole image rows per thread");
    float v[NU];
#pragma unroll
    for (int u = 0; u < NU; ++u) {
      const int e = tid + u * NT;
      const int s = e / (IMGP * IMGP), r = e - s * IMGP * IMGP, y = r / IMGP - 2, x = r % IMGP - 2;
      v[u] = (s < ns && y >= 0 && y < IMG && x >= 0 && x < IMG) ? X[((size_t)k * B + s0 + s) * IMG * IMG + y * IMG + x] : 0.f;
    }
#pragma unroll
    for (int u = 0; u < NU; ++u) {
      const int e = tid + u * NT, r = e & (IMGP * IMGP - 1);
      img[(e >> 10) * IMGP * IRF + (r >> 5) * IRF + (r & 31)] = v[u];
    }
  }
  for (int e = tid; e < FSG * NPOS * PRQ; e += NT) p1q[e] = make_uint4(0u, 0u, 0u, 0u);
  __syncthreads();

  // ---- conv1 (fp32 MFMA, K = 28): pooled outputs to global and, split, into the pool1 records
  _Float16* p1h = reinterpret_cast<_Float16*>(p1q);
  {
    float bw[K1P / 4];
    int toff[K1P / 4];
#pragma unroll
    for (int ks = 0; ks < K1P / 4; ++ks) {
      const int kk = ks * 4 + kq;
      bw[ks] = w1s[i * K1P + kk];
      toff[ks] = kk < K1 ? (kk / 5) * IRF + kk % 5 : 0;   // w1s is zero there
    }
    const int nu = ns * 49;
    for (int u = wave; u < nu; u += 2 * NW) {
      const int u1 = u + NW < nu ? u + NW : u;
      int ubs[2];
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const int uu = h ? u1 : u, s = uu / 49, mt = uu - s * 49;
        const int w = mt * 4 + (i >> 2), pos = i & 3;
        ubs[h] = s * IMGP * IRF + (2 * (w / Q1) + (pos >> 1)) * IRF + 2 * (w % Q1) + (pos & 1);
      }
      float av[2][K1P / 4];
#pragma unroll
      for (int h = 0; h < 2; ++h)
#pragma unroll
        for (int ks = 0; ks < K1P / 4; ++ks) av[h][ks] = img[ubs[h] + toff[ks]];
      f4 acc[2] = {f4{0.f, 0.f, 0.f, 0.f}, f4{0.f, 0.f, 0.f, 0.f}};
#pragma unroll
      for (int ks = 0; ks < K1P / 4; ++ks)
#pragma unroll
        for (int h = 0; h < 2; ++h) acc[h] = mfma(av[h][ks], bw[ks], acc[h]);
      // lane holds window wo = mt*4 + kq, its 4 positions, channel o = i
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        if (h == 1 && u1 == u) break;
        const int uu = h ? u1 : u, s = uu / 49, mt = uu - s * 49;
        const int wo = mt * 4 + kq, o = i;
        int arg;
        const float best = relu_pool(acc[h], b1s[o], arg);
        const size_t so = ((size_t)k * B + s0 + s) * C1 * Q1 * Q1 + o * Q1 * Q1 + wo;
        pool1[so] = best;
        am1[so] = (uint8_t)arg;
        const int pos = (wo / Q1 + 2) * P1P + (wo % Q1) + 2;
        const _Float16 hi = (_Float16)best, lo = (_Float16)(best - (float)hi);
        _Float16* rec = p1h + (size_t)(s * NPOS + pos) * PRQ * 8 + (o & 7);
        rec[8 * p1_chunk(pos, o >> 3)] = hi;
        rec[8 * p1_chunk(pos, 2 + (o >> 3))] = lo;
      }
    }
  }
  __syncthreads();   // images consumed: the region takes the split W2

  {
    _Float16* w2h = reinterpret_cast<_Float16*>(w2q);
#pragma unroll
    for (int u = 0; u < NU2; ++u) {
      const int e = tid + u * NT;
      if (e < C2 * K2) {
        const int o = e / K2, rem = e - o * K2, ci = rem / 25, tap = rem - ci * 25;
        const float x = w2v[u] * SW2;
        const _Float16 hi = (_Float16)x, lo = (_Float16)(x - (float)hi);
        _Float16* rec = w2h + (size_t)(o * W2Q + tap * W2T) * 8 + (ci & 7);
        rec[8 * (ci >> 3)] = hi;
        rec[8 * (2 + (ci >> 3))] = lo;
      }
    }
    if (tid < C2 * PRQ) w2q[(tid >> 2) * W2Q + (K1 * W2T) + (tid & 3)] = make_uint4(0u, 0u, 0u, 0u);   // tap 25
  }
  __syncthreads();

  // ---- conv2: full m-tiles
  const uint4* w2l = w2q + i * W2Q;
  constexpr float USC = 1.f / SW2;
#pragma unroll 1
  for (int gq = 0; gq < 2; ++gq) {
    const int u = 6 * wave + 3 * gq, s = u / 12, mt0 = u - s * 12;
    if (s >= ns) break;
    int apos[3];
#pragma unroll
    for (int m = 0; m < 3; ++m) apos[m] = fwd_q2((mt0 + m) * 16 + i);
    f4 acc[3][2] = {};
    fwd_conv2<3>(p1q + s * NPOS * PRQ, apos, w2l, kq, 0, NSL, acc);
#pragma unroll
    for (int m = 0; m < 3; ++m) {
      const int wo = fwd_win((mt0 + m) * 4 + kq);
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const int o = h * 16 + i;
        int arg;
        const float best = relu_pool(acc[m][h] * USC, b2s[o], arg);
        const size_t so = ((size_t)k * B + s0 + s) * C2 * Q2 * Q2 + o * Q2 * Q2 + wo;
        pool2[so] = best;
        am2[so] = (uint8_t)arg;
      }
    }
  }
  // ---- conv2: window 48 (m-tile 12), half of the slabs per wave
  {
    const int s = wave >> 1, half = wave & 1;
    f4 acc[1][2] = {};
    if (s < ns) {
      const int apos[1] = {fwd_q2(12 * 16 + i)};
      fwd_conv2<1>(p1q + s * NPOS * PRQ, apos, w2l, kq, half ? 7 : 0, half ? NSL : 7, acc);
    }
    if (s < ns && kq == 0) {
#pragma unroll
      for (int h = 0; h < 2; ++h)
#pragma unroll
        for (int r = 0; r < 4; ++r) red[((s * 2 + half) * C2 + h * 16 + i) * 4 + r] = acc[0][h][r];
    }
  }
  __syncthreads();
  if (tid < ns * C2) {
    const int s = tid / C2, o = tid - s * C2;
    f4 v;
#pragma unroll
    for (int r = 0; r < 4; ++r) v[r] = (red[((s * 2) * C2 + o) * 4 + r] + red[((s * 2 + 1) * C2 + o) * 4 + r]) * USC;
    int arg;
    const float best = relu_pool(v, b2s[o], arg);
    const size_t so = ((size_t)k * B + s0 + s) * C2 * Q2 * Q2 + o * Q2 * Q2 + fwd_win(Q2 * Q2 - 1);
    pool2[so] = best;
    am2[so] = (uint8_t)arg;
  }
}

// --------------------------------------------------------------------------------------------
// backward of the conv stack for bs samples of one client -> per-workgroup gradient partials
//   part[(k*G + g)][ dW2 (12800) | db2 (32) | dW1 (400) | db1 (16) ]
//
// Per sample the three GEMMs are laid out so that no operand needs an index table and every
// MFMA operand is one unpredicated ds_read_b32 from a per-lane base:
//   conv2 wgrad  D[o][(tap, ci)] = sum_p dC2[o][p] P1pad[ci][q(p) + off(tap)]    M=32  N=26x16 K=196
//                n-tile = one tap (lane = ci), plus a 26th "ones" n-tile that yields db2
//   conv2 dgrad  D[p][ci] = sum_{tap,o} dC2pad[o][rb(p) - off(tap)] W2[o][ci][tap] M=196 N=16    K=25x32
//                on the fp16 pipe like the forward conv2: one K = 32 slab per tap (k = o), dC2 staged as split
//                channel-minor position records with a per-sample power-of-two scale, W2 as split (ci, tap)
//                records scaled by 2^8; the wgrad rebuilds its dC2 operand from the same records (hi + lo)
//   conv1 wgrad  D[o][tap] = sum_p dC1[o][p] img[p + off1(tap)]                    M=16  N=32    K=784
//                tap 25 is a ones column (db1); taps 26..31 are discarded
// Work split (MFMA count per SIMD balanced; waves w and w+4 share a SIMD): wave w<4 owns dgrad
// m-tiles 2w, 2w+1 and 7 wgrad n-tiles; wave w>=4 owns dgrad m-tile 4+w, a quarter of the
// reduction of m-tile 12 (rows 192..195, the only partial tile) and 6 wgrad n-tiles.  Every wave
// also takes an eighth of the previous sample's conv1 wgrad (its inputs are double buffered), so
// a sample costs two barriers; the next sample's global inputs load into registers meanwhile.
// --------------------------------------------------------------------------------------------
constexpr int BS_MAX = 16;         // samples per backward workgroup, at most (bwd_bs)
constexpr int DRQ = 8;             // 16-byte chunks per dC2 position record / split W2 (ci, tap) record:
                                   // hi o 0-7 | hi o 8-15 | hi o 16-23 | hi o 24-31 | lo o 0-7 | ... | lo o 24-31
constexpr int W2B = 202;           // chunks per input channel of the split W2 image (25 taps x 8 + 2 pad: the 16
                                   // lanes of a ds_read_b128 group land on distinct 16-byte bank slots)
// dC2 record chunk c of position pos sits at chunk c ^ (pos & 7): conflict-free b128 dgrad A reads for every m-tile,
// tap and lane group (exhaustive check; 4.3-way on average unswizzled)
__device__ __forceinline__ int dc_chunk(int pos, int c) { return c ^ (pos & 7); }
// Power-of-two scale of one sample's dC2 for the fp16 split: the largest |value| lands in [2^14, 2^15)
// (conv-stack gradients are ~1e-5..1e-3: unscaled, their fp16 halves would be subnormal)
__device__ __forceinline__ float dc_scale(float m) {
  if (!(m > 0.f)) return 1.f;
  int e;
  (void)frexpf(m, &e);
  return ldexpf(1.f, 15 - e);
}
__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}
constexpr int DPS = 198;           // LDS stride of the dP1 / argmax1 rows
constexpr int IMS = 37;            // LDS row stride of the padded image
constexpr int NT2 = 26;            // conv2 wgrad n-tiles (25 taps + ones)
constexpr int PART = C2 * K2 + C2 + C1 * K1 + C1;

// conv2 dgrad GEMM row (m-tile * 16 + row) -> dp1 pixel p = 14 y + x.  Tile t holds the t-th pixel (in row order) of
// every residue class of (2 y + x) mod 16; rows 192..195 (partial m-tile 12) the four classes that have a 13th.  (Chosen
// for the round-5 fp32 channel-strided image; with the split position records and dc_chunk's XOR the b128 A reads are
// conflict-free in this order.)
__constant__ uint8_t kDgPix[H2 * H2] = {
    0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 26, 27, 40, 41, 14, 15, 16, 17, 18, 19, 20, 21, 22, 23,
    24, 25, 38, 39, 52, 53, 54, 55, 28, 29, 30, 31, 32, 33, 34, 35, 36, 37, 50, 51, 64, 65, 66, 67, 68, 69, 42, 43,
    44, 45, 46, 47, 48, 49, 62, 63, 76, 77, 78, 79, 80, 81, 82, 83, 56, 57, 58, 59, 60, 61, 74, 75, 88, 89, 90, 91,
    92, 93, 94, 95, 96, 97, 70, 71, 72, 73, 86, 87, 100, 101, 102, 103, 104, 105, 106, 107, 108, 109, 110, 111, 84, 85, 98, 99,
    112, 113, 114, 115, 116, 117, 118, 119, 120, 121, 122, 123, 124, 125, 138, 139, 152, 153, 126, 127, 128, 129, 130, 131, 132, 133, 134, 135,
    136, 137, 150, 151, 164, 165, 166, 167, 140, 141, 142, 143, 144, 145, 146, 147, 148, 149, 162, 163, 176, 177, 178, 179, 180, 181, 154, 155,
    156, 157, 158, 159, 160, 161, 174, 175, 188, 189, 190, 191, 192, 193, 194, 195, 168, 169, 170, 171, 172, 173, 186, 187, 182, 183, 184, 185,
};
__device__ __forceinline__ int dg_pix(int row) { return kDgPix[min(row, H2 * H2 - 1)]; }

// conv2 wgrad of one sample on the fp16 pipe: D[o][(tap, ci)] += sum_k dC2[o][p_k] P1[ci][p_k + off(tap)], K = the
// 196 pool2-resolution positions in row order, padded to 7 slabs of 32 (pad rows read the zero corner record).
// Both operands have K on their LDS rows (position records) and M / N on the record's columns, so they are fetched
// with ds_read_b64_tr_b16: lane 4q + p of a 16-lane group addresses row q, columns 4p .. 4p + 3 of a 4 x 16 block,
// and lane i receives column i of the 4 rows - the MFMA's 8 consecutive k of its column in two reads.
typedef short v4s __attribute__((vector_size(8)));
__device__ __forceinline__ uint2 lds_tr16(const void* p) {
  const v4s v = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) v4s*)p);
  return __builtin_bit_cast(uint2, v);
}
__device__ __forceinline__ uint4 cat2(uint2 a, uint2 b) { return make_uint4(a.x, a.y, b.x, b.y); }
constexpr int WG_SL = 7;           // wgrad K slabs (224 rows >= 196 positions)

struct WgradSet {
  uint4 bh, bl;
};

// wgrad of one sample into acc[j] (n-tiles nt0 + j, NJ of them; n-tile 25 = the db2 ones column) for the o rows of
// m-tile wmt.  qk = the lane's block row (lane & 15) >> 2, pc = its column quad lane & 3, g = lane >> 4.
template <int NJ>
__device__ __forceinline__ void bwd_wgrad2(const char* dcb, const char* p1b, int wmt, int nt0, int g, int qk, int pc,
                                           f4 (&acc)[7]) {
  const int cA = 2 * wmt + (pc >> 1), cB = pc >> 1, eo = 8 * (pc & 1);
  const uint4 ones = make_uint4(0x3C003C00u, 0x3C003C00u, 0x3C003C00u, 0x3C003C00u);
#pragma unroll 1
  for (int sl = 0; sl < WG_SL; ++sl) {
    int q[2];   // the lane's two block rows: k = 32 sl + 8 g + 4 h + qk -> position offset q14 (-1: pad row)
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int k = 32 * sl + 8 * g + 4 * h + qk;
      q[h] = k < H2 * H2 ? q14(k) : -1;
    }
    uint4 ah, al;
    {
      uint2 rh[2], rl[2];
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const int pos = q[h] < 0 ? 0 : q[h] + 2 * P1P + 2;
        const char* rec = dcb + pos * DRQ * 16 + eo;
        rh[h] = lds_tr16(rec + 16 * dc_chunk(pos, cA));
        rl[h] = lds_tr16(rec + 16 * dc_chunk(pos, 4 + cA));
      }
      ah = cat2(rh[0], rh[1]);
      al = cat2(rl[0], rl[1]);
    }
    auto load = [&](int j, WgradSet& st) {
      const int nt = nt0 + j;
      if (nt >= 25) return;   // wave-uniform: the ones column reads nothing
      const int ro = tap_off(nt);
      uint2 bh[2], bl[2];
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const int pos = (q[h] < 0 ? 0 : q[h]) + ro;
        const char* rec = p1b + pos * PRQ * 16 + eo;
        bh[h] = lds_tr16(rec + 16 * p1_chunk(pos, cB));
        bl[h] = lds_tr16(rec + 16 * p1_chunk(pos, 2 + cB));
      }
      st.bh = cat2(bh[0], bh[1]);
      st.bl = cat2(bl[0], bl[1]);
    };
    // n-tiles one at a time, the next one's operands in flight (all of them at once would take 56 more VGPRs)
    WgradSet cur, nxt;
    load(0, cur);
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
      if (j + 1 < NJ) load(j + 1, nxt);
      __builtin_amdgcn_sched_barrier(0);
      if (nt0 + j >= 25) {
        acc[j] = mfma_h(ah, ones, acc[j]);
        acc[j] = mfma_h(al, ones, acc[j]);
      } else {
        acc[j] = mfma_h(ah, cur.bh, acc[j]);
        acc[j] = mfma_h(ah, cur.bl, acc[j]);
        acc[j] = mfma_h(al, cur.bh, acc[j]);
      }
      __builtin_amdgcn_sched_barrier(0);
      cur = nxt;
    }
  }
}

// conv2 dgrad of NM m-tiles over taps [r0, r1) on the fp16 pipe: one K = 32 slab per tap (k = o), A = the split dC2
// records at the row's position minus the tap offset, B = the lane column's (ci) split W2 record of the tap
template <int NM>
struct DgradSet {
  uint4 ah[NM], al[NM], bh, bl;
};

template <int NM>
__device__ __forceinline__ void bwd_dgrad2(const uint4* dcr, const int (&apos)[NM], const uint4* w2, int g, int r0,
                                           int r1, f4 (&acc)[NM]) {
  pipelined<DgradSet<NM>>(
      r0, r1,
      [&](int r, DgradSet<NM>& st) {
        const uint4* bp = w2 + r * DRQ;
        st.bh = bp[g];
        st.bl = bp[4 + g];
        const int ro = tap_off(r);
#pragma unroll
        for (int m = 0; m < NM; ++m) {
          const int pos = apos[m] - ro;
          const uint4* rec = dcr + pos * DRQ;
          st.ah[m] = rec[dc_chunk(pos, g)];
          st.al[m] = rec[dc_chunk(pos, 4 + g)];
        }
      },
      [&](const DgradSet<NM>& st) {
#pragma unroll
        for (int m = 0; m < NM; ++m) {
          acc[m] = mfma_h(st.ah[m], st.bh, acc[m]);
          acc[m] = mfma_h(st.ah[m], st.bl, acc[m]);
          acc[m] = mfma_h(st.al[m], st.bh, acc[m]);
        }
      });
}

// conv1 wgrad operands of one k-step: unpool1 (argmax code vs position) is resolved at MFMA time
struct C1Set {
  float d, b0, b1;
  int a1, pos;
};

// dP1 rows of a finished dgrad m-tile, ReLU-masked by pool1 > 0 (the conv1 ReLU derivative)
// (a1s bit 7 = pool1 > 0, set at staging)
__device__ __forceinline__ void bwd_dp1_store(float* dp1, const uint8_t* a1s, int mt, f4 acc, int i, int kq) {
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int row = mt * 16 + 4 * kq + r, p = dg_pix(row);
    if (row < H2 * H2) dp1[i * DPS + p] = (a1s[i * DPS + p] & 0x80) ? acc[r] : 0.f;
  }
}

// one sample's conv-stack inputs in registers (fixed per-thread element lists, all loads in flight at once)
struct BwdStage {
  static constexpr int ND = (C2 * Q2 * Q2 + NT - 1) / NT, NP = (C1 * Q1 * Q1 + NT - 1) / NT,
                       NI = (IMG * IMG + NT - 1) / NT;
  uint8_t am2[ND], a1[NP];
  float pl2[ND], dp2[ND], p1[NP], im[NI];

  __device__ __forceinline__ void load(size_t sidx, const float* __restrict__ X, const float* __restrict__ pool1,
                                       const uint8_t* __restrict__ am1, const float* __restrict__ pool2,
                                       const uint8_t* __restrict__ am2g, const float* __restrict__ dP2, int tid) {
#pragma unroll
    for (int j = 0; j < ND; ++j) {   // pooled conv2 gradients: one 2x2 window each
      const int e = tid + j * NT;
      if (e < C2 * Q2 * Q2) {
        const size_t q = sidx * C2 * Q2 * Q2 + e;
        am2[j] = am2g[q];
        pl2[j] = pool2[q];
        dp2[j] = dP2[q];
      }
    }
#pragma unroll
    for (int j = 0; j < NP; ++j) {
      const int e = tid + j * NT;
      if (e < C1 * Q1 * Q1) {
        p1[j] = pool1[sidx * C1 * Q1 * Q1 + e];
        a1[j] = am1[sidx * C1 * Q1 * Q1 + e];
      }
    }
#pragma unroll
    for (int j = 0; j < NI; ++j) {
      const int e = tid + j * NT;
      if (e < IMG * IMG) im[j] = X[sidx * IMG * IMG + e];
    }
  }
  // max |dC2| of this thread's windows (the sample's split scale)
  __device__ __forceinline__ float maxabs(int tid) const {
    float m = 0.f;
#pragma unroll
    for (int j = 0; j < ND; ++j)
      if (tid + j * NT < C2 * Q2 * Q2 && pl2[j] > 0.f) m = fmaxf(m, fabsf(dp2[j]));
    return m;
  }
  // unpool2 (+ReLU mask) into the padded split dC2 records (values x scale), pool1 -> its padded split records,
  // argmax1 (bit 7: pool1 > 0), image
  __device__ __forceinline__ void store(_Float16* dch, float scale, _Float16* p1h, uint8_t* a1s, float* img, int tid) const {
#pragma unroll
    for (int j = 0; j < ND; ++j) {
      const int e = tid + j * NT;
      if (e < C2 * Q2 * Q2) {
        const int o = e / (Q2 * Q2), w = e - o * Q2 * Q2, wy = w / Q2, wx = w - wy * Q2;
        const float v = pl2[j] > 0.f ? dp2[j] * scale : 0.f;
        const _Float16 hi = (_Float16)v, lo = (_Float16)(v - (float)hi), z = (_Float16)0.f;
        const int p0 = (2 * wy + 2) * P1P + 2 * wx + 2;
#pragma unroll
        for (int c = 0; c < 4; ++c) {
          const int pos = p0 + (c >> 1) * P1P + (c & 1);
          _Float16* rec = dch + pos * DRQ * 8 + (o & 7);
          rec[8 * dc_chunk(pos, o >> 3)] = am2[j] == c ? hi : z;
          rec[8 * dc_chunk(pos, 4 + (o >> 3))] = am2[j] == c ? lo : z;
        }
      }
    }
#pragma unroll
    for (int j = 0; j < NP; ++j) {
      const int e = tid + j * NT;
      if (e < C1 * Q1 * Q1) {
        const int ci = e / (Q1 * Q1), r = e - ci * Q1 * Q1;
        const int pos = (r / Q1 + 2) * P1P + (r % Q1) + 2;
        const _Float16 hi = (_Float16)p1[j], lo = (_Float16)(p1[j] - (float)hi);
        _Float16* rec = p1h + pos * PRQ * 8 + (ci & 7);
        rec[8 * p1_chunk(pos, ci >> 3)] = hi;
        rec[8 * p1_chunk(pos, 2 + (ci >> 3))] = lo;
        a1s[ci * DPS + r] = (uint8_t)(a1[j] | (p1[j] > 0.f ? 0x80 : 0));
      }
    }
#pragma unroll
    for (int j = 0; j < NI; ++j) {
      const int e = tid + j * NT;
      if (e < IMG * IMG) img[(e / IMG + 2) * IMS + (e % IMG) + 2] = im[j];
    }
  }
};

__global__ void __launch_bounds__(NT) cnn_bwd(const float* __restrict__ X, const float* __restrict__ params,
                                              int P, int B, int G, CnnOff off, const float* __restrict__ pool1,
                                              const uint8_t* __restrict__ am1, const float* __restrict__ pool2,
                                              const uint8_t* __restrict__ am2, const float* __restrict__ dP2,
                                              int bs, float* __restrict__ part) {
  extern __shared__ __attribute__((aligned(16))) float sm[];
  uint4* w2b = reinterpret_cast<uint4*>(sm);                // [16][202] split W2: w2b[ci][tap * 8 + chunk(o)]
  uint4* dcr = w2b + C1 * W2B;                              // [324][8] split padded dL/d conv2-output records
  _Float16* dch = reinterpret_cast<_Float16*>(dcr);
  uint4* p1r = dcr + NPOS * DRQ;                            // [324][4] split padded pool1 records (conv2 input)
  _Float16* p1h = reinterpret_cast<_Float16*>(p1r);
  // conv1 wgrad of sample s runs during sample s+1's conv2 work: its inputs are double buffered (index s & 1)
  float* dp1b = reinterpret_cast<float*>(p1r + NPOS * PRQ);   // [2][16][198] dL/d pool1, ReLU-masked
  float* imgb = dp1b + 2 * C1 * DPS;        // [2][32][37]  padded images
  float* red12 = imgb + 2 * IMGP * IMS;     // [4][64]   m-tile 12 partials of waves 4..7
  float* smax = red12 + 256;                // [8]       per-wave max |dC2| of the next staged sample
  uint8_t* a1sb = reinterpret_cast<uint8_t*>(smax + 8);   // [2][16][198] argmax of pool1
  float* red = reinterpret_cast<float*>(dcr);   // [8 waves][2][256] conv1 wgrad partials (after the sample loop)

  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);   // wave-uniform (SGPR): per-wave branches are scalar
  const int k = blockIdx.x / G, g = blockIdx.x - k * G;
  const int s0 = g * bs;
  const int ns = min(bs, B - s0);
  const float* prow = params + (size_t)k * P;
  const int i = lane & 15, kq = lane >> 4;

  {   // W2 [o][ci][tap], scaled by 2^8 and split into the dgrad B records
    constexpr int NU = (C2 * K2 + NT - 1) / NT;
    float v[NU];
#pragma unroll
    for (int u = 0; u < NU; ++u) {
      const int e = tid + u * NT;
      if (e < C2 * K2) v[u] = prow[off.w2 + e];
    }
    _Float16* w2h = reinterpret_cast<_Float16*>(w2b);
#pragma unroll
    for (int u = 0; u < NU; ++u) {
      const int e = tid + u * NT;
      if (e < C2 * K2) {
        const int o = e / K2, rem = e - o * K2, ci = rem / 25, tap = rem - ci * 25;
        const float x = v[u] * SW2;
        const _Float16 hi = (_Float16)x, lo = (_Float16)(x - (float)hi);
        _Float16* rec = w2h + (size_t)(ci * W2B + tap * DRQ) * 8 + (o & 7);
        rec[8 * (o >> 3)] = hi;
        rec[8 * (4 + (o >> 3))] = lo;
      }
    }
  }
  for (int e = tid; e < NPOS * DRQ; e += NT) dcr[e] = make_uint4(0u, 0u, 0u, 0u);
  for (int e = tid; e < NPOS * PRQ; e += NT) p1r[e] = make_uint4(0u, 0u, 0u, 0u);
  for (int e = tid; e < 2 * IMGP * IMS; e += NT) imgb[e] = 0.f;

  // conv2 wgrad tiles: m-tile (o rows) and 7 / 6 n-tiles (taps; n-tile 25 = ones -> db2)
  const int wmt = (wave >> 1) & 1;
  const int nt0 = wave < 4 ? (wave & 1) * 7 : 14 + (wave & 1) * 6;
  // the wgrad accumulators hold sum_s D_s x (the latest sample's dC2 scale): rescaled by a power of two per sample
  float wscale = 1.f;
  f4 wacc[7];
#pragma unroll
  for (int j = 0; j < 7; ++j) wacc[j] = f4{0.f, 0.f, 0.f, 0.f};
  f4 c1acc[2] = {f4{0.f, 0.f, 0.f, 0.f}, f4{0.f, 0.f, 0.f, 0.f}};
  const uint4* dgw2 = w2b + i * W2B;                 // dgrad B: lane column ci = i
  BwdStage st;
  st.load((size_t)k * B + s0, X, pool1, am1, pool2, am2, dP2, tid);
  {
    const float m = wave_max(st.maxabs(tid));
    if (lane == 0) smax[wave] = m;
  }
  __syncthreads();

  // conv1 wgrad (dC1 = unpool1(dp1) on the fly; K = 784 split across the 8 waves) of one finished sample
  const int toff0 = (i / 5) * IMS + i % 5;
  const int t1 = min(16 + i, 24);
  const int toff1 = (t1 / 5) * IMS + t1 % 5;
  const bool one1 = 16 + i >= K1;
  auto conv1_wgrad = [&](const float* dp1, const uint8_t* a1s, const float* img) {
    pipelined<C1Set>(
        0, (H1 * H1 / 4 - wave + NW - 1) / NW,
        [&](int m, C1Set& c) {
          const int p = (wave + NW * m) * 4 + kq, y = p / H1, x = p - y * H1;
          const int w = (y >> 1) * Q1 + (x >> 1);
          c.pos = ((y & 1) << 1) | (x & 1);
          c.a1 = a1s[i * DPS + w];
          c.d = dp1[i * DPS + w];
          const float* im = img + y * IMS + x;
          c.b0 = im[toff0];
          c.b1 = im[toff1];
        },
        [&](const C1Set& c) {
          const float a = (c.a1 & 3) == c.pos ? c.d : 0.f;
          c1acc[0] = mfma(a, c.b0, c1acc[0]);
          c1acc[1] = mfma(a, one1 ? 1.f : c.b1, c1acc[1]);
        });
  };

  for (int s = 0; s < ns; ++s) {
    float* dp1 = dp1b + (s & 1) * C1 * DPS;
    // ---- stage the sample loaded during the previous one (dC2 split with its own power-of-two scale); then issue
    //      the next sample's loads, which complete behind this sample's MFMA work (one workgroup per CU)
    float mx = smax[0];
#pragma unroll
    for (int w = 1; w < NW; ++w) mx = fmaxf(mx, smax[w]);
    const float scale = dc_scale(mx), inv = 1.f / scale, dinv = inv * (1.f / SW2);
    st.store(dch, scale, p1h, a1sb + (s & 1) * C1 * DPS, imgb + (s & 1) * IMGP * IMS, tid);
    if (s + 1 < ns) st.load((size_t)k * B + s0 + s + 1, X, pool1, am1, pool2, am2, dP2, tid);
    __syncthreads();   // staged sample visible; the previous sample's dp1 complete

    // ---- conv2 wgrad (accumulates over the workgroup's samples, fp16 pipe)
    {
      const float rs = scale / wscale;   // exact: both powers of two
#pragma unroll
      for (int j = 0; j < 7; ++j) wacc[j] *= rs;
      wscale = scale;
    }
    const uint8_t* a1cur = a1sb + (s & 1) * C1 * DPS;
    if (wave < 4) bwd_wgrad2<7>((const char*)dcr, (const char*)p1r, wmt, nt0, kq, i >> 2, i & 3, wacc);
    else bwd_wgrad2<6>((const char*)dcr, (const char*)p1r, wmt, nt0, kq, i >> 2, i & 3, wacc);

    // ---- conv2 dgrad -> dp1 (fp16 pipe, 3-term split)
    if (wave < 4) {
      const int mt0 = 2 * wave;
      const int apos[2] = {q14(dg_pix(mt0 * 16 + i)) + 4 * P1P + 4, q14(dg_pix(mt0 * 16 + 16 + i)) + 4 * P1P + 4};
      f4 acc[2] = {};
      bwd_dgrad2<2>(dcr, apos, dgw2, kq, 0, 25, acc);
      bwd_dp1_store(dp1, a1cur, mt0, acc[0] * dinv, i, kq);
      bwd_dp1_store(dp1, a1cur, mt0 + 1, acc[1] * dinv, i, kq);
    } else {
      const int mt = 4 + wave;
      const int apos[1] = {q14(dg_pix(mt * 16 + i)) + 4 * P1P + 4};
      f4 acc[1] = {};
      bwd_dgrad2<1>(dcr, apos, dgw2, kq, 0, 25, acc);
      bwd_dp1_store(dp1, a1cur, mt, acc[0] * dinv, i, kq);
      // m-tile 12: rows 192..195 valid (rows past 195 read a clamped in-range row and are dropped)
      const int w4 = wave - 4;
      const int apos12[1] = {q14(dg_pix(192 + i)) + 4 * P1P + 4};
      f4 acc12[1] = {};
      bwd_dgrad2<1>(dcr, apos12, dgw2, kq, w4 == 0 ? 0 : 1 + 6 * w4, 7 + 6 * w4, acc12);
      if (kq == 0) {
#pragma unroll
        for (int r = 0; r < 4; ++r) red12[w4 * 64 + r * 16 + i] = acc12[0][r] * dinv;
      }
    }

    // ---- conv1 wgrad of the previous sample (its buffers are not touched by this sample)
    if (s > 0) conv1_wgrad(dp1b + ((s - 1) & 1) * C1 * DPS, a1sb + ((s - 1) & 1) * C1 * DPS,
                           imgb + ((s - 1) & 1) * IMGP * IMS);

    // m-tile 12 partials in fixed wave order -> dp1 rows 192..195.  The ReLU mask is read before the barrier:
    // after it the other waves may already restage the pool1 records for the next sample.
    const int r12 = tid >> 4, ci12 = tid & 15;
    const int p12 = dg_pix(192 + r12);
    const bool m12 = tid < 64 && (a1cur[ci12 * DPS + p12] & 0x80);
    if (s + 1 < ns) {   // the next sample's split scale (its loads have landed behind this sample's work)
      const float m = wave_max(st.maxabs(tid));
      if (lane == 0) smax[wave] = m;
    }
    __syncthreads();
    if (tid < 64) {
      const float v = ((red12[tid] + red12[64 + tid]) + red12[128 + tid]) + red12[192 + tid];
      dp1[ci12 * DPS + p12] = m12 ? v : 0.f;
    }
  }
  __syncthreads();   // the last sample's dp1 rows 192..195
  if (ns > 0) conv1_wgrad(dp1b + ((ns - 1) & 1) * C1 * DPS, a1sb + ((ns - 1) & 1) * C1 * DPS,
                          imgb + ((ns - 1) & 1) * IMGP * IMS);
  __syncthreads();   // red aliases the dC2 records

  // ---- write partials (fixed order: deterministic)
  {
    const float us = 1.f / wscale;
#pragma unroll
    for (int j = 0; j < 7; ++j) wacc[j] *= us;
  }
  float* out = part + (size_t)blockIdx.x * PART;
  const int nj = wave < 4 ? 7 : 6;
#pragma unroll
  for (int j = 0; j < 7; ++j) {
    const int nt = nt0 + j;
    if (j < nj) {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int o = wmt * 16 + 4 * kq + r;
        if (nt < 25) out[o * K2 + i * 25 + nt] = wacc[j][r];
        else if (i == 0) out[C2 * K2 + o] = wacc[j][r];
      }
    }
  }
#pragma unroll
  for (int h = 0; h < 2; ++h)
#pragma unroll
    for (int r = 0; r < 4; ++r) red[(wave * 2 + h) * 256 + (4 * kq + r) * 16 + i] = c1acc[h][r];
  __syncthreads();
  for (int e = tid; e < C1 * (K1 + 1); e += NT) {   // taps 0..24 -> dW1, tap 25 (ones) -> db1
    const int o = e / (K1 + 1), tap = e - o * (K1 + 1), h = tap >> 4, j = tap & 15;
    float sacc = 0.f;
    for (int w = 0; w < NW; ++w) sacc += red[(w * 2 + h) * 256 + o * 16 + j];
    if (tap < K1) out[C2 * K2 + C2 + o * K1 + tap] = sacc;
    else out[C2 * K2 + C2 + C1 * K1 + o] = sacc;
  }
}

// grad[k][dst(e)] = sum_g part[k*G + g][e]   (fixed order over groups), into the gradient sink
__global__ void cnn_reduce(const float* __restrict__ part, int G, CnnSgd sg, int P, CnnOff off) {
  const int k = blockIdx.y;
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= PART) return;
  float sacc = 0.f;
  for (int g = 0; g < G; ++g) sacc += part[((size_t)k * G + g) * PART + e];
  int dst;
  if (e < C2 * K2) dst = off.w2 + e;
  else if (e < C2 * K2 + C2) dst = off.b2 + (e - C2 * K2);
  else if (e < C2 * K2 + C2 + C1 * K1) dst = off.w1 + (e - C2 * K2 - C2);
  else dst = off.b1 + (e - C2 * K2 - C2 - C1 * K1);
  sink_put(sg, P, k, dst, sacc);
}

// --------------------------------------------------------------------------------------------
// fc head, one block per client: h1 = sum of the cnn_fc1_fwd partials (fixed order) + b1; a = ReLU(h1) * dropout;
// logits = W a + b; weighted CE; backward:
// dh1 = (W^T dlogits) * dropout * [h1 > 0]; fc2 grads.  Samples go through LDS in chunks of HB; every
// stage spreads (sample, class) or (sample, unit) pairs over the block, and all sums over samples run in
// a fixed order (deterministic).
// --------------------------------------------------------------------------------------------
constexpr int HID = 64, CMAXC = 16, HB = 64;
constexpr int F1IN = C2 * Q2 * Q2;   // 1568 fc1 inputs
constexpr int FC_KS = 7, FC_KC = F1IN / FC_KS, FC_T16 = FC_KC / 16;   // fc1 split: 224 inputs, 14 x 16 per chunk
static_assert(FC_KC * FC_KS == F1IN && FC_T16 * 16 == FC_KC, "fc1 split");
typedef float f4u __attribute__((ext_vector_type(4), aligned(4)));   // client parameter rows are only 4-B aligned
constexpr int HG = (CMAXC * HID + CMAXC + 255) / 256;   // fc2 gradient entries per thread

// Dropout: either a [K*B, 64] mask, or (mask == nullptr) the client's keyed Philox uniforms u (element b*64 + j of
// stream drop_stream, tinycnn.dropout_masks' exact values) kept x drop_scale where u >= drop_p - generated here
// instead of by a uniforms kernel and elementwise launches.
__global__ void __launch_bounds__(256) cnn_head(const float* __restrict__ h1, int off_b1,
                                                const float* __restrict__ mask, const long long* __restrict__ dkeys,
                                                unsigned drop_stream, float drop_p, float drop_scale,
                                                const float* __restrict__ params, long pstride, int P, int off_w,
                                                int off_b, int C, int B, const long long* __restrict__ y,
                                                const float* __restrict__ wts, float* __restrict__ dh1,
                                                float* __restrict__ dlog, float* __restrict__ loss,
                                                float* __restrict__ correct, CnnSgd sg) {
  __shared__ float Ws[CMAXC * HID];
  __shared__ float bs[CMAXC];
  __shared__ float b1s[HID];               // fc1 bias
  __shared__ float hv[HB][HID + 1];        // h1, then dh1 (fc1 bias gradient)
  __shared__ float act[HB][HID + 1];       // ReLU(h1) * dropout of the chunk
  __shared__ float dl[HB][CMAXC + 1];      // logits, then weighted dlogits
  __shared__ float lsb[HB], csb[HB];       // per-sample weighted loss / correct flag
  const int k = blockIdx.x, tid = threadIdx.x;
  const float* prow = params + (size_t)k * pstride;
  for (int e = tid; e < C * HID; e += 256) Ws[e] = prow[off_w + e];
  if (tid < C) bs[tid] = prow[off_b + tid];
  if (tid < HID) b1s[tid] = prow[off_b1 + tid];
  float gacc[HG];
#pragma unroll
  for (int m = 0; m < HG; ++m) gacc[m] = 0.f;
  float lsum = 0.f, csum = 0.f, db1 = 0.f;
  for (int b0 = 0; b0 < B; b0 += HB) {
    const int nb = min(HB, B - b0);
    const size_t sb = (size_t)k * B + b0;
    __syncthreads();   // previous chunk fully consumed (and Ws / bs staged)
    for (int e = tid; e < nb * HID; e += 256) {
      const int b = e / HID, j = e - b * HID;
      float h = 0.f;                           // the FC_KS fc1 partials in fixed order, then the bias
#pragma unroll
      for (int g = 0; g < FC_KS; ++g) h += h1[(((size_t)k * FC_KS + g) * B + b0 + b) * HID + j];
      h += b1s[j];
      hv[b][j] = h;
      const float mk = mask ? mask[sb * HID + e]
                            : (philox_uniform_at((uint64_t)(b0 * HID + e), (uint32_t)dkeys[2 * k],
                                                 (uint32_t)dkeys[2 * k + 1], drop_stream) >= drop_p ? drop_scale : 0.f);
      act[b][j] = fmaxf(h, 0.f) * mk;
    }
    __syncthreads();
    for (int e = tid; e < nb * C; e += 256) {
      const int b = e / C, c = e - b * C;
      float t = bs[c];
#pragma unroll 16
      for (int j = 0; j < HID; ++j) t = fmaf(Ws[c * HID + j], act[b][j], t);
      dl[b][c] = t;
    }
    __syncthreads();
    if (tid < nb) {   // one thread per sample: log-softmax, CE, argmax, dlogits
      const int b = tid;
      float m = -INFINITY;
      int am = 0;
      for (int c = 0; c < C; ++c) {
        m = fmaxf(m, dl[b][c]);
        if (dl[b][c] > dl[b][am]) am = c;
      }
      float se = 0.f;
      for (int c = 0; c < C; ++c) se += expf(dl[b][c] - m);
      const float lse = m + logf(se);
      const int yy = (int)y[sb + b];
      const float ws = wts[sb + b];
      lsb[b] = ws * (lse - dl[b][yy]);
      csb[b] = (am == yy && ws > 0.f) ? 1.f : 0.f;
      for (int c = 0; c < C; ++c) {
        const float d = (expf(dl[b][c] - lse) - (c == yy ? 1.f : 0.f)) * ws;
        dl[b][c] = d;
        dlog[(sb + b) * CMAXC + c] = d;
      }
    }
    __syncthreads();
    for (int e = tid; e < nb * HID; e += 256) {   // dh1 (kept in hv for the fc1 bias gradient)
      const int b = e / HID, j = e - b * HID;
      float d = 0.f;
      for (int c = 0; c < C; ++c) d = fmaf(Ws[c * HID + j], dl[b][c], d);
      if (mask)
        d = hv[b][j] > 0.f ? d * mask[sb * HID + e] : 0.f;
      else   // keyed mask values are 0 or drop_scale: kept with h1 > 0 exactly where act > 0
        d = act[b][j] > 0.f ? d * drop_scale : 0.f;
      dh1[sb * HID + e] = d;
      hv[b][j] = d;
    }
#pragma unroll
    for (int m = 0; m < HG; ++m) {   // fc2 grads: dW[c][j] += sum_b dl[b][c] a[b][j], db[c] += sum_b dl[b][c]
      const int e = tid + m * 256;
      if (e < C * HID) {
        const int c = e / HID, j = e - c * HID;
        for (int b = 0; b < nb; ++b) gacc[m] = fmaf(dl[b][c], act[b][j], gacc[m]);
      } else if (e < C * HID + C) {
        const int c = e - C * HID;
        for (int b = 0; b < nb; ++b) gacc[m] += dl[b][c];
      }
    }
    if (tid == 0)
      for (int b = 0; b < nb; ++b) { lsum += lsb[b]; csum += csb[b]; }
    __syncthreads();
    if (tid < HID)   // fc1 bias gradient: sum over samples of dh1 (fixed order)
      for (int b = 0; b < nb; ++b) db1 += hv[b][tid];
  }
  // the fc2 weights / biases and the fc1 bias were staged in LDS before the chunk loop: an in-place SGD step of the
  // same row (sg.pin == params) cannot race this block's reads
  if (tid < HID) sink_put(sg, P, k, off_b1 + tid, db1);
#pragma unroll
  for (int m = 0; m < HG; ++m) {
    const int e = tid + m * 256;
    if (e < C * HID) sink_put(sg, P, k, off_w + e, gacc[m]);
    else if (e < C * HID + C) sink_put(sg, P, k, off_b + (e - C * HID), gacc[m]);
  }
  if (tid == 0) {
    loss[k] = lsum;
    correct[k] = csum;
    if (sg.pout) sg.t_out[k] = sg.t_in[k] + sg.act[k];
  }
}

// --------------------------------------------------------------------------------------------
// fc1 weight gradient written straight into the parameter-gradient rows:
//   grad[k][off_w1 + j*1568 + c] = sum_s dh1[k,s][j] pool2[k,s][c]
// grid (64-column tile, client): M = 64 units (one m-tile per wave), N = 64 columns (4 n-tiles), K = the client's
// samples in chunks of 32; operands come straight from global (dh1 rows stay in L2, each pool2 tile is read once),
// all 40 loads of a chunk in flight before its MFMAs.  Bandwidth-bound: pool2 read + gradient write once.
// --------------------------------------------------------------------------------------------
__global__ void __launch_bounds__(256) cnn_fc1_wgrad(const float* __restrict__ dh1, const float* __restrict__ pool2,
                                                     int B, CnnSgd sg, int P, int off_w1) {
  const int k = blockIdx.y, c0 = blockIdx.x * 64;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int i = lane & 15, kq = lane >> 4;
  const float* dh = dh1 + (size_t)k * B * HID + wave * 16 + i;
  const float* p2 = pool2 + (size_t)k * B * F1IN + c0 + i;
  f4 acc[4] = {f4{0.f, 0.f, 0.f, 0.f}, f4{0.f, 0.f, 0.f, 0.f}, f4{0.f, 0.f, 0.f, 0.f}, f4{0.f, 0.f, 0.f, 0.f}};
  for (int s0 = 0; s0 < B; s0 += 32) {
    float a[8], b[8][4];
#pragma unroll
    for (int ks = 0; ks < 8; ++ks) {
      const int s = s0 + ks * 4 + kq;
      const bool ok = s < B;
      a[ks] = ok ? dh[(size_t)s * HID] : 0.f;
#pragma unroll
      for (int nt = 0; nt < 4; ++nt)
        b[ks][nt] = (ok && c0 + nt * 16 + i < F1IN) ? p2[(size_t)s * F1IN + nt * 16] : 0.f;
    }
    // transposed product (pool2 as the A operand): lane (i, kq) accumulates dW[unit wave * 16 + i][4 kq .. 4 kq + 3 of
    // n-tile nt], four consecutive row entries - one 16-byte sink access instead of four 4-byte ones
#pragma unroll
    for (int ks = 0; ks < 8; ++ks)
#pragma unroll
      for (int nt = 0; nt < 4; ++nt) acc[nt] = mfma(b[ks][nt], a[ks], acc[nt]);
  }
  const long e0 = off_w1 + (long)(wave * 16 + i) * F1IN + c0 + 4 * kq;
#pragma unroll
  for (int nt = 0; nt < 4; ++nt)
    if (c0 + nt * 16 < F1IN)          // F1IN % 16 == 0: a 16-column tile is all in range or all out
      sink_put4(sg, P, k, e0 + nt * 16, acc[nt]);
}

// --------------------------------------------------------------------------------------------
// fc1 forward, split over the inputs:  h1p[k][g][s][j] = sum_{c in chunk g} pool2[k][s][c] W1[k][j][c]
// grid (sample tile of 32, client, chunk g < FC_KS): 4 waves, wave w owns units 16w .. 16w + 15 (one n-tile) of
// two m-tiles (32 samples).  K order: MFMA step 4T + u, lane group kq <-> input c = g FC_KC + 16 T + 4 kq + u, so
// one 16-byte load per lane feeds four steps (A: a pool2 row, B: a W1 row, both contiguous in c) and the 64 lanes
// of a load read 16 rows x 64 contiguous bytes.  The next T's loads are in flight during this T's MFMAs.  The
// FC_KS partial sums are added in fixed order by the consumer (cnn_head / cnn_eval_head), so a client's h1 never
// depends on how many clients share the launch (unlike a library batched GEMM, whose algorithm and split-K change
// with the batch count).
// --------------------------------------------------------------------------------------------
__global__ void __launch_bounds__(256) cnn_fc1_fwd(const float* __restrict__ pool2, const float* __restrict__ params,
                                                   int P, int off_w1, int B, float* __restrict__ h1p) {
  const int s0 = blockIdx.x * 32, k = blockIdx.y, g = blockIdx.z;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int i = lane & 15, kq = lane >> 4;
  const int cb = g * FC_KC + 4 * kq;
  const bool ok0 = s0 + i < B, ok1 = s0 + 16 + i < B;
  const f4u* a0 = (const f4u*)(pool2 + ((size_t)k * B + (ok0 ? s0 + i : 0)) * F1IN + cb);
  const f4u* a1 = (const f4u*)(pool2 + ((size_t)k * B + (ok1 ? s0 + 16 + i : 0)) * F1IN + cb);
  const f4u* bw = (const f4u*)(params + (size_t)k * P + off_w1 + (size_t)(wave * 16 + i) * F1IN + cb);
  const f4u zero = {0.f, 0.f, 0.f, 0.f};
  f4 acc0 = {0.f, 0.f, 0.f, 0.f}, acc1 = {0.f, 0.f, 0.f, 0.f};
  f4u x0 = ok0 ? a0[0] : zero, x1 = ok1 ? a1[0] : zero, w = bw[0];
#pragma unroll
  for (int T = 0; T < FC_T16; ++T) {
    f4u nx0 = zero, nx1 = zero, nw = zero;
    if (T + 1 < FC_T16) {                         // 16 inputs ahead = 4 float4
      nx0 = ok0 ? a0[4 * (T + 1)] : zero;
      nx1 = ok1 ? a1[4 * (T + 1)] : zero;
      nw = bw[4 * (T + 1)];
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      acc0 = mfma(x0[u], w[u], acc0);
      acc1 = mfma(x1[u], w[u], acc1);
    }
    x0 = nx0;
    x1 = nx1;
    w = nw;
  }
  float* out = h1p + (((size_t)k * FC_KS + g) * B) * HID + wave * 16 + i;
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int sa = s0 + 4 * kq + r, sb = s0 + 16 + 4 * kq + r;
    if (sa < B) out[(size_t)sa * HID] = acc0[r];
    if (sb < B) out[(size_t)sb * HID] = acc1[r];
  }
}

// --------------------------------------------------------------------------------------------
// fc1 input gradient:  dP2[k][s][c] = sum_j dh1[k][s][j] W1[k][j][c]
// grid (256-input chunk, client, sample tile of 32): wave w owns inputs cw = c0 + 64 w + [0, 64) as four n-tiles
// whose columns interleave (n-tile q, lane i <-> input cw + 4 i + q), so ONE 16-byte W1 load per lane holds the B
// operand of all four n-tiles at one unit j, and a load's 64 lanes read 4 rows x 256 contiguous bytes.  K order:
// step 4T + u, lane group kq <-> unit j = 16 T + 4 kq + u (dh1 rows: one 16-byte load per lane feeds four steps).
// The four n-tiles of an accumulator row are four consecutive inputs: one 16-byte store.
// --------------------------------------------------------------------------------------------
__global__ void __launch_bounds__(256) cnn_fc1_dgrad(const float* __restrict__ dh1, const float* __restrict__ params,
                                                     int P, int off_w1, int B, float* __restrict__ dP2) {
  const int c0 = blockIdx.x * 256, k = blockIdx.y, s0 = blockIdx.z * 32;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int i = lane & 15, kq = lane >> 4;
  const int cc = c0 + 64 * wave + 4 * i;                 // this lane's 4 consecutive inputs
  const bool okc = cc < F1IN;                            // F1IN % 4 == 0: all four or none
  const bool ok0 = s0 + i < B, ok1 = s0 + 16 + i < B;
  const f4u* d0 = (const f4u*)(dh1 + ((size_t)k * B + (ok0 ? s0 + i : 0)) * HID + 4 * kq);
  const f4u* d1 = (const f4u*)(dh1 + ((size_t)k * B + (ok1 ? s0 + 16 + i : 0)) * HID + 4 * kq);
  const float* w = params + (size_t)k * P + off_w1 + (okc ? cc : 0);
  const f4u zero = {0.f, 0.f, 0.f, 0.f};
  f4u x0[4], x1[4];
#pragma unroll
  for (int T = 0; T < 4; ++T) {
    x0[T] = ok0 ? d0[4 * T] : zero;
    x1[T] = ok1 ? d1[4 * T] : zero;
  }
  f4 acc[2][4];
#pragma unroll
  for (int m = 0; m < 2; ++m)
#pragma unroll
    for (int q = 0; q < 4; ++q) acc[m][q] = f4{0.f, 0.f, 0.f, 0.f};
  auto wrow = [&](int T, int u) -> f4u {
    return okc ? *(const f4u*)(w + (size_t)(16 * T + 4 * kq + u) * F1IN) : zero;
  };
  f4u wv[4];
#pragma unroll
  for (int u = 0; u < 4; ++u) wv[u] = wrow(0, u);
#pragma unroll
  for (int T = 0; T < 4; ++T) {
    f4u nw[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) nw[u] = T + 1 < 4 ? wrow(T + 1, u) : zero;
#pragma unroll
    for (int u = 0; u < 4; ++u)
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        acc[0][q] = mfma(x0[T][u], wv[u][q], acc[0][q]);
        acc[1][q] = mfma(x1[T][u], wv[u][q], acc[1][q]);
      }
#pragma unroll
    for (int u = 0; u < 4; ++u) wv[u] = nw[u];
  }
  if (!okc) return;
#pragma unroll
  for (int m = 0; m < 2; ++m)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int sm = s0 + 16 * m + 4 * kq + r;
      if (sm < B) {
        const f4 v = {acc[m][0][r], acc[m][1][r], acc[m][2][r], acc[m][3][r]};
        *(f4*)(dP2 + ((size_t)k * B + sm) * F1IN + cc) = v;
      }
    }
}

// --------------------------------------------------------------------------------------------
// Evaluation head (reference evaluate_model, Classical_FL.py:83-102): h1 = sum of the FC_KS fc1 partials (fixed
// order) + b1, ReLU (no dropout), logits = W2 h1 + b2 -> logits [K * B, C]; with labels, per-block fixed-order
// sums of the cross-entropy and of the argmax hits -> stats[block] = (loss_sum, correct) in float64.
// grid (sample tile of 64, client), 256 threads: thread (sample, class) pairs for the logits, one thread per sample
// for the softmax / argmax (first maximum, as torch.argmax).
// --------------------------------------------------------------------------------------------
__global__ void __launch_bounds__(256) cnn_eval_head(const float* __restrict__ h1p, const float* __restrict__ params,
                                                     int P, int off_b1, int off_w, int off_b, int C, int B,
                                                     const long long* __restrict__ y, float* __restrict__ logits,
                                                     double* __restrict__ stats) {
  __shared__ float Ws[CMAXC * HID];
  __shared__ float bs[CMAXC], b1s[HID];
  __shared__ float act[HB][HID + 1];
  __shared__ float dl[HB][CMAXC + 1];
  __shared__ double ls[HB], cs[HB];
  const int s0 = blockIdx.x * HB, k = blockIdx.y, tid = threadIdx.x;
  const int nb = min(HB, B - s0);
  const float* prow = params + (size_t)k * P;
  for (int e = tid; e < C * HID; e += 256) Ws[e] = prow[off_w + e];
  if (tid < C) bs[tid] = prow[off_b + tid];
  if (tid < HID) b1s[tid] = prow[off_b1 + tid];
  __syncthreads();
  for (int e = tid; e < nb * HID; e += 256) {
    const int b = e / HID, j = e - b * HID;
    float h = 0.f;
#pragma unroll
    for (int g = 0; g < FC_KS; ++g) h += h1p[(((size_t)k * FC_KS + g) * B + s0 + b) * HID + j];
    act[b][j] = fmaxf(h + b1s[j], 0.f);
  }
  __syncthreads();
  for (int e = tid; e < nb * C; e += 256) {
    const int b = e / C, c = e - b * C;
    float t = bs[c];
#pragma unroll 16
    for (int j = 0; j < HID; ++j) t = fmaf(Ws[c * HID + j], act[b][j], t);
    dl[b][c] = t;
    logits[((size_t)k * B + s0 + b) * C + c] = t;
  }
  __syncthreads();
  if (!y) return;
  if (tid < HB) {
    double l = 0.0, h = 0.0;
    if (tid < nb) {
      const int b = tid;
      float m = -INFINITY;
      int am = 0;
      for (int c = 0; c < C; ++c) {
        m = fmaxf(m, dl[b][c]);
        if (dl[b][c] > dl[b][am]) am = c;
      }
      float se = 0.f;
      for (int c = 0; c < C; ++c) se += expf(dl[b][c] - m);
      const int yy = (int)y[(size_t)k * B + s0 + b];
      l = (double)(m + logf(se) - dl[b][yy]);
      h = am == yy ? 1.0 : 0.0;
    }
    ls[tid] = l;
    cs[tid] = h;
  }
  __syncthreads();
  if (tid == 0) {
    double l = 0.0, h = 0.0;
    for (int b = 0; b < nb; ++b) {
      l += ls[b];
      h += cs[b];
    }
    const size_t blk = (size_t)k * gridDim.x + blockIdx.x;
    stats[2 * blk] = l;
    stats[2 * blk + 1] = h;
  }
}

size_t fwd_lds() { return (size_t)FWD_LDS; }
constexpr int BWD_LDS = (C1 * W2B + NPOS * DRQ + NPOS * PRQ) * 16 + (2 * C1 * DPS + 2 * IMGP * IMS + 256 + 8) * 4 +
                        2 * C1 * DPS;
static_assert(BWD_LDS <= 160 * 1024, "cnn_bwd LDS");
static_assert(NW * 2 * 256 * 4 <= NPOS * DRQ * 16, "conv1 wgrad partials alias the dC2 records");
size_t bwd_lds() { return (size_t)BWD_LDS; }

}  // namespace cnn
}  // namespace qfx

using namespace qfx::cnn;

extern "C" int qfx_cnn_mfma_probe(const float* A, const float* B, float* D, int K, hipStream_t st) {
  hipLaunchKernelGGL(mfma_probe, dim3(1), dim3(64), 0, st, A, B, D, K);
  return (int)hipGetLastError();
}

extern "C" int qfx_cnn_forward(const float* X, const float* params, int P, int K, int B, const int* off4, float* pool1,
                               uint8_t* am1, float* pool2, uint8_t* am2, hipStream_t st) {
  const int G = (B + FSG - 1) / FSG;
  const CnnOff off{off4[0], off4[1], off4[2], off4[3]};
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute((const void*)cnn_fwd, hipFuncAttributeMaxDynamicSharedMemorySize, (int)fwd_lds());
    attr = true;
  }
  hipLaunchKernelGGL(cnn_fwd, dim3(K * G), dim3(NT), fwd_lds(), st, X, params, P, B, G, off, pool1, am1, pool2, am2);
  return (int)hipGetLastError();
}

// Samples per backward workgroup: a function of the client batch B ONLY (half of it, a power of two, at most
// BS_MAX: B = 32 -> 16, two workgroups per client).  The workgroup accumulates its samples' weight gradients in MFMA registers and cnn_reduce
// sums the per-workgroup partials in fixed order, so the grouping fixes the fp32 summation order: choosing
// it from the per-rank client count or the CU count (as round 2 did) made a client's gradient depend on how
// many clients share its rank, breaking the bitwise rank-count invariance of the federated result.
static int bwd_bs(int /*K*/, int B) {
  int bs = 1;
  while (bs * 2 <= BS_MAX && bs * 2 * 2 <= B) bs *= 2;
  return bs;
}

// params: read rows with stride pstride (0: every client reads theta); gradients (row stride P) into the sink
extern "C" int qfx_cnn_backward(const float* X, const float* params, int pstride, int P, int K, int B,
                                const int* off4, const float* pool1, const uint8_t* am1, const float* pool2,
                                const uint8_t* am2, const float* dP2, float* part, const CnnSgd* sink,
                                hipStream_t st) {
  const int bs = bwd_bs(K, B), G = (B + bs - 1) / bs;
  const CnnOff off{off4[0], off4[1], off4[2], off4[3]};
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute((const void*)cnn_bwd, hipFuncAttributeMaxDynamicSharedMemorySize, (int)bwd_lds());
    attr = true;
  }
  hipLaunchKernelGGL(cnn_bwd, dim3(K * G), dim3(NT), bwd_lds(), st, X, params, pstride, B, G, off, pool1, am1, pool2,
                     am2, dP2, bs, part);
  hipLaunchKernelGGL(cnn_reduce, dim3((PART + 255) / 256, K), dim3(256), 0, st, part, G, *sink, P, off);
  return (int)hipGetLastError();
}

extern "C" int qfx_cnn_head(const float* h1, int off_b1, const float* mask, const long long* dkeys,
                            unsigned drop_stream, float drop_p, float drop_scale, const float* params, int pstride,
                            int P, int off_w, int off_b, int C, int K, int B, const long long* y, const float* wts,
                            float* dh1, float* dlog, float* loss, float* correct, const CnnSgd* sink, hipStream_t st) {
  if (C > CMAXC) return -2;
  if (!mask && !dkeys) return -3;
  hipLaunchKernelGGL(cnn_head, dim3(K), dim3(256), 0, st, h1, off_b1, mask, dkeys, drop_stream, drop_p, drop_scale,
                     params, (long)pstride, P, off_w, off_b, C, B, y, wts, dh1, dlog, loss, correct, *sink);
  return (int)hipGetLastError();
}

extern "C" int qfx_cnn_fc1_wgrad(const float* dh1, const float* pool2, int K, int B, const CnnSgd* sink, int P,
                                 int off_w1, hipStream_t st) {
  if (K <= 0 || B <= 0) return 0;
  hipLaunchKernelGGL(cnn_fc1_wgrad, dim3((F1IN + 63) / 64, K), dim3(256), 0, st, dh1, pool2, B, *sink, P, off_w1);
  return (int)hipGetLastError();
}

extern "C" int qfx_cnn_partial_size() { return PART; }
extern "C" int qfx_cnn_bwd_groups(int K, int B) {
  const int bs = bwd_bs(K, B);
  return (B + bs - 1) / bs;
}

extern "C" int qfx_cnn_fc1_forward(const float* pool2, const float* params, int P, int off_w1, int K, int B, float* h1p,
                                   hipStream_t st) {
  if (K <= 0 || B <= 0) return 0;
  hipLaunchKernelGGL(cnn_fc1_fwd, dim3((B + 31) / 32, K, FC_KS), dim3(256), 0, st, pool2, params, P, off_w1, B, h1p);
  return (int)hipGetLastError();
}

extern "C" int qfx_cnn_fc1_dgrad(const float* dh1, const float* params, int P, int off_w1, int K, int B, float* dP2,
                                 hipStream_t st) {
  if (K <= 0 || B <= 0) return 0;
  hipLaunchKernelGGL(cnn_fc1_dgrad, dim3((F1IN + 255) / 256, K, (B + 31) / 32), dim3(256), 0, st, dh1, params, P,
                     off_w1, B, dP2);
  return (int)hipGetLastError();
}

extern "C" int qfx_cnn_eval_head(const float* h1p, const float* params, int P, int off_b1, int off_w, int off_b, int C,
                                 int K, int B, const long long* y, float* logits, double* stats, hipStream_t st) {
  if (C > CMAXC) return -2;
  if (K <= 0 || B <= 0) return 0;
  hipLaunchKernelGGL(cnn_eval_head, dim3((B + HB - 1) / HB, K), dim3(256), 0, st, h1p, params, P, off_b1, off_w, off_b,
                     C, B, y, logits, stats);
  return (int)hipGetLastError();
}

extern "C" int qfx_cnn_fc1_splits() { return FC_KS; }
extern "C" int qfx_cnn_eval_blocks(int B) { return (B + HB - 1) / HB; }
