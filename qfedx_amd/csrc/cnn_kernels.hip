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
constexpr int W2S = 401;           // LDS row stride of W2 [32][400] (odd: conflict-free B fetches)
constexpr int FSG = 2;             // samples per forward workgroup

struct CnnOff {                    // float offsets of the tensors inside one client's parameter row
  int w1, b1, w2, b2;
};

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
// forward: conv1 -> ReLU -> pool -> conv2 -> ReLU -> pool for FSG samples of one client
//   outputs per sample: pool1 [16][196], am1 [16][196] (argmax 0..3), pool2 [32][49], am2 [32][49]
// --------------------------------------------------------------------------------------------
__global__ void __launch_bounds__(NT) cnn_fwd(const float* __restrict__ X, const float* __restrict__ params,
                                              int P, int B, int G, CnnOff off, float* __restrict__ pool1,
                                              uint8_t* __restrict__ am1, float* __restrict__ pool2,
                                              uint8_t* __restrict__ am2) {
  extern __shared__ __attribute__((aligned(16))) float sm[];
  float* w2s = sm;                          // [32][401]
  float* w1s = w2s + C2 * W2S;              // [16][28]  (k >= 25 zero)
  float* b1s = w1s + C1 * K1P;              // [16]
  float* b2s = b1s + C1;                    // [32]
  int* koff2 = reinterpret_cast<int*>(b2s + C2);   // [400] (ci,dy,dx) -> offset in padded pool1
  int* koff1 = koff2 + K2;                  // [28]  (dy,dx) -> offset in padded image
  float* img = reinterpret_cast<float*>(koff1 + K1P);   // [FSG][32*32]
  float* p1s = img + FSG * IMGP * IMGP;     // [FSG][16][18*18]

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int k = blockIdx.x / G, g = blockIdx.x - k * G;
  const int s0 = g * FSG;
  const int ns = min(FSG, B - s0);
  const float* prow = params + (size_t)k * P;

  for (int e = tid; e < C2 * K2; e += NT) { const int o = e / K2, kk = e - o * K2; w2s[o * W2S + kk] = prow[off.w2 + e]; }
  for (int e = tid; e < C1 * K1P; e += NT) {
    const int o = e / K1P, kk = e - o * K1P;
    w1s[e] = kk < K1 ? prow[off.w1 + o * K1 + kk] : 0.f;
  }
  if (tid < C1) b1s[tid] = prow[off.b1 + tid];
  if (tid < C2) b2s[tid] = prow[off.b2 + tid];
  for (int kk = tid; kk < K2; kk += NT) {
    const int ci = kk / 25, r = kk - ci * 25;
    koff2[kk] = ci * P1P * P1P + (r / 5) * P1P + (r % 5);
  }
  if (tid < K1P) koff1[tid] = tid < K1 ? (tid / 5) * IMGP + (tid % 5) : 0;
  for (int e = tid; e < FSG * IMGP * IMGP; e += NT) {
    const int s = e / (IMGP * IMGP), r = e - s * IMGP * IMGP, y = r / IMGP - 2, x = r % IMGP - 2;
    img[e] = (s < ns && y >= 0 && y < IMG && x >= 0 && x < IMG) ? X[((size_t)k * B + s0 + s) * IMG * IMG + y * IMG + x] : 0.f;
  }
  for (int e = tid; e < FSG * C1 * P1P * P1P; e += NT) p1s[e] = 0.f;
  __syncthreads();

  // ---- conv1: 49 m-tiles (196 pool windows x 4) per sample, N = 16, K = 28
  const int i = lane & 15, kq = lane >> 4;
  for (int t = wave; t < ns * 49; t += NW) {
    const int s = t / 49, mt = t - s * 49;
    const int w = mt * 4 + (i >> 2), pos = i & 3;
    const int py = 2 * (w / Q1) + (pos >> 1), px = 2 * (w % Q1) + (pos & 1);
    const float* im = img + s * IMGP * IMGP + py * IMGP + px;
    f4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int ks = 0; ks < K1P / 4; ++ks) {
      const int kk = ks * 4 + kq;
      acc = mfma(im[koff1[kk]], w1s[i * K1P + kk], acc);
    }
    // lane holds window wo = mt*4 + kq, its 4 positions, channel o = i
    const int wo = mt * 4 + kq, o = i;
    const float bo = b1s[o];
    float best = fmaxf(acc[0] + bo, 0.f);
    int arg = 0;
#pragma unroll
    for (int r = 1; r < 4; ++r) {
      const float v = fmaxf(acc[r] + bo, 0.f);
      if (v > best) { best = v; arg = r; }
    }
    const size_t so = ((size_t)k * B + s0 + s) * C1 * Q1 * Q1 + o * Q1 * Q1 + wo;
    pool1[so] = best;
    am1[so] = (uint8_t)arg;
    p1s[s * C1 * P1P * P1P + o * P1P * P1P + (wo / Q1 + 2) * P1P + (wo % Q1) + 2] = best;
  }
  __syncthreads();

  // ---- conv2: 13 m-tiles (49 windows x 4, padded to 52) per sample, N = 32 (two n-tiles), K = 400
  for (int t = wave; t < ns * 13; t += NW) {
    const int s = t / 13, mt = t - s * 13;
    const int w = mt * 4 + (i >> 2), pos = i & 3;
    const bool valid = w < Q2 * Q2;
    const int wc = valid ? w : 0;
    const int py = 2 * (wc / Q2) + (pos >> 1), px = 2 * (wc % Q2) + (pos & 1);
    const float* in = p1s + s * C1 * P1P * P1P + py * P1P + px;
    f4 acc0 = {0.f, 0.f, 0.f, 0.f}, acc1 = {0.f, 0.f, 0.f, 0.f};
#pragma unroll 4
    for (int ks = 0; ks < K2 / 4; ++ks) {
      const int kk = ks * 4 + kq;
      const float a = valid ? in[koff2[kk]] : 0.f;
      acc0 = mfma(a, w2s[i * W2S + kk], acc0);
      acc1 = mfma(a, w2s[(16 + i) * W2S + kk], acc1);
    }
    const int wo = mt * 4 + kq;
    if (wo < Q2 * Q2) {
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const f4 acc = h ? acc1 : acc0;
        const int o = h * 16 + i;
        const float bo = b2s[o];
        float best = fmaxf(acc[0] + bo, 0.f);
        int arg = 0;
#pragma unroll
        for (int r = 1; r < 4; ++r) {
          const float v = fmaxf(acc[r] + bo, 0.f);
          if (v > best) { best = v; arg = r; }
        }
        const size_t so = ((size_t)k * B + s0 + s) * C2 * Q2 * Q2 + o * Q2 * Q2 + wo;
        pool2[so] = best;
        am2[so] = (uint8_t)arg;
      }
    }
  }
}

// --------------------------------------------------------------------------------------------
// backward of the conv stack for BS samples of one client -> per-workgroup gradient partials
//   part[(k*G + g)][ dW2 (12800) | db2 (32) | dW1 (400) | db1 (16) ]
// --------------------------------------------------------------------------------------------
constexpr int BS = 4;              // samples per backward workgroup
constexpr int W2T = 801;           // LDS stride of the transposed W2 [16 ci][800 (o,dy,dx)]
constexpr int PART = C2 * K2 + C2 + C1 * K1 + C1;

__global__ void __launch_bounds__(NT) cnn_bwd(const float* __restrict__ X, const float* __restrict__ params,
                                              int P, int B, int G, CnnOff off, const float* __restrict__ pool1,
                                              const uint8_t* __restrict__ am1, const float* __restrict__ pool2,
                                              const uint8_t* __restrict__ am2, const float* __restrict__ dP2,
                                              float* __restrict__ part) {
  extern __shared__ __attribute__((aligned(16))) float sm[];
  float* w2t = sm;                          // [16][801]: w2t[ci][o*25+r] = W2[o][ci][r]
  float* dc2 = w2t + C1 * W2T;              // [32][18*18] padded dL/d conv2-output (post-unpool, ReLU-masked)
  float* p1s = dc2 + C2 * P1P * P1P;        // [16][18*18] padded pool1 (conv2 input)
  float* dp1 = p1s + C1 * P1P * P1P;        // [16][196]   dL/d pool1
  float* img = dp1 + C1 * Q1 * Q1;          // [32*32] padded image
  float* red = img + IMGP * IMGP;           // [8 waves][2 tiles][256]: conv1-wgrad wave partials
  float* bsum = red + NW * 2 * 256;         // [48]: db2 | db1 accumulators
  int* kofT = reinterpret_cast<int*>(bsum + 48);   // [800] (o,dy,dx) -> offset in padded dc2 (dgrad)
  int* kof2 = kofT + 2 * K2;                // [400] (ci,dy,dx) -> offset in padded pool1 (wgrad)
  uint8_t* a1s = reinterpret_cast<uint8_t*>(kof2 + K2);   // [16][196] argmax of pool1

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int k = blockIdx.x / G, g = blockIdx.x - k * G;
  const int s0 = g * BS;
  const int ns = min(BS, B - s0);
  const float* prow = params + (size_t)k * P;
  const int i = lane & 15, kq = lane >> 4;

  for (int e = tid; e < C2 * K2; e += NT) {   // W2 [o][ci][r] -> w2t[ci][o*25 + r]
    const int o = e / K2, rem = e - o * K2, ci = rem / 25, r = rem - ci * 25;
    w2t[ci * W2T + o * 25 + r] = prow[off.w2 + e];
  }
  for (int kk = tid; kk < 2 * K2; kk += NT) {  // dgrad: kk = (o,dy,dx): -o*324 ... taps flipped
    const int o = kk / 25, r = kk - o * 25;
    kofT[kk] = o * P1P * P1P - (r / 5) * P1P - (r % 5);
  }
  for (int kk = tid; kk < K2; kk += NT) {
    const int ci = kk / 25, r = kk - ci * 25;
    kof2[kk] = ci * P1P * P1P + (r / 5) * P1P + (r % 5);
  }
  for (int e = tid; e < C2 * P1P * P1P; e += NT) dc2[e] = 0.f;
  for (int e = tid; e < C1 * P1P * P1P; e += NT) p1s[e] = 0.f;
  for (int e = tid; e < IMGP * IMGP; e += NT) img[e] = 0.f;
  if (tid < 48) bsum[tid] = 0.f;

  // conv2 wgrad accumulators: wave owns m-tile (wave & 1) and n-tiles nt = (wave >> 1) + 4j
  constexpr int NJ = 7;
  f4 wacc[NJ];
#pragma unroll
  for (int j = 0; j < NJ; ++j) wacc[j] = f4{0.f, 0.f, 0.f, 0.f};
  f4 c1acc[2] = {f4{0.f, 0.f, 0.f, 0.f}, f4{0.f, 0.f, 0.f, 0.f}};
  __syncthreads();

  for (int s = 0; s < ns; ++s) {
    const size_t sidx = (size_t)k * B + s0 + s;
    // ---- stage: unpool2 (+ReLU mask) into padded dc2, pool1 -> padded p1s, image, argmax1
    for (int e = tid; e < C2 * H2 * H2; e += NT) {
      const int o = e / (H2 * H2), r = e - o * H2 * H2, y = r / H2, x = r % H2;
      const int w = (y >> 1) * Q2 + (x >> 1), pos = ((y & 1) << 1) | (x & 1);
      const size_t q = sidx * C2 * Q2 * Q2 + o * Q2 * Q2 + w;
      dc2[o * P1P * P1P + (y + 2) * P1P + x + 2] = (am2[q] == pos && pool2[q] > 0.f) ? dP2[q] : 0.f;
    }
    for (int e = tid; e < C1 * Q1 * Q1; e += NT) {
      const int ci = e / (Q1 * Q1), r = e - ci * Q1 * Q1;
      p1s[ci * P1P * P1P + (r / Q1 + 2) * P1P + (r % Q1) + 2] = pool1[sidx * C1 * Q1 * Q1 + e];
      a1s[e] = am1[sidx * C1 * Q1 * Q1 + e];
    }
    for (int e = tid; e < IMG * IMG; e += NT) img[(e / IMG + 2) * IMGP + (e % IMG) + 2] = X[sidx * IMG * IMG + e];
    __syncthreads();
    // db2 += sum over the 14x14 map
    if (tid < C2) {
      float sacc = 0.f;
      for (int y = 0; y < H2; ++y)
        for (int x = 0; x < H2; ++x) sacc += dc2[tid * P1P * P1P + (y + 2) * P1P + x + 2];
      bsum[tid] += sacc;
    }

    // ---- conv2 wgrad: dW2[o][kk] += sum_p dc2[o][p] * pool1pad[p + kof2[kk]]   (M=32, N=400, K=196)
    {
      const int mt = wave & 1;
      const int o = mt * 16 + i;
      for (int ks = 0; ks < 49; ++ks) {
        const int p = ks * 4 + kq, y = p / H2, x = p % H2;
        const float a = dc2[o * P1P * P1P + (y + 2) * P1P + x + 2];
        const float* base = p1s + y * P1P + x;
#pragma unroll
        for (int j = 0; j < NJ; ++j) {
          const int nt = (wave >> 1) + 4 * j;
          if (nt < K2 / 16) wacc[j] = mfma(a, base[kof2[nt * 16 + i]], wacc[j]);
        }
      }
    }

    // ---- conv2 dgrad: dP1[ci][p] = sum_{o,dy,dx} dc2pad[o][p + 4*19 - tap] W2[o][ci][tap]  (M=196, N=16, K=800)
    for (int mt = wave; mt < 13; mt += NW) {
      const int p = mt * 16 + i;
      const bool valid = p < H2 * H2;
      const int pc = valid ? p : 0;
      const float* base = dc2 + (pc / H2 + 4) * P1P + (pc % H2) + 4;
      f4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll 4
      for (int ks = 0; ks < 2 * K2 / 4; ++ks) {
        const int kk = ks * 4 + kq;
        acc = mfma(valid ? base[kofT[kk]] : 0.f, w2t[i * W2T + kk], acc);
      }
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int pr = mt * 16 + 4 * kq + r;
        if (pr < H2 * H2) dp1[i * Q1 * Q1 + pr] = acc[r];
      }
    }
    __syncthreads();
    // db1 += sum of the unpooled (ReLU-masked) dP1
    if (tid < C1) {
      float sacc = 0.f;
      for (int w = 0; w < Q1 * Q1; ++w) {
        const float pv = p1s[tid * P1P * P1P + (w / Q1 + 2) * P1P + (w % Q1) + 2];
        sacc += pv > 0.f ? dp1[tid * Q1 * Q1 + w] : 0.f;
      }
      bsum[C2 + tid] += sacc;
    }

    // ---- conv1 wgrad: dW1[o][kk] += sum_{p in 28x28} dC1[o][p] img[p + tap(kk)]  (M=16, N=25->32, K=784)
    //      dC1 = unpool1(dP1) on the fly; K split across the 8 waves (partials reduced at the end)
    for (int ks = wave; ks < H1 * H1 / 4; ks += NW) {
      const int p = ks * 4 + kq, y = p / H1, x = p % H1;
      const int w = (y >> 1) * Q1 + (x >> 1), pos = ((y & 1) << 1) | (x & 1);
      const int o = i;
      const float pv = p1s[o * P1P * P1P + (w / Q1 + 2) * P1P + (w % Q1) + 2];
      const float a = (a1s[o * Q1 * Q1 + w] == pos && pv > 0.f) ? dp1[o * Q1 * Q1 + w] : 0.f;
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const int tap = h * 16 + i;      // B[kk = p][j = tap]
        const float b = tap < K1 ? img[(y + tap / 5) * IMGP + x + tap % 5] : 0.f;
        c1acc[h] = mfma(a, b, c1acc[h]);
      }
    }
    __syncthreads();   // LDS is restaged for the next sample
  }

  // ---- write partials (fixed order: deterministic)
  float* out = part + (size_t)blockIdx.x * PART;
  {
    const int mt = wave & 1;
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
      const int nt = (wave >> 1) + 4 * j;
      if (nt < K2 / 16) {
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int o = mt * 16 + 4 * kq + r, kk = nt * 16 + i;
          out[o * K2 + kk] = wacc[j][r];
        }
      }
    }
  }
#pragma unroll
  for (int h = 0; h < 2; ++h)
#pragma unroll
    for (int r = 0; r < 4; ++r) red[(wave * 2 + h) * 256 + (4 * kq + r) * 16 + i] = c1acc[h][r];
  __syncthreads();
  for (int e = tid; e < C1 * K1; e += NT) {
    const int o = e / K1, tap = e - o * K1, h = tap >> 4, j = tap & 15;
    float sacc = 0.f;
    for (int w = 0; w < NW; ++w) sacc += red[(w * 2 + h) * 256 + o * 16 + j];
    out[C2 * K2 + C2 + e] = sacc;
  }
  if (tid < C2) out[C2 * K2 + tid] = bsum[tid];
  if (tid < C1) out[C2 * K2 + C2 + C1 * K1 + tid] = bsum[C2 + tid];
}

// grad[k][dst(e)] = sum_g part[k*G + g][e]   (fixed order over groups)
__global__ void cnn_reduce(const float* __restrict__ part, int G, float* __restrict__ grad, int P, CnnOff off) {
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
  grad[(size_t)k * P + dst] = sacc;
}

// --------------------------------------------------------------------------------------------
// fc head, one block per client: a = ReLU(h1) * dropout; logits = W a + b; weighted CE; backward:
// dh1 = (W^T dlogits) * dropout * [h1 > 0]; fc2 grads (fixed-order sums over samples)
// --------------------------------------------------------------------------------------------
constexpr int HID = 64, CMAXC = 16;

__global__ void __launch_bounds__(256) cnn_head(const float* __restrict__ h1, const float* __restrict__ mask,
                                                const float* __restrict__ params, int P, int off_w, int off_b,
                                                int C, int B, const long long* __restrict__ y,
                                                const float* __restrict__ wts, float* __restrict__ dh1,
                                                float* __restrict__ dlog, float* __restrict__ loss,
                                                float* __restrict__ correct, float* __restrict__ grad) {
  __shared__ float Ws[CMAXC * HID];
  __shared__ float bs[CMAXC];
  __shared__ float red[2 * 256];
  const int k = blockIdx.x, tid = threadIdx.x;
  const float* prow = params + (size_t)k * P;
  for (int e = tid; e < C * HID; e += 256) Ws[e] = prow[off_w + e];
  if (tid < C) bs[tid] = prow[off_b + tid];
  __syncthreads();
  float lsum = 0.f, csum = 0.f;
  for (int b = tid; b < B; b += 256) {      // one thread per sample
    const size_t s = (size_t)k * B + b;
    float lg[CMAXC];
    float m = -INFINITY;
    for (int c = 0; c < C; ++c) {
      float t = bs[c];
      for (int j = 0; j < HID; ++j) t = fmaf(Ws[c * HID + j], fmaxf(h1[s * HID + j], 0.f) * mask[s * HID + j], t);
      lg[c] = t;
      m = fmaxf(m, t);
    }
    float se = 0.f;
    int am = 0;
    for (int c = 0; c < C; ++c) {
      se += expf(lg[c] - m);
      if (lg[c] > lg[am]) am = c;
    }
    const float lse = m + logf(se);
    const int yy = (int)y[s];
    const float ws = wts[s];
    lsum += ws * (lse - lg[yy]);
    csum += (am == yy && ws > 0.f) ? 1.f : 0.f;
    for (int c = 0; c < C; ++c) dlog[s * CMAXC + c] = (expf(lg[c] - lse) - (c == yy ? 1.f : 0.f)) * ws;
    for (int j = 0; j < HID; ++j) {
      float d = 0.f;
      for (int c = 0; c < C; ++c) d = fmaf(Ws[c * HID + j], dlog[s * CMAXC + c], d);
      dh1[s * HID + j] = h1[s * HID + j] > 0.f ? d * mask[s * HID + j] : 0.f;
    }
  }
  red[tid] = lsum;
  red[256 + tid] = csum;
  __syncthreads();
  if (tid == 0) {
    float a = 0.f, c2 = 0.f;
    for (int t = 0; t < 256; ++t) { a += red[t]; c2 += red[256 + t]; }
    loss[k] = a;
    correct[k] = c2;
  }
  // fc2 grads: dW[c][j] = sum_b dlog[b][c] * a[b][j], db[c] = sum_b dlog[b][c]   (sequential over b)
  for (int e = tid; e < C * HID + C; e += 256) {
    float sacc = 0.f;
    if (e < C * HID) {
      const int c = e / HID, j = e - c * HID;
      for (int b = 0; b < B; ++b) {
        const size_t s = (size_t)k * B + b;
        sacc = fmaf(dlog[s * CMAXC + c], fmaxf(h1[s * HID + j], 0.f) * mask[s * HID + j], sacc);
      }
      grad[(size_t)k * P + off_w + e] = sacc;
    } else {
      const int c = e - C * HID;
      for (int b = 0; b < B; ++b) sacc += dlog[((size_t)k * B + b) * CMAXC + c];
      grad[(size_t)k * P + off_b + c] = sacc;
    }
  }
}

size_t fwd_lds() {
  return (size_t)(C2 * W2S + C1 * K1P + C1 + C2) * 4 + (K2 + K1P) * 4 + (size_t)(FSG * IMGP * IMGP + FSG * C1 * P1P * P1P) * 4;
}
size_t bwd_lds() {
  return (size_t)(C1 * W2T + C2 * P1P * P1P + C1 * P1P * P1P + C1 * Q1 * Q1 + IMGP * IMGP + NW * 2 * 256 + 48) * 4 +
         (size_t)(2 * K2 + K2) * 4 + C1 * Q1 * Q1;
}

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

extern "C" int qfx_cnn_backward(const float* X, const float* params, int P, int K, int B, const int* off4,
                                const float* pool1, const uint8_t* am1, const float* pool2, const uint8_t* am2,
                                const float* dP2, float* part, float* grad, hipStream_t st) {
  const int G = (B + BS - 1) / BS;
  const CnnOff off{off4[0], off4[1], off4[2], off4[3]};
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute((const void*)cnn_bwd, hipFuncAttributeMaxDynamicSharedMemorySize, (int)bwd_lds());
    attr = true;
  }
  hipLaunchKernelGGL(cnn_bwd, dim3(K * G), dim3(NT), bwd_lds(), st, X, params, P, B, G, off, pool1, am1, pool2, am2,
                     dP2, part);
  hipLaunchKernelGGL(cnn_reduce, dim3((PART + 255) / 256, K), dim3(256), 0, st, part, G, grad, P, off);
  return (int)hipGetLastError();
}

extern "C" int qfx_cnn_head(const float* h1, const float* mask, const float* params, int P, int off_w, int off_b,
                            int C, int K, int B, const long long* y, const float* wts, float* dh1, float* dlog,
                            float* loss, float* correct, float* grad, hipStream_t st) {
  if (C > CMAXC) return -2;
  hipLaunchKernelGGL(cnn_head, dim3(K), dim3(256), 0, st, h1, mask, params, P, off_w, off_b, C, B, y, wts, dh1, dlog,
                     loss, correct, grad);
  return (int)hipGetLastError();
}

extern "C" int qfx_cnn_partial_size() { return PART; }
extern "C" int qfx_cnn_bwd_groups(int B) { return (B + BS - 1) / BS; }
