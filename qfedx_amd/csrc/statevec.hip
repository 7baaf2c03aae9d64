// gfx950 (MI355X / CDNA4) statevector pass kernels: forward, readout, adjoint gradients.
//
// Replaces the reference's CPU Qiskit simulation (src/QFed/qAmplitude.py:44-46) and implements the
// ROADMAP VQC (ROADMAP.md:20-23,125-135) - SURVEY kernels K9/K11 (state init), K12 (gates),
// K13/K14 (<Z> readout), K16 (adjoint differentiation).
//
// Execution model (see qfx_plan.h): one launch = one pass over every 2^k-amplitude tile of every
// sample.  A 256-thread workgroup (4 wave64s) holds 256*R amplitudes in REGISTERS (R per lane);
// gates on register bits are VALU-only (fused per register bit into "G1 groups": one 2x2 apply for
// RX.RZ in the forward pass, one per-pair sweep with inverse + gradient in the adjoint pass), gates
// on thread bits are reached through LDS remaps whose slot arithmetic the host planner precomputed
// (GF(2)-linear CNOT maps and the XOR bank swizzle fold into per-register / per-thread-bit XOR
// tables), so the device loop is: one uniform op fetch, then pure data movement / FMA work.
// Small states (n <= 12) fit one tile -> the whole circuit is ONE launch with no HBM state traffic;
// 16-24 qubit states stream once per pass with 128-byte coalesced rows.  Adjoint mode carries psi
// and lambda together and reduces every parameter's Im<lambda|P|psi> deterministically
// (wave64 xor-tree, fixed-order cross-wave sum).
#include "qfx_device.h"

namespace qfx {

template <int R, bool ADJ>
__global__ void __launch_bounds__(256) qfx_pass_kernel(PassArgs A) {
  constexpr int RB = (R == 4) ? 2 : (R == 8) ? 3 : (R == 16) ? 4 : 5;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  cint_p blob = (cint_p)(A.blob);
  cint_p pd = blob + A.pass_off;
  cint_p gt = blob + blob[HF_GATES];
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
  const int nops = pd[PF_NOPS];
  cint_p ops = blob + pd[PF_OPS];

  uint32_t gbase = 0;
  {
    const int nn = pd[PF_NNONTILE];
    for (int j = 0; j < nn; ++j) gbase |= ((tau >> j) & 1u) << pd[PF_NONTILE + j];
  }
  // LDS: [exchange 256R v2f][readout 64 f][grad partials A.n_grad*5 f][coef tiles_pb*G v2f]
  //      [prefix vectors tiles_pb*n float4]; tables only when a tile spans >= one wave (T >= 64)
  v2f* xb = reinterpret_cast<v2f*>(smem) + (size_t)tib * (1u << k);
  float* red = reinterpret_cast<float*>(smem + 256 * R * sizeof(v2f));
  float* gacc = red + 64;
  v2f* ctab = reinterpret_cast<v2f*>(gacc + ((A.n_grad * 5 + 3) & ~3));
  float4* vtab = reinterpret_cast<float4*>(ctab + ((tiles_pb * G + 1) & ~1));
  const int init = pd[PF_INIT];
  const bool use_tab = T >= 64;
  if (use_tab) {
    const long tile0 = (long)blockIdx.x * tiles_pb;
    for (int e = tid; e < tiles_pb * G; e += 256) {
      const int tb_ = e / G, g = e - tb_ * G;
      long sm = (tile0 + tb_) >> ltps;
      if (sm >= A.n_samples) sm = 0;
      ctab[e] = gate_cs(gt, g, A.params + (size_t)(sm / A.spc) * A.p_stride, A.xang + (size_t)sm * A.x_stride,
                        n_theta);
    }
    if (init == INIT_PRODUCT) {
      for (int e = tid; e < tiles_pb * n; e += 256) {
        const int tb_ = e / n, q = e - tb_ * n;
        long sm = (tile0 + tb_) >> ltps;
        if (sm >= A.n_samples) sm = 0;
        vtab[e] = prefix_vec(blob, q, A.params + (size_t)(sm / A.spc) * A.p_stride,
                             A.xang + (size_t)sm * A.x_stride, n_theta);
      }
    }
    __syncthreads();
  }

  v2f a[R];
  v2f l[R];
#pragma unroll
  for (int r = 0; r < R; ++r) l[r] = mk(0.f, 0.f);

  // ------------------------------------------------------------------ init
  if (init == INIT_PRODUCT) {
    v2f base = mk(1.f, 0.f);
    const int nn = pd[PF_NNONTILE];
    for (int j = 0; j < nn; ++j) {
      const int q = pd[PF_NONTILE + j];
      const float4 v = use_tab ? vtab[tib * n + q] : prefix_vec(blob, q, prow, xrow, n_theta);
      base = cmul(base, ((gbase >> q) & 1u) ? mk(v.z, v.w) : mk(v.x, v.y));
    }
    for (int p = RB; p < k; ++p) {
      const int q = pd[PF_Q0 + p];
      const float4 v = use_tab ? vtab[tib * n + q] : prefix_vec(blob, q, prow, xrow, n_theta);
      base = cmul(base, ((tl >> (p - RB)) & 1) ? mk(v.z, v.w) : mk(v.x, v.y));
    }
    a[0] = base;
#pragma unroll
    for (int p = 0; p < RB; ++p) {
      const int q = pd[PF_Q0 + p];
      const float4 v = use_tab ? vtab[tib * n + q] : prefix_vec(blob, q, prow, xrow, n_theta);
#pragma unroll
      for (int r = 0; r < (1 << p); ++r) {
        a[r | (1 << p)] = cmul(mk(v.z, v.w), a[r]);
        a[r] = cmul(mk(v.x, v.y), a[r]);
      }
    }
  } else {
    const uint32_t gthr = xor_bits(pd + PF_GTHR0, tb, tl);
#pragma unroll
    for (int r = 0; r < R; ++r) {
      const size_t off = sbase + gbase + (gthr | (uint32_t)pd[PF_GREG0 + r]);
      a[r] = valid ? A.psi[off] : mk(0.f, 0.f);
      if constexpr (ADJ) {
        if (init == INIT_LOAD_BOTH) l[r] = valid ? A.lam[off] : mk(0.f, 0.f);
      }
    }
    if constexpr (ADJ) {
      if (init == INIT_PSI_LAMBDA) {
        const int C = pd[PF_NREAD];
        float wv[8];
#pragma unroll
        for (int c = 0; c < 8; ++c) wv[c] = (c < C && valid) ? A.w_read[(size_t)s_eff * C + c] : 0.f;
#pragma unroll
        for (int r = 0; r < R; ++r) {
          float s = 0.f;
#pragma unroll
          for (int c = 0; c < 8; ++c) {
            if (c < C) s += pbit<RB>(pd[PF_LAM_PHYS + c], r, tl, gbase) ? -wv[c] : wv[c];
          }
          l[r] = mk(a[r].x * s, a[r].y * s);
        }
      }
    }
  }

  int gcount = 0;

  // ------------------------------------------------------------------ micro-ops
  for (int i = 0; i < nops; ++i) {
    const int code = ops[i * OP_WORDS + 0];
    const int oa = ops[i * OP_WORDS + 1];
    const int ob = ops[i * OP_WORDS + 2];
    const int oc = ops[i * OP_WORDS + 3];
    if (code == OP_G1) {
      cint_p glist = blob + oc;
      if constexpr (!ADJ) {
        const int g0 = glist[0];
        M2 m = gate_m2(gt[g0 * GATE_WORDS], use_tab ? ctab[tib * G + g0] : gate_cs(gt, g0, prow, xrow, n_theta),
                       false);
        for (int j = 1; j < ob; ++j) {
          const int g = glist[j];
          m = m2mul(gate_m2(gt[g * GATE_WORDS], use_tab ? ctab[tib * G + g] : gate_cs(gt, g, prow, xrow, n_theta),
                            false),
                    m);
        }
        QFX_RB_DISPATCH(oa, (m2_apply<R, RBT>(a, m)));
      } else {
        for (int j = 0; j < ob; ++j) {
          const int g = glist[j];
          const int kind = gt[g * GATE_WORDS];
          const int slot = gt[g * GATE_WORDS + 3];
          const bool isg = slot >= 0 && slot < n_theta && kind <= K_P;
          const int cls = isg ? (kind == K_RX ? CLS_RX : kind == K_RY ? CLS_RY : CLS_RZ)
                              : (kind_is_diag(kind) ? CLS_DIAG : (kind == K_RX ? CLS_RX : kind == K_RY ? CLS_RY : CLS_GEN));
          const M2 mi = gate_m2(kind, use_tab ? ctab[tib * G + g] : gate_cs(gt, g, prow, xrow, n_theta), true);
          float part = 0.f;
          QFX_RB_DISPATCH(oa, QFX_CLS_DISPATCH(cls, RBT, part));
          if (isg) {
            part = group_sum(part, T);
            if (T <= 64) {
              if (tl == 0 && valid) A.gslab[(size_t)tile * G + g] = part;
            } else if (lane == 0) {
              gacc[gcount * 5 + wave] = part;
              if (wave == 0) gacc[gcount * 5 + 4] = __int_as_float(g);
            }
            ++gcount;
          }
        }
      }
    } else if (code == OP_D1T) {
      const int kind = gt[oc * GATE_WORDS];
      const M2 m = gate_m2(kind, use_tab ? ctab[tib * G + oc] : gate_cs(gt, oc, prow, xrow, n_theta), ADJ);
      const int bit = pbit<RB>(oa, 0, tl, gbase);   // thread or non-tile bit: same for all registers
      const v2f ph = bit ? m.d : m.a;
      if constexpr (ADJ) {
        const int slot = gt[oc * GATE_WORDS + 3];
        if (slot >= 0 && slot < n_theta && (kind == K_RZ || kind == K_P)) {
          float part = 0.f;
#pragma unroll
          for (int r = 0; r < R; ++r) part += imcl(l[r], a[r]);
          part = group_sum(bit ? -part : part, T);
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
        a[r] = cmul(ph, a[r]);
        if constexpr (ADJ) l[r] = cmul(ph, l[r]);
      }
    } else if (code == OP_REMAP) {
      do_remap<R>(a, xb, blob + oa, tb, tl);
      if constexpr (ADJ) do_remap<R>(l, xb, blob + oa, tb, tl);
    } else if (code == OP_CX) {
      QFX_RB_DISPATCH(ob, (cx_apply<R, RB, RBT, ADJ>(a, l, oa, tl, gbase)));
    } else if (code == OP_CZ) {
#pragma unroll
      for (int r = 0; r < R; ++r) {
        if (pbit<RB>(oa, r, tl, gbase) & pbit<RB>(ob, r, tl, gbase)) {
          a[r] = mk(-a[r].x, -a[r].y);
          if constexpr (ADJ) l[r] = mk(-l[r].x, -l[r].y);
        }
      }
    }
  }

  // ------------------------------------------------------------------ finalize
  const int fin = pd[PF_FINAL];
  if constexpr (ADJ) {
    if (T > 64 && gcount > 0) {
      // a tile spans WPT = T/64 waves (2 tiles per block at T=128): sum only its own waves
      __syncthreads();
      const int WPT = T >> 6;
      for (int e = tid; e < tiles_pb * gcount; e += 256) {
        const int tb_ = e / gcount, g = e - tb_ * gcount;
        float sum = 0.f;
        for (int w = 0; w < WPT; ++w) sum += gacc[g * 5 + tb_ * WPT + w];
        const long tile_ = (long)blockIdx.x * tiles_pb + tb_;
        if ((tile_ >> ltps) < A.n_samples) A.gslab[(size_t)tile_ * G + __float_as_int(gacc[g * 5 + 4])] = sum;
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
        const float pr = fmaf(a[r].x, a[r].x, a[r].y * a[r].y);
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
      const int WPT = T >> 6;
      for (int e = tid; e < tiles_pb * C; e += 256) {
        const int tb_ = e / C, c = e - tb_ * C;
        float sum = 0.f;
        for (int w = 0; w < WPT; ++w) sum += red[c * 4 + tb_ * WPT + w];
        const long tile_ = (long)blockIdx.x * tiles_pb + tb_;
        if ((tile_ >> ltps) < A.n_samples) A.out_read[(size_t)tile_ * C + c] = sum;
      }
    }
  }
  if (fin & FIN_STORE) {
    const uint32_t gthr = xor_bits(pd + PF_GTHRF, tb, tl);
    if (valid) {
#pragma unroll
      for (int r = 0; r < R; ++r) {
        const size_t off = sbase + gbase + (gthr | (uint32_t)pd[PF_GREGF + r]);
        A.psi[off] = a[r];
        if constexpr (ADJ) A.lam[off] = l[r];
      }
    }
  }
}

}  // namespace qfx

// ----------------------------------------------------------------------------------- launchers
extern "C" int qfx_launch_pass(int R, int adjoint, const int* blob, int pass_off, int k, int n, int n_ops,
                               int n_gates, void* psi, void* lam, const float* params, int p_stride, int spc,
                               const float* xang, int x_stride, const float* w_read, float* out_read,
                               float* gslab, int n_samples, int n_grad_ops, hipStream_t stream) {
  using namespace qfx;
  (void)n_ops;
  const int tb = k - (R == 4 ? 2 : R == 8 ? 3 : R == 16 ? 4 : 5);
  if (tb < 0 || tb > 8) return -3;
  const int tiles_pb = 256 >> tb;
  const long tiles_total = (long)n_samples << (n - k);
  const long blocks = (tiles_total + tiles_pb - 1) / tiles_pb;
  if (blocks <= 0) return 0;
  PassArgs A{blob, pass_off, static_cast<v2f*>(psi), static_cast<v2f*>(lam), params, p_stride, spc, xang, x_stride, w_read, out_read, gslab, n_samples,
             n_grad_ops};
  const bool tab = (1 << tb) >= 64;
  const size_t lds = 256 * (size_t)R * sizeof(v2f) + 64 * sizeof(float) +
                     (size_t)((n_grad_ops * 5 + 3) & ~3) * sizeof(float) +
                     (tab ? (size_t)((tiles_pb * n_gates + 1) & ~1) * sizeof(v2f) + (size_t)tiles_pb * n * sizeof(float4)
                          : 0);
  if (lds > 160 * 1024) return -4;
  dim3 grid((unsigned)blocks), block(256);
#define QFX_L(RR, AA) hipLaunchKernelGGL((qfx_pass_kernel<RR, AA>), grid, block, lds, stream, A)
  if (R == 4) { if (adjoint) QFX_L(4, true); else QFX_L(4, false); }
  else if (R == 16) { if (adjoint) QFX_L(16, true); else QFX_L(16, false); }
  else return -1;
#undef QFX_L
  return (int)hipGetLastError();
}

// ----------------------------------------------------------------------------------- amplitude encoding (K9)
// Raw features x[s, 0:F] (F <= N = 2^n, zero-padded) -> normalised state psi[s, 0:N] in logical order:
// psi = x / ||x||_2 (float64 norm), a zero row -> the uniform state 1/sqrt(N) (reference
// normalize_for_amplitude, qAmplitude.py:11-22).  Two deterministic stages: per-(chunk, sample) float64
// partial sums of squares, then a write pass whose blocks first reduce their sample's partials in fixed
// order.  The state is written directly in the pass storage format (complex64 or packed bf16x2).
constexpr int AMP_CHUNK = 4096;

__device__ __forceinline__ double wave_sum_d(double v) {
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

__global__ void __launch_bounds__(256) qfx_amp_norm_kernel(const float* __restrict__ x, long F, long ld, int nch,
                                                          double* __restrict__ part) {
  __shared__ double sm[4];
  const long s = blockIdx.y;
  const long beg = (long)blockIdx.x * AMP_CHUNK, end = beg + AMP_CHUNK < F ? beg + AMP_CHUNK : F;
  const float* row = x + s * ld;
  double acc = 0.0;
  for (long i = beg + threadIdx.x; i < end; i += 256) {
    const double v = row[i];
    acc += v * v;
  }
  acc = wave_sum_d(acc);
  if ((threadIdx.x & 63) == 0) sm[threadIdx.x >> 6] = acc;
  __syncthreads();
  if (threadIdx.x == 0) part[s * nch + blockIdx.x] = (sm[0] + sm[1]) + (sm[2] + sm[3]);
}

template <bool BF16>
__global__ void __launch_bounds__(256) qfx_amp_write_kernel(const float* __restrict__ x, long F, long ld, int nch,
                                                           const double* __restrict__ part, long N,
                                                           void* __restrict__ psi) {
  __shared__ double sm[4];
  const long s = blockIdx.y;
  double acc = 0.0;
  for (int c = threadIdx.x; c < nch; c += 256) acc += part[s * nch + c];
  acc = wave_sum_d(acc);
  if ((threadIdx.x & 63) == 0) sm[threadIdx.x >> 6] = acc;
  __syncthreads();
  const double nrm2 = (sm[0] + sm[1]) + (sm[2] + sm[3]);
  const bool zero = !(nrm2 > 0.0);
  const double inv = zero ? 0.0 : 1.0 / sqrt(nrm2);
  const float uni = (float)(1.0 / sqrt((double)N));
  const float* row = x + s * ld;
  const long beg = (long)blockIdx.x * AMP_CHUNK;
  for (long i = beg + threadIdx.x; i < beg + AMP_CHUNK && i < N; i += 256) {
    const float a = zero ? uni : (i < F ? (float)((double)row[i] * inv) : 0.0f);
    if constexpr (BF16) {
      static_cast<uint32_t*>(psi)[s * N + i] = qfx::pack_bf16x2(qfx::mk(a, 0.0f));
    } else {
      static_cast<float2*>(psi)[s * N + i] = make_float2(a, 0.0f);
    }
  }
}

extern "C" int qfx_amp_scratch(long F) { return (int)((F + AMP_CHUNK - 1) / AMP_CHUNK); }

extern "C" int qfx_launch_amp_init(const float* x, long F, long ld, int n_samples, int n, double* part, void* psi,
                                   int bf16, hipStream_t stream) {
  const long N = 1L << n;
  if (F > N || F <= 0 || ld < F || n_samples <= 0) return -2;
  const int nch = (int)((F + AMP_CHUNK - 1) / AMP_CHUNK);
  const unsigned wch = (unsigned)((N + AMP_CHUNK - 1) / AMP_CHUNK);
  hipLaunchKernelGGL(qfx_amp_norm_kernel, dim3((unsigned)nch, (unsigned)n_samples), dim3(256), 0, stream, x, F, ld,
                     nch, part);
  if (bf16)
    hipLaunchKernelGGL(qfx_amp_write_kernel<true>, dim3(wch, (unsigned)n_samples), dim3(256), 0, stream, x, F, ld, nch,
                       part, N, psi);
  else
    hipLaunchKernelGGL(qfx_amp_write_kernel<false>, dim3(wch, (unsigned)n_samples), dim3(256), 0, stream, x, F, ld,
                       nch, part, N, psi);
  return (int)hipGetLastError();
}
