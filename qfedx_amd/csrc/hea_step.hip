// Per-step kernels of the MFMA statevector engine (passes: hea_mfma.hip): the unitary fragments of every (client,
// slot) before a step, and the fixed-order gradient reduction of the pass kernels' slab (with the fused readout
// sums and the optional fused Adam step).  hea_mfma_bf16.hip includes this file for the bf16 fragment build.
#include "hea_common.h"
#include "hea_frag.h"
#include "qfx_fedavg.h"

namespace HEA_NS {

// Unitary fragments of every (client, slot): hea_frag.h (layout), one 256-thread block each.
__global__ void __launch_bounds__(256) hea_frag_kernel(const float* __restrict__ params, int p_stride,
                                                       const int* __restrict__ slot_tab, int n_slots,
                                                       uint4* __restrict__ frags) {
  const int slot = blockIdx.x, k = blockIdx.y;
  hea_frag::build<st_t>(params + (size_t)k * p_stride, slot_tab + slot * 9, threadIdx.x,
                        frags + (size_t)(k * n_slots + slot) * 4 * 128);
}

// Per client and gradient op: exact int64 sums of the 32 partial-trace slots over the client's samples and
// the op's tiles, then per real qubit j (slots 8j + 4y + 2x + comp = n_j[y][x].(re, im))
//   d/dtheta = Im(e^{-i phi} n10 + e^{i phi} n01),   d/dphi = Im(n00 - n11).
//
// Optional Adam epilogue (ad.m != nullptr; the local optimizer step fused into this launch): Adam is elementwise,
// and every parameter's gradient is formed by exactly one block (its gradient op's, or the readout block's for the
// readout parameters; the host checks the cover, HeaMfmaProgram.grad_cover_exact), so each block updates the
// parameters it owns right after forming their gradients, with the element update of qfx_adam_kernel (qfx_adam.h):
// bitwise the separate launch, and no per-client hand-off.  A block reads only its own op's parameters (before it
// updates them).  Block (k, 0) writes the client's step counter.
#if !QFX_HEA_BF16
__global__ void __launch_bounds__(256) hea_grad_reduce_kernel(const long long* __restrict__ gslab, int slab_tiles,
                                                              int n_gradops, const int* __restrict__ gmeta, int spc,
                                                              float* __restrict__ params,
                                                              float* __restrict__ grad, int p_stride, QfxAdamArgs ad,
                                                              QfxReadoutRed ro, QfxFedTail ft) {
  // 8 groups of 32 lanes split the client's (sample, tile) rows; 16 independent loads in flight per lane; the
  // int64 sums are exact, so the group split and the LDS combine do not change a bit of the result
  const int k = blockIdx.x, g = blockIdx.y, tid = threadIdx.x, lane = tid & 31, grp = tid >> 5;
  // fused Adam of one owned parameter i (row k) from its gradient, then - the round's last local step - the
  // client's exact FedAvg term of it into the round buffer
  const double SC = 4294967296.0;
  int nsat = 0;
  auto owned_step = [&](int i, float gi) {
    const long e = (long)k * p_stride + i;
    qfx_adam_elem(params, gi, ad.m, ad.v, ad.t_in, ad.t_out, ad.active, k, e, false, ad.lr, ad.b1, ad.b2, ad.eps);
    if (!ft.buf) return;
    double d = (double)params[e] - (double)ft.theta_g[i];
    if (ft.wrap && ft.mask[i]) d = qfx::wrap_pi(d);
    const long long v = qfx::fixed_term(ft.weights[k] * d * SC, nsat);
    if (v) atomicAdd((unsigned long long*)&ft.buf[i], (unsigned long long)v);
  };
  if (g == n_gradops) {
    // fused readout: the client's per-sample records summed in a fixed order - loss, hits, and the readout gradients
    // d/da_c = sum dl_c z_c, d/db_c = sum dl_c.  Thread t < GS * NV sums value q = t % NV of samples t / NV + GS i
    // (its loads are contiguous across threads and all in flight), then thread q sums the GS partials in order.
    // (A loop over q with a load and a tree per value serialised NV global round trips: this block was the
    // straggler of the 8-client reduction.)
    __shared__ float rs[256];
    const int NV = 2 * ro.C + 2, GS = 256 / NV;
    const float* rec = ro.rec + (size_t)k * spc * NV;
    float v = 0.f;
    if (tid < GS * NV)
      for (int j = tid / NV; j < spc; j += GS) v += rec[j * NV + tid % NV];
    rs[tid] = v;
    __syncthreads();
    if (tid < NV) {
      float tot = 0.f;
      for (int j = 0; j < GS; ++j) tot += rs[j * NV + tid];
      if (tid < 2 * ro.C) {
        grad[(size_t)k * p_stride + ro.n_theta + tid] = tot;
        if (ad.m) owned_step(ro.n_theta + tid, tot);
      } else if (tid == 2 * ro.C)
        ro.loss[k] = tot;
      else
        ro.correct[k] = tot;
    }
  } else {
    const int* m = gmeta + g * 10;
    // m[1]: nreal in bits 0..3; bit 4 = cross matrix taken at the op INPUT (transposed BACK ops)
    const int nt = m[0], nreal = m[1] & 15, inside = (m[1] >> 4) & 1;
    const int R = spc * nt;
    __shared__ long long part[8][32];
    __shared__ double pt[32];
    auto row = [&](int r) -> long long {
      const int s = k * spc + r / nt, t = r % nt;
      return gslab[(((size_t)s * slab_tiles + t) * n_gradops + g) * 32 + lane];
    };
    // RU rows per lane in flight: the slab rows come from other XCDs' passes (an L2 miss each), and a 4-deep chain
    // made the 8-client reduction 8 dependent round trips long
    constexpr int RU = 16;
    long long tot = 0;
    int r = grp;
    for (; r + 8 * (RU - 1) < R; r += 8 * RU) {
      long long v[RU];
#pragma unroll
      for (int u = 0; u < RU; ++u) v[u] = row(r + 8 * u);
#pragma unroll
      for (int u = 0; u < RU; ++u) tot += v[u];
    }
    for (; r < R; r += 8) tot += row(r);
    part[grp][lane] = tot;
    __syncthreads();
    if (tid < 32) {
      long long v = 0;
      for (int j = 0; j < 8; ++j) v += part[j][tid];
      pt[tid] = (double)v / FIX;
    }
    __syncthreads();
    if (tid < nreal) {
      const double* p = pt + 8 * tid;
      const float* prm = params + (size_t)k * p_stride;
      float gth, gph;
      if (inside) {
        // at the op input: d/dtheta = Im<lam|X|psi> = Im(n01 + n10);
        // d/dphi = Im<lam|RX^H Z RX|psi> = cos(theta) Im(n00 - n11) + sin(theta) Re(n01 - n10)
        const double th = prm[m[2 + tid]];
        const double ct = cos(th), st = sin(th);
        gth = (float)(p[3] + p[5]);
        gph = (float)(ct * (p[1] - p[7]) + st * (p[2] - p[4]));
      } else {
        const double ph = prm[m[6 + tid]];
        const double cp = cos(ph), sp = sin(ph);
        gth = (float)((cp * p[5] - sp * p[4]) + (cp * p[3] + sp * p[2]));
        gph = (float)(p[1] - p[7]);
      }
      grad[(size_t)k * p_stride + m[2 + tid]] = gth;
      grad[(size_t)k * p_stride + m[6 + tid]] = gph;
      if (ad.m) {
        owned_step(m[2 + tid], gth);
        owned_step(m[6 + tid], gph);
      }
    }
  }
  if (!ad.m) return;
  if (g == 0 && tid == 0) {
    ad.t_out[k] = ad.t_in[k] + ad.active[k];          // the client's step counter (qfx_adam_elem's `first`)
    if (ft.buf) {
      const long long v = qfx::fixed_term(ft.weights[k] * SC, nsat);
      if (v) atomicAdd((unsigned long long*)&ft.buf[p_stride], (unsigned long long)v);
    }
  }
  if (!ft.buf) return;
  // ---- the round's FedAvg (QfxFedTail): every block added its owned parameters' terms above; the last block of
  // the launch packs the metrics and (single rank) applies the round
  if (nsat) atomicAdd((unsigned long long*)&ft.buf[p_stride + 5], (unsigned long long)nsat);   // saturated terms
  __shared__ int flast_s;
  // The block's stores and atomics are complete in L2 after the barrier; ONE agent-scope release (thread 0) makes
  // them visible across XCDs before the arrival (issued by every thread, a release - an L2 writeback here - made
  // the launch 7x slower: 16q x 64 clients, 13 -> 98 us).
  __syncthreads();
  if (tid == 0) {
    __threadfence();
    flast_s = atomicAdd(ft.cnt, 1u) == gridDim.x * gridDim.y - 1;
    if (flast_s) *ft.cnt = 0u;
  }
  __syncthreads();
  if (!flast_s) return;
  if (tid == 0) {                                      // every client's terms and metrics: acquire, drained
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    __asm__ volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  __syncthreads();
  qfx::round_pack_block(qfx::RoundPack{ft.buf, ft.loss, ft.correct, ft.nvalid, ft.act, ft.n_metrics, nullptr,
                                       nullptr, 0},
                        p_stride);
  if (!ft.apply_theta) return;
  __syncthreads();
  auto ld = [&](long i) { return __hip_atomic_load(&ft.buf[i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); };
  const double wsum = (double)ld(p_stride) / SC;
  for (long e = tid; e < (long)p_stride + 6 + ft.n_norms; e += 256)
    qfx::round_apply_elem(ft.buf, p_stride, ft.apply_theta, 1.0, ft.apply_out, 0, 1.0, ft.n_norms, e, wsum, ld);
}
#endif  // !QFX_HEA_BF16

}  // namespace HEA_NS

extern "C" int HEA_EXT(qfx_hea_frags)(const float* params, int p_stride, const int* slot_tab, int n_slots, int K, void* frags,
                             hipStream_t st) {
  if (n_slots == 0 || K == 0) return 0;
  hipLaunchKernelGGL(HEA_NS::hea_frag_kernel, dim3(n_slots, K), dim3(256), 0, st, params, p_stride, slot_tab, n_slots,
                     (uint4*)frags);
  return (int)hipGetLastError();
}

#if !QFX_HEA_BF16
extern "C" int qfx_hea_grad_reduce(const long long* gslab, int slab_tiles, int n_gradops, const int* gmeta, int spc,
                                   int K, float* params, float* grad, int p_stride, const QfxAdamArgs* adam,
                                   const QfxReadoutRed* readout, const QfxFedTail* fed, hipStream_t st) {
  if (K == 0) return 0;
  QfxReadoutRed ro{};
  if (readout) ro = *readout;
  const int rows = n_gradops + (ro.rec ? 1 : 0);
  if (rows == 0) return adam && adam->m ? (int)hipErrorInvalidValue : 0;   // no block would run the epilogue
  QfxAdamArgs ad{};
  if (adam) ad = *adam;
  QfxFedTail ftl{};
  if (fed) {
    if (!adam || !adam->m) return (int)hipErrorInvalidValue;   // the FedAvg tail runs in the Adam epilogue
    ftl = *fed;
  }
  hipLaunchKernelGGL(HEA_NS::hea_grad_reduce_kernel, dim3(K, rows), dim3(256), 0, st, gslab, slab_tiles, n_gradops,
                     gmeta, spc, params, grad, p_stride, ad, ro, ftl);
  return (int)hipGetLastError();
}

extern "C" int qfx_hea_args_size() { return (int)sizeof(HEA_NS::PassArgs); }
#endif  // !QFX_HEA_BF16

