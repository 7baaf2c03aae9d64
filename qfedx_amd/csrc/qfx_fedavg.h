// FedAvg epilogue pieces shared by the fused FedAvg reduce (train_kernels.hip) and the MFMA engine's gradient
// reduction when it folds the round's FedAvg into its Adam epilogue (hea_step.hip): the wrapped update, the exact
// fixed-point term, the metric pack and the apply of one all-reduced entry - one definition, so both paths produce
// the same bits.
#pragma once
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>

namespace qfx {

__device__ __forceinline__ double wrap_pi(double d) {
  const double tp = 6.283185307179586;
  double r = fmod(d + 3.141592653589793, tp);
  if (r < 0) r += tp;
  return r - 3.141592653589793;
}

// one client's fixed-point FedAvg term of parameter e.  A term is held to |v| <= FA_SAT = 2^53 (exactly
// representable, and up to 2^10 such terms still sum inside int64): a larger w_k * Delta (|w Delta| > 2^21, e.g.
// sample-count weights times a diverged CNN delta) is clamped and counted in *nsat instead of wrapping in llrint.
constexpr double FA_SAT = 9007199254740992.0;
__device__ __forceinline__ long long fixed_term(double v, int& nsat) {
  if (!(fabs(v) <= FA_SAT)) {          // also catches NaN (clamped to 0)
    ++nsat;
    v = v > 0.0 ? FA_SAT : (v < 0.0 ? -FA_SAT : 0.0);
  }
  return llrint(v);
}

// round epilogue 1 body: metrics -> exact fixed point in the all-reduce buffer tail, fixed summation order
//   buf[P+1..P+4] = round(2^32 * [sum loss*nvalid, sum correct*act, sum nvalid (samples), sum act (steps)])
// Everything comes from device tables (nothing round-dependent is a kernel argument), so the launch can sit
// inside a captured round graph.  One 256-thread block: strided float64 partials, then a fixed-shape tree.
struct RoundPack {          // metrics of the round epilogue (buf == nullptr: not packed by this launch)
  long long* buf;
  const float *loss, *correct, *nvalid, *act;
  int n;
  // CC6: the K local clients' update norms (DP: pre-clip l2 norms) scattered as 2^32 fixed point into the
  // buffer's per-client slots buf[P + 6 + cid[k]] (zero elsewhere on this rank): the round's SUM all-reduce then
  // delivers every client's norm to every rank with no extra collective.  norms == nullptr: not logged.
  const double* norms;
  const int* cid;
  int K;
};

__device__ __forceinline__ void round_pack_block(const RoundPack& rp, int P) {
  // the first 256 threads of the block (the fedavg launch's pack block has more; they only join the barriers)
  __shared__ double red[4][256];
  const int t = threadIdx.x;
  const bool on = t < 256;
  double ls = 0.0, cs = 0.0, ns = 0.0, as = 0.0;
  for (int i = t; on && i < rp.n; i += 256) {
    const double nv = (double)rp.nvalid[i], ac = (double)rp.act[i];
    ls += (double)rp.loss[i] * nv;
    cs += (double)rp.correct[i] * ac;
    ns += nv;
    as += ac;
  }
  if (on) {
    red[0][t] = ls;
    red[1][t] = cs;
    red[2][t] = ns;
    red[3][t] = as;
  }
  __syncthreads();
  for (int h = 128; h > 0; h >>= 1) {
    if (t < h)
      for (int j = 0; j < 4; ++j) red[j][t] += red[j][t + h];
    __syncthreads();
  }
  if (t < 4) rp.buf[P + 1 + t] = llrint(red[t][0] * 4294967296.0);
  if (rp.norms && on)
    for (int k = t; k < rp.K; k += 256) rp.buf[P + 6 + rp.cid[k]] = llrint(rp.norms[k] * 4294967296.0);
}

// round epilogue 2 for one entry e of the all-reduced buffer (qfx_round_apply_kernel below, or the last block of a
// single-rank FedAvg reduce, FusedApply):
// theta += lr * (sum w Delta) / (sum w) in float64, rounded to fp32 - the same operations as Aggregator.finalize +
// apply; rounds with zero total weight keep theta.
//   out[0..3] = metrics, out[4] = saturated FedAvg terms over all ranks (buf[P + 5], which this zeroes for the next
//   round: nothing else reads it, and the next round's reduce runs after it), out[5] = weight sum
// With SecAgg (bits > 0) the update and weight entries are ring elements: reduced mod 2^bits, read as signed and
// divided by the SecAgg scale (decode_fixed); the metric tail stays plain 2^32 fixed point.  ``ld`` loads an entry
// of buf (a device-coherent load when other blocks of the same launch wrote it).
__device__ __forceinline__ double ring_decode(long long v, int bits, double scale) {
  const long long m = (1LL << bits) - 1;
  long long u = v & m;
  if (u >> (bits - 1)) u -= (1LL << bits);
  return (double)u / scale;
}

template <typename Ld>
__device__ __forceinline__ void round_apply_elem(long long* buf, int P, float* theta, double lr, double* out, int bits,
                                                 double ring_scale, int n_norms, long e, double wsum, Ld ld) {
  const double SC = 4294967296.0;
  if (e < P) {
    const long long b = ld(e);
    const double upd = bits ? ring_decode(b, bits, ring_scale) : (double)b / SC;
    const double mean = upd / fmax(wsum, 1e-300);
    const double th = (double)theta[e];
    theta[e] = wsum > 0.0 ? (float)(th + lr * mean) : (float)th;
  } else if (e < P + 6) {
    const int j = (int)(e - P);
    if (j < 4) {
      out[j] = (double)ld(P + 1 + j) / SC;
    } else if (j == 4) {
      out[j] = (double)ld(P + 5);
      buf[P + 5] = 0;
    } else {
      out[j] = wsum;
    }
  } else if (e < P + 6 + n_norms) {    // CC6 per-client norm slots: read out, zeroed for the next round
    const int j = (int)(e - P);
    out[j] = (double)ld(P + j) / SC;
    buf[P + j] = 0;
  }
}

}  // namespace qfx
