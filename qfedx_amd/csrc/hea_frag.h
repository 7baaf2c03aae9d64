// Unitary fragments of the MFMA statevector engine, shared by hea_frag_kernel (hea_step.hip: per client and slot
// before a local step) and the round prologue (train_kernels.hip: a round's first step, when every client row is the
// global parameter vector, builds ONE shared set in the same launch that sets the rows - one dispatch fewer).
//
// Per slot: U and U^H in the real 32 x 32 embedding, laid out as the MFMA A operand of v_mfma_f32_16x16x32_f16 /
// _bf16 (lane l: row 16h + (l & 15), k = 8 (l >> 4) .. +7), hi and lo halves.  Rows are ordered (component,
// amplitude): row 16 h + m' is the re (h = 0) or im (h = 1) part of output m'.  The same registers are the B operand
// of the transposed product X^T M^T (group_back_t).
// frags[((k * n_slots + slot) * 4 + f) * 128 + h * 64 + lane], f = 0 U hi, 1 U lo, 2 U^H hi, 3 U^H lo.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

namespace hea_frag {

// one (client row, slot) of fragments by a 256-thread block: thread t = (U or U^H, re or im rows, lane).
// ST: _Float16 or __bf16 (the state storage type).  prm: the client's parameter row; st: the slot's table row
// (nreal, 4 theta slots, 4 phi slots); out: the (client, slot) fragment base.
template <typename ST>
__device__ __forceinline__ void build(const float* __restrict__ prm, const int* __restrict__ st, int t, uint4* out) {
  typedef ST h2 __attribute__((ext_vector_type(2)));
  const int dag = t >> 7, h = (t >> 6) & 1, lane = t & 63;
  const int nreal = st[0];
  // per qubit j: RZ(ph) RX(th) = [[e- c, -i e- s], [-i e+ s, e+ c]], e-+ = cp -+ i sp (identity past nreal)
  float cj[4], sj[4], cpj[4], spj[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    cj[j] = 1.f, sj[j] = 0.f, cpj[j] = 1.f, spj[j] = 0.f;
    if (j < nreal) {
      __sincosf(0.5f * prm[st[1 + j]], &sj[j], &cj[j]);
      __sincosf(0.5f * prm[st[5 + j]], &spj[j], &cpj[j]);
    }
  }
  // real output row r = 16 h + (lane & 15) is component cr = h (0 re, 1 im) of amplitude m' = lane & 15: a block's
  // result then holds the re and im of one amplitude in the same register of its two 16-row tiles
  ST hi[8], lo[8];
#pragma unroll
  for (int jj = 0; jj < 8; ++jj) {
    const int kk = 8 * (lane >> 4) + jj;
    const int mp = lane & 15, cr = h, m = kk >> 1, ck = kk & 1;
    const int row = dag ? m : mp, colm = dag ? mp : m;   // U^H[mp][m] = conj(U[m][mp])
    float vx = 1.f, vy = 0.f;
    // entry (row_j, col_j) of qubit j's 2 x 2 factor, formed arithmetically (a run-time index into a table of
    // the four entries put it in scratch): diagonal (cp c, +-sp c), off-diagonal (+-sp s, -cp s), sign + for row 1
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const bool rb = (row >> j) & 1, cb = (colm >> j) & 1;
      const float e = rb ? spj[j] : -spj[j];
      const float fx = rb == cb ? cpj[j] * cj[j] : e * sj[j], fy = rb == cb ? e * cj[j] : -cpj[j] * sj[j];
      const float nx = vx * fx - vy * fy, ny = vx * fy + vy * fx;
      vx = nx;
      vy = ny;
    }
    if (dag) vy = -vy;
    const float val = cr == 0 ? (ck == 0 ? vx : -vy) : (ck == 0 ? vy : vx);
    hi[jj] = (ST)val;
    lo[jj] = (ST)(val - (float)hi[jj]);
  }
  uint4 H, Lw;
  uint32_t* hp = (uint32_t*)&H;
  uint32_t* lp = (uint32_t*)&Lw;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    h2 a2 = {hi[2 * i], hi[2 * i + 1]}, b2 = {lo[2 * i], lo[2 * i + 1]};
    hp[i] = __builtin_bit_cast(uint32_t, a2);
    lp[i] = __builtin_bit_cast(uint32_t, b2);
  }
  uint4* base = out + (size_t)(2 * dag) * 128;
  base[h * 64 + lane] = H;
  base[128 + h * 64 + lane] = Lw;
}

}  // namespace hea_frag
