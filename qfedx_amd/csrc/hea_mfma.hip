// MFMA statevector engine for the hardware-efficient VQC (plan: qfedx_amd/ops/hea_plan.py).
//
// One workgroup owns one LDS tile of 2^t amplitudes of one sample (t <= 14; fp16 (re, im) packed in a
// u32 = 64 KB per state).  A pass = [product-state generation | tile load] -> op list -> [store],
// where every rotation op is a 16 x 16 complex unitary on a 4-dim GF(2) subspace of the tile:
//
//     Y[m', col] = sum_m U[m', m] X[m, col]        (columns = cosets of the subspace, 2^(t-4) of them)
//
// executed as v_mfma_f32_16x16x32_f16 with the complex matrix in its real 32 x 32 embedding (two
// 16-row blocks, K = 32 = 16 amplitudes x (re, im)) and split hi + lo in fp16 so the unitary is exact
// to ~2^-22 (the state itself is fp16 between ops, fp32 inside the MFMA).  Column c of a block maps to
// tile address  y'(c) ^ OFF[m ^ b(c)]  with y' a deposit of c into the non-pivot bits and b(c) the
// logical bits of y' in the op's CNOT frame (parities with the frame's row masks) - the CNOT chains are
// never executed, only folded into this addressing.
//
// Adjoint ops: gradient cross matrix N[b][a] = sum_col psi[b] conj(lam[a]) as two MFMAs per 16 columns
// (A = psi, B = lam and i*lam), reduced over waves in LDS; each qubit's 2x2 partial trace of N gives
// d/dtheta = Im(e^-i.phi n10 + e^i.phi n01) and d/dphi = Im(n00 - n11) (RZ(phi) RX(theta) rotation).
// Per-workgroup gradient partials go to a slab that hea_grad_reduce sums in a fixed order.
#include "hea_common.h"

#if QFX_CHECKS_ON
__device__ unsigned int qfx_check_word = 0;
#endif


namespace HEA_NS {

// Pass-output tiles are stored with the non-temporal hint when a pass's states exceed the Infinity Cache (PassArgs::
// nt_store, set by the host: 16q x 2048 samples = 512 MB per pass; the next pass reads them back from HBM anyway):
// interleaved A/B, 64 clients 1.820 -> 1.784 ms per step; at 8 clients (64 MB, MALL-resident) the plain stores are
// faster (profiles/r6_tile_nt_priority_ab.txt).  Non-temporal tile LOADS measured slower and are not used.
__device__ __forceinline__ void tile_st(uint32_t* p, uint4 v, int nt) {
  if (nt) {
    __builtin_nontemporal_store(u4v{v.x, v.y, v.z, v.w}, (u4v*)p);
    return;
  }
  *(uint4*)p = v;
}

// memory index of tile position tau
__device__ __forceinline__ uint32_t mem_of(uint32_t tau, const PassArgs& a, uint32_t fixed) {
  const uint32_t cm = (1u << a.c) - 1u;
  return (tau & cm) | ((tau >> a.c) << a.lo) | fixed;
}

// LDS swizzle h(x) (5 bank bits) of the high tile bits x = tau >> 5
__device__ __forceinline__ uint32_t swz(const PassArgs& a, uint32_t x) {
  uint32_t r = 0;
#pragma unroll
  for (int b = 0; b < 5; ++b) r |= (uint32_t)par((uint32_t)a.hrow[b] & x) << b;
  return r;
}

// out[j] = in[j ^ r]: a 16-byte quad whose dwords the swizzle permutes inside their aligned quad
__device__ __forceinline__ uint4 quad_perm(uint4 v, uint32_t r) {
  if (r & 1u) v = make_uint4(v.y, v.x, v.w, v.z);
  if (r & 2u) v = make_uint4(v.z, v.w, v.x, v.y);
  return v;
}

// Global [mem order] <-> LDS [swizzled] tile copies: quad q = 4 (tid + NT i) of the tile sits at LDS dword
// (q ^ h) & ~3 with its dwords permuted by h & 3, h = h(q >> 5) = h(tid >> 3) ^ h(4 NT / 32 * i).  All of a
// thread's global loads are issued before its LDS writes.
template <int NT, int TB = TMAX>
__device__ __forceinline__ void load_tile(const PassArgs& a, const uint32_t* src, uint32_t* dst, int tid, int T,
                                          uint32_t h_q, uint32_t fixed) {
  constexpr int MQ = (1 << TB) / (4 * NT);
  uint4 v[MQ];
#pragma unroll
  for (int i = 0; i < MQ; ++i) {
    const uint32_t q = 4u * (tid + NT * i);
    if (q < (uint32_t)T) v[i] = *(const uint4*)&src[mem_of(q, a, fixed)];
  }
#pragma unroll
  for (int i = 0; i < MQ; ++i) {
    const uint32_t q = 4u * (tid + NT * i);
    if (q < (uint32_t)T) {
      const uint32_t h = h_q ^ swz(a, (uint32_t)(4 * NT / 32) * i);
      *(uint4*)&dst[(q ^ h) & ~3u] = quad_perm(v[i], h & 3u);
    }
  }
}

template <int NT, int TB = TMAX>
__device__ __forceinline__ void store_tile(const PassArgs& a, uint32_t* dst, const uint32_t* src, int tid, int T,
                                           uint32_t h_q, uint32_t fixed) {
  constexpr int MQ = (1 << TB) / (4 * NT);
  uint4 v[MQ];
#pragma unroll
  for (int i = 0; i < MQ; ++i) {
    const uint32_t q = 4u * (tid + NT * i);
    if (q < (uint32_t)T) {
      const uint32_t h = h_q ^ swz(a, (uint32_t)(4 * NT / 32) * i);
      v[i] = quad_perm(*(const uint4*)&src[(q ^ h) & ~3u], h & 3u);
    }
  }
#pragma unroll
  for (int i = 0; i < MQ; ++i) {
    const uint32_t q = 4u * (tid + NT * i);
    if (q < (uint32_t)T) tile_st(&dst[mem_of(q, a, fixed)], v[i], a.nt_store);
  }
}

// Adjoint LDS image, interleaved: word 2w = psi, 2w + 1 = lambda of swizzled amplitude w.  One ds_read_b64 /
// ds_write_b64 moves an amplitude's (psi, lambda) pair: half the LDS instructions of two b32 accesses (the LDS
// issue rate, not bandwidth, bounds this kernel: PMC WAIT_INST_LDS), at a v_mov per dword splitting the pairs into
// MFMA operands.  (Separate psi / lambda planes halve the bank conflicts but double the LDS instructions: measured
// slower, round 3.)  Without a lambda input the lambda words are zeroed (the observable op writes them).
template <int NT, int TB>
__device__ __forceinline__ void load_tile_il(const PassArgs& a, const uint32_t* psrc, const uint32_t* lsrc,
                                             uint32_t* tile, int tid, int T, uint32_t h_q, uint32_t fixed) {
  constexpr int MQ = (1 << TB) / (4 * NT);
  uint4 v[MQ], l[MQ];
#pragma unroll
  for (int i = 0; i < MQ; ++i) {
    const uint32_t q = 4u * (tid + NT * i);
    if (q < (uint32_t)T) {
      v[i] = *(const uint4*)&psrc[mem_of(q, a, fixed)];
      l[i] = lsrc ? *(const uint4*)&lsrc[mem_of(q, a, fixed)] : make_uint4(0u, 0u, 0u, 0u);
    }
  }
#pragma unroll
  for (int i = 0; i < MQ; ++i) {
    const uint32_t q = 4u * (tid + NT * i);
    if (q < (uint32_t)T) {
      const uint32_t h = h_q ^ swz(a, (uint32_t)(4 * NT / 32) * i);
      const uint32_t w0 = (q ^ h) & ~3u;
      const uint4 pv = quad_perm(v[i], h & 3u), lv = quad_perm(l[i], h & 3u);
      *(uint4*)&tile[2 * w0] = make_uint4(pv.x, lv.x, pv.y, lv.y);
      *(uint4*)&tile[2 * w0 + 4] = make_uint4(pv.z, lv.z, pv.w, lv.w);
    }
  }
}

template <int NT, int TB>
__device__ __forceinline__ void store_lam_il(const PassArgs& a, uint32_t* dst, const uint32_t* tile, int tid, int T,
                                             uint32_t h_q, uint32_t fixed) {
  constexpr int MQ = (1 << TB) / (4 * NT);
  uint4 v[MQ];
#pragma unroll
  for (int i = 0; i < MQ; ++i) {
    const uint32_t q = 4u * (tid + NT * i);
    if (q < (uint32_t)T) {
      const uint32_t h = h_q ^ swz(a, (uint32_t)(4 * NT / 32) * i);
      const uint32_t w0 = 2u * ((q ^ h) & ~3u);
      const uint4 a0 = *(const uint4*)&tile[w0], a1 = *(const uint4*)&tile[w0 + 4];
      v[i] = quad_perm(make_uint4(a0.y, a0.w, a1.y, a1.w), h & 3u);
    }
  }
#pragma unroll
  for (int i = 0; i < MQ; ++i) {
    const uint32_t q = 4u * (tid + NT * i);
    if (q < (uint32_t)T) tile_st(&dst[mem_of(q, a, fixed)], v[i], a.nt_store);
  }
}

// RZ(ph) RX(th) F(x)|0> for a layer-1 qubit
__device__ __forceinline__ void l1_factor(float x, float th, float ph, int feature, float2* w) {
  float sa, ca;
  __sincosf(0.5f * x, &sa, &ca);
  float2 v0, v1;
  if (feature == 1) {          // rx
    v0 = make_float2(ca, 0.f);
    v1 = make_float2(0.f, -sa);
  } else if (feature == 2) {   // rz
    v0 = make_float2(ca, -sa);
    v1 = make_float2(0.f, 0.f);
  } else {                     // ry
    v0 = make_float2(ca, 0.f);
    v1 = make_float2(sa, 0.f);
  }
  float s, c;
  __sincosf(0.5f * th, &s, &c);
  // RX: w0 = c v0 - i s v1 ; w1 = -i s v0 + c v1      (-i z = (z.y, -z.x))
  float2 w0 = make_float2(c * v0.x + s * v1.y, c * v0.y - s * v1.x);
  float2 w1 = make_float2(c * v1.x + s * v0.y, c * v1.y - s * v0.x);
  float sp, cp;
  __sincosf(0.5f * ph, &sp, &cp);
  w[0] = cmul(w0, make_float2(cp, -sp));
  w[1] = cmul(w1, make_float2(cp, sp));
}

// LDS images, addressed by BYTE offsets that combine by XOR (each access is one XOR of per-lane constants):
//   forward: psi only, amplitude tau at byte 4 sigma(tau);
//   adjoint: psi and lambda interleaved, amplitude tau at bytes 8 sigma(tau) (psi) and 8 sigma(tau) + 4
//   (lambda).  Every adjoint access touches psi and lambda at the same amplitude, so they move as 8-byte
//   ds_read_b64 / ds_write_b64 pairs: twice the bytes of ds_read_b32 in the same LDS cycles, and one
//   6-cycle store instead of two 4-cycle ones.  The b64 read bank is (byte / 4) mod 64 per 32 lanes, i.e.
//   the pair index sigma(tau) mod 32, so the planner's conflict-free b32 swizzle stays conflict free.
__device__ __forceinline__ uint2 lds_ld2(const uint32_t* tile, uint32_t byte) {
  return *(const uint2*)((const char*)tile + byte);
}
__device__ __forceinline__ void lds_st2(uint32_t* tile, uint32_t byte, uint2 v) {
  *(uint2*)((char*)tile + byte) = v;
}

__device__ __forceinline__ uint32_t lds_ld(const uint32_t* tile, uint32_t byte) {
  return *(const uint32_t*)((const char*)tile + byte);
}
__device__ __forceinline__ void lds_st(uint32_t* tile, uint32_t byte, uint32_t v) {
  *(uint32_t*)((char*)tile + byte) = v;
}


// (int)floor(x + 0.5f) in one instruction (round half up; the compiler's rint + convert is two)
__device__ __forceinline__ int cvt_rpi(float x) {
  int r;
  __asm__("v_cvt_rpi_i32_f32 %0, %1" : "=v"(r) : "v"(x));
  return r;
}

// i * (re, im) = (-im, re) on a packed fp16 pair: dst.lo = src.hi * (-1), dst.hi = src.lo * 1
__device__ __forceinline__ uint32_t mul_i(uint32_t v) {
#if QFX_HEA_BF16
  // no packed bf16 multiply: swap the halves (rotate by 16) and flip the sign of the new low half
  return __builtin_amdgcn_alignbit(v, v, 16) ^ 0x00008000u;
#else
  uint32_t r;
  __asm__("v_pk_mul_f16 %0, %1, %2 op_sel:[1,0] op_sel_hi:[0,1]" : "=v"(r) : "v"(v), "s"(0x3C00BC00u));
  return r;
#endif
}

// Y = U X on the op's column blocks.  Lane (g4, cl) owns column cl of a 16-column block: it reads amplitudes
// m = 4 g4 .. 4 g4 + 3 (B operand, k = 2m + re/im) and writes the same amplitudes back (row 4 g4 + i of output tile
// 0 / 1 = re / im of m' = 4 g4 + i).  A wave's blocks are blk = wave + NW i (i < nbw <= MAXB, fully unrolled):
// (blk & 1) = (wave & 1), so the block bases are BL[lane] ^ BH[blk >> 1] precomputed in registers.  Blocks go in
// pairs (independent MFMA chains).
//   ADJ = false: forward psi image; the next pair's operands are read before the current pair is written.
//   ADJ = true : interleaved adjoint image, U applied to lambda only (a pass's last BACK op when psi is no longer
//                needed), plus the op's gradient cross matrix N = sum psi lambda^H from the SAME registers: an MFMA
//                against the constant identity fragments IRE / IIM (exact in fp16) transposes each block's psi and
//                lambda so the column index lands in registers - lane cl then holds (re, im) of amplitude cl for
//                columns 4 g4 .. 4 g4 + 3, packed as the K = 32 operand of one MFMA that sums over columns
//                (acc[0]: B = lambda, acc[1]: B = i lambda).  Accumulator layout as group_cross: lane (g4, cl)
//                holds N[4 g4 + i][cl].
template <int NW, bool ADJ, int TB = TMAX>
__device__ __forceinline__ void group_apply(uint32_t* tile, const uint4* F, const int* opw, uint32_t fo, int lane,
                                            int wave, int nbw, f4* acc = nullptr) {
  constexpr int MAXB = (1 << (TB - 8)) / NW;   // column blocks per wave per op (t = 14: 64 blocks)
  constexpr int NL = ADJ ? 2 : 1;              // registers loaded per block: psi and lambda for the cross
  constexpr int SH = ADJ ? 3 : 2;
  const int g4 = lane >> 4, cl = lane & 15;
  uint32_t oin[4];
#pragma unroll
  for (int jj = 0; jj < 4; ++jj) oin[jj] = ((uint32_t)opw[W_OFF + 4 * g4 + jj] ^ fo) << SH;
  // identity fragments (rows: re of amplitude n, then im), built here from an opaque copy of the lane index so the
  // compiler cannot hoist them out of the kernel's op loop (hoisted, they were spilled to scratch there)
  uint4 IRE = {}, IIM = {};
  if constexpr (ADJ) {
    int ln = lane;
    __asm__ volatile("" : "+v"(ln));
    const int dg = (ln & 15) - 4 * (ln >> 4);
    uint32_t* re = (uint32_t*)&IRE;
    uint32_t* im = (uint32_t*)&IIM;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      re[j] = dg == j ? ONE_LO : 0u;
      im[j] = dg == j ? ONE_HI : 0u;
    }
  }
  const uint32_t bl = (uint32_t)opw[W_BL + (wave & 1) * 16 + cl];
  uint32_t base[MAXB];
#pragma unroll
  for (int i = 0; i < MAXB; ++i) base[i] = (bl ^ (uint32_t)opw[W_BH + ((wave + NW * i) >> 1)]) << SH;
  auto load = [&](uint32_t b, uint4* X) {
    const uint32_t a0 = b ^ oin[0], a1 = b ^ oin[1], a2 = b ^ oin[2], a3 = b ^ oin[3];
    if constexpr (ADJ) {
      const uint2 p0 = lds_ld2(tile, a0), p1 = lds_ld2(tile, a1), p2 = lds_ld2(tile, a2), p3 = lds_ld2(tile, a3);
      X[0] = make_uint4(p0.x, p1.x, p2.x, p3.x);
      X[1] = make_uint4(p0.y, p1.y, p2.y, p3.y);
    } else {
      X[0] = make_uint4(lds_ld(tile, a0), lds_ld(tile, a1), lds_ld(tile, a2), lds_ld(tile, a3));
    }
  };
  auto compute_store = [&](uint32_t b, const uint4* XL) {
    const f4 z = {0.f, 0.f, 0.f, 0.f};
    if constexpr (ADJ) {
      const f4 pr = mfma(XL[0], IRE, z), pi = mfma(XL[0], IIM, z), lr = mfma(XL[1], IRE, z), li = mfma(XL[1], IIM, z);
      const uint4 A = make_uint4(pack_h2(pr[0], pi[0]), pack_h2(pr[1], pi[1]), pack_h2(pr[2], pi[2]), pack_h2(pr[3], pi[3]));
      const uint4 Br = make_uint4(pack_h2(lr[0], li[0]), pack_h2(lr[1], li[1]), pack_h2(lr[2], li[2]), pack_h2(lr[3], li[3]));
#if QFX_HEA_BF16   // i lambda = (-im, re) packed straight from fp32 (rounding is sign symmetric: exactly i Br)
      const uint4 Bi = make_uint4(pack_h2(-li[0], lr[0]), pack_h2(-li[1], lr[1]), pack_h2(-li[2], lr[2]), pack_h2(-li[3], lr[3]));
#else
      const uint4 Bi = make_uint4(mul_i(Br.x), mul_i(Br.y), mul_i(Br.z), mul_i(Br.w));
#endif
      acc[0] = mfma(A, Br, acc[0]);
      acc[1] = mfma(A, Bi, acc[1]);
    }
    const uint4 X = XL[NL - 1];                   // the apply target: psi (forward) or lambda (adjoint)
    f4 d0 = mfma(F[0], X, z), d1 = mfma(F[1], X, z);
    if (QFX_HEA_GATE_LO) {
      d0 = mfma(F[2], X, d0);
      d1 = mfma(F[3], X, d1);
    }
    // output amplitude 4 g4 + i = (tile 0, tile 1) register i, written where it was read (adjoint: the lambda word)
#pragma unroll
    for (int i = 0; i < 4; ++i) lds_st(tile, (b ^ oin[i]) ^ (ADJ ? 4u : 0u), pack_h2(d0[i], d1[i]));
  };
  if (nbw <= 0) return;
  uint4 B0[NL], B1[NL];
  load(base[0], B0);
  if (nbw > 1) load(base[1], B1);
  constexpr bool PREFETCH = !ADJ;               // the fused cross needs the registers of the prefetched pair
#pragma unroll
  for (int p = 0; p < MAXB; p += 2) {
    if (p >= nbw) break;
    uint4 C0[NL], C1[NL];
    if (PREFETCH && p + 2 < MAXB && p + 2 < nbw) {
      load(base[p + 2 < MAXB ? p + 2 : 0], C0);
      if (p + 3 < nbw) load(base[p + 3 < MAXB ? p + 3 : 0], C1);
    }
    compute_store(base[p], B0);
    if (p + 1 < nbw) compute_store(base[p + 1 < MAXB ? p + 1 : 0], B1);
    if (PREFETCH) {
#pragma unroll
      for (int x = 0; x < NL; ++x) {
        B0[x] = C0[x];
        B1[x] = C1[x];
      }
    } else if (p + 2 < MAXB && p + 2 < nbw) {
      load(base[p + 2 < MAXB ? p + 2 : 0], B0);
      if (p + 3 < nbw) load(base[p + 3 < MAXB ? p + 3 : 0], B1);
    }
  }
}

// Gradient cross matrix N[b][a] += sum_col psi[b][col] conj(lam[a][col]) over the op's column blocks:
// K = 16 columns x (re, im), lane (g4, cl) reads amplitude m = cl of columns 4 g4 .. 4 g4 + 3; accR / accI
// end up holding N[4 g4 + i][cl] (real / imaginary).
template <int NW, int TB = TMAX>
__device__ __forceinline__ void group_cross(const uint32_t* tile, const int* opw, uint32_t fo, int lane, int wave,
                                            int nbw, f4& accR, f4& accI) {
  constexpr int MAXB = (1 << (TB - 8)) / NW;
  const int g4 = lane >> 4, cl = lane & 15;
  const uint32_t om = (uint32_t)opw[W_OFF + cl] ^ fo;
  uint32_t gb[4];
#pragma unroll
  for (int jj = 0; jj < 4; ++jj) gb[jj] = ((uint32_t)opw[W_BL + (wave & 1) * 16 + 4 * g4 + jj] ^ om) << 3;
#pragma unroll
  for (int i = 0; i < MAXB; ++i) {
    if (i >= nbw) break;
    const uint32_t bh = (uint32_t)opw[W_BH + ((wave + NW * i) >> 1)] << 3;
    uint32_t pv[4], lv[4];
#pragma unroll
    for (int jj = 0; jj < 4; ++jj) {            // psi and lambda of one amplitude: one b64 pair
      const uint2 v = lds_ld2(tile, gb[jj] ^ bh);
      pv[jj] = v.x;
      lv[jj] = v.y;
    }
    const uint4 A = make_uint4(pv[0], pv[1], pv[2], pv[3]);
    const uint4 Br = make_uint4(lv[0], lv[1], lv[2], lv[3]);
    // i*lam: (re, im) -> (-im, re), one v_pk_mul_f16 per dword (exact: a product with +-1)
    const uint4 Bi = make_uint4(mul_i(lv[0]), mul_i(lv[1]), mul_i(lv[2]), mul_i(lv[3]));
    accR = mfma(A, Br, accR);
    accI = mfma(A, Bi, accI);
  }
}

// Transposed BACK op (F_BACK_TRANS): psi_in = U^H psi_out and lambda_in = U^H lambda_out as Y^T = X^T M^T, the
// state block as the A operand and the U^H fragments as the B operand (the fragment registers of M are the B
// layout of M^T).  The A registers are the ones the U-as-A form reads (lane (g4, cl): column cl, amplitudes
// 4 g4 .. 4 g4 + 3), and the result lands transposed: lane (g4, cl) holds amplitude m' = cl of columns 4 g4 + i
// in register i, re in tile 0 and im in tile 1 (fragment rows (component, m')).  That is the operand layout of the
// cross-matrix MFMA (K = columns), so the op's gradient cross matrix is taken at its INPUT,
// N = sum_col psi_in lambda_in^H, from the rounded results themselves: per block 8 apply + 2 cross MFMAs and no
// transposes (the output-side fused form needs 4 identity-MFMA transposes and their packs), and
// hea_grad_reduce applies the input-side generators (X, and RX^H Z RX = cos(theta) Z + sin(theta) Y).  The
// results go back amplitude-major: lane (g4, cl) writes amplitude cl of columns 4 g4 .. 4 g4 + 3, one 16-lane
// b64 store group = 16 amplitudes of one column (the planner keeps their pair banks distinct).
template <int NW, int TB>
__device__ __forceinline__ void group_back_t(uint32_t* tile, const uint4* F, const int* opw, uint32_t fo, int lane,
                                             int wave, int nbw, f4* acc) {
  constexpr int MAXB = (1 << (TB - 8)) / NW;
  constexpr int SH = 3;
  const int g4 = lane >> 4, cl = lane & 15;
  // load address of block i, amplitude 4 g4 + j: lo[j] ^ bh[i]; store address of column 4 g4 + r: ost[r] ^ bh[i]
  uint32_t lo[4], ost[4], bh[MAXB];
  const uint32_t om = (uint32_t)opw[W_OFF + cl] ^ fo, bl = (uint32_t)opw[W_BL + (wave & 1) * 16 + cl] ^ fo;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    lo[j] = ((uint32_t)opw[W_OFF + 4 * g4 + j] ^ bl) << SH;
    ost[j] = ((uint32_t)opw[W_BL + (wave & 1) * 16 + 4 * g4 + j] ^ om) << SH;
  }
#pragma unroll
  for (int i = 0; i < MAXB; ++i) bh[i] = (uint32_t)opw[W_BH + ((wave + NW * i) >> 1)] << SH;
  auto load = [&](int i, uint4* X) {
    const uint32_t b = bh[i];
    const uint2 p0 = lds_ld2(tile, b ^ lo[0]), p1 = lds_ld2(tile, b ^ lo[1]), p2 = lds_ld2(tile, b ^ lo[2]),
                p3 = lds_ld2(tile, b ^ lo[3]);
    X[0] = make_uint4(p0.x, p1.x, p2.x, p3.x);
    X[1] = make_uint4(p0.y, p1.y, p2.y, p3.y);
  };
  auto compute_store = [&](int i, const uint4* X) {
    const f4 z = {0.f, 0.f, 0.f, 0.f};
    f4 pr = mfma(X[0], F[0], z);
    f4 pi = mfma(X[0], F[1], z);
    f4 lr = mfma(X[1], F[0], z);
    f4 li = mfma(X[1], F[1], z);
    if (QFX_HEA_GATE_LO) {
      pr = mfma(X[0], F[2], pr);
      pi = mfma(X[0], F[3], pi);
      lr = mfma(X[1], F[2], lr);
      li = mfma(X[1], F[3], li);
    }
    // (re, im) of amplitude cl, columns 4 g4 + r: the stored values, the cross matrix's A (psi) and B (lambda,
    // i lambda = (-im, re): exactly i times the rounded lambda, rounding is sign symmetric)
    const uint4 P = make_uint4(pack_h2(pr[0], pi[0]), pack_h2(pr[1], pi[1]), pack_h2(pr[2], pi[2]), pack_h2(pr[3], pi[3]));
    const uint4 Lr = make_uint4(pack_h2(lr[0], li[0]), pack_h2(lr[1], li[1]), pack_h2(lr[2], li[2]), pack_h2(lr[3], li[3]));
#if QFX_HEA_BF16   // i lambda = (-im, re) packed straight from fp32 (one cvt; the bf16 mul_i is two instructions)
    const uint4 Li = make_uint4(pack_h2(-li[0], lr[0]), pack_h2(-li[1], lr[1]), pack_h2(-li[2], lr[2]), pack_h2(-li[3], lr[3]));
#else              // (the packed form pushed the fp16 kernels' register allocation into spills)
    const uint4 Li = make_uint4(mul_i(Lr.x), mul_i(Lr.y), mul_i(Lr.z), mul_i(Lr.w));
#endif
    acc[0] = mfma(P, Lr, acc[0]);
    acc[1] = mfma(P, Li, acc[1]);
    const uint32_t bb = bh[i];
    const uint32_t* Pw = (const uint32_t*)&P;
    const uint32_t* Lw = (const uint32_t*)&Lr;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      // psi and lambda words from two unpaired registers in one ds_write2_b32 (a b64 store needs them adjacent,
      // and the cross-matrix operands need each of psi and lambda in four adjacent registers: the compiler merges
      // two dword stores into a b64 with two v_movs).  Issued as asm, the store is unknown to the wait-count pass;
      // LDS operations complete in order, so its waits only become conservative.
      const uint32_t la = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) char*)((char*)tile + (ost[r] ^ bb));
      __asm__ volatile("ds_write2_b32 %0, %1, %2 offset1:1" ::"v"(la), "v"(Pw[r]), "v"(Lw[r]) : "memory");
    }
  };
  // one block at a time with the next block's reads in flight (four independent MFMA chains per block; a pair of
  // blocks plus the next pair's operands pushed the kernel past 128 VGPRs into spills)
  if (nbw <= 0) return;
  uint4 Bc[2];
  load(0, Bc);
#pragma unroll
  for (int i = 0; i < MAXB; ++i) {
    if (i >= nbw) break;
    uint4 Bn[2];
    if (i + 1 < MAXB && i + 1 < nbw) load(i + 1 < MAXB ? i + 1 : 0, Bn);
    compute_store(i, Bc);
    Bc[0] = Bn[0];
    Bc[1] = Bn[1];
  }
}

// An op's unitary fragments go to an LDS slot by direct global -> LDS DMA (global_load_lds_dwordx4, 1 KB per
// wave-instruction), issued one op ahead by wave 0 alone: no VGPRs are held for the prefetch, and the other waves
// never wait on vector memory at an op barrier (the wave that flushes gradient partials to the slab must not wait
// for those stores there).  Only the re rows (hi and lo halves, 2 KB per group) travel: the im rows of the real
// embedding are i times them per (re, im) word (frag_regs).  A pair op's second group fills the slot's upper half.
// The LDS base of a wave-instruction is wave-uniform (M0); the DMA is complete once wave 0 has passed
// s_waitcnt vmcnt(0) (op_barrier).
__device__ __forceinline__ void dma_frags(const PassArgs& a, int k, const int* fi, int lane, int wave, uint4* slot) {
  if (wave != 0) return;
#pragma unroll
  for (int g = 0; g < 2; ++g) {
    if (fi[g] < 0) continue;
    const uint4* fr = (const uint4*)a.frags + ((size_t)(a.frag_shared ? 0 : k) * a.n_slots * 4 + fi[g]) * 128 + lane;
    // Issued as inline asm: the compiler's wait-count pass cannot tell which LDS bytes a builtin DMA writes (no
    // alias scopes reach codegen), so it waited for the DMA before the op's first LDS store or atomic and exposed
    // the fragment latency in every op.  The slot is only read after op_barrier's vmcnt(0) + barrier, and a
    // vector-memory op unknown to the pass can only make its other waits longer, never shorter.
#pragma unroll
    for (int j = 0; j < 2; ++j) {                 // hi re rows (f), lo re rows (f + 1: 128 uint4 further)
      const uint32_t lds = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) uint4*)(slot + 128 * g + 64 * j);
      // s_nop: an LDS DMA reads M0 one wait state after an SALU write of it (the compiler's hazard recognizer does
      // not look inside this asm statement)
      __asm__ volatile("s_mov_b32 m0, %1\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %0, off" ::"v"(fr + 128 * j),
                       "s"(__builtin_amdgcn_readfirstlane(lds))
                       : "memory", "m0");
    }
  }
}

// Fragment registers of group g of the slot: F[0] / F[2] = hi / lo re rows, F[1] / F[3] = hi / lo im rows.  Row
// (re, m') of the real 32 x 32 embedding holds (Re U, -Im U) per (re, im) column pair, row (im, m') (Im U, Re U): the
// im row's word is i times the re row's word, exactly (a sign flip and a swap; hi / lo halves alike).
__device__ __forceinline__ void frag_regs(const uint4* slot, int g, int lane, uint4* F) {
  F[0] = slot[128 * g + lane];
  F[2] = slot[128 * g + 64 + lane];
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const uint4 v = F[2 * h];
    F[2 * h + 1] = make_uint4(mul_i(v.x), mul_i(v.y), mul_i(v.z), mul_i(v.w));
  }
}

// ------------------------------------------------------------------------------------------- chained pair ops
// A block is one coset of span(X, Y) in the tile: 256 amplitudes at  base ^ OFF_X[x] ^ OFF_Y[y] ^ fo.  Lane
// (g4, cl) first holds (x = 4 g4 + j, y = cl) in register j - the operand layout of X's product over x with y as the
// column.  X runs in the TRANSPOSED form (state block as the A operand, fragments as B): the result lands with the
// lane holding x = cl for y = 4 g4 + i in register i, which is exactly the operand layout of Y's product over y with x
// as the column.  So the pair's second product needs no data movement at all: one LDS read and one write of the
// coset per pair (and one op barrier), against two of each for two single ops.  The state is rounded to the
// storage type between the two products, as the LDS store between two single ops rounds it.

// Per-lane address words of a pair op (byte offsets, SH = log2 bytes per amplitude image entry):
//   xa[j] = (x = 4 g4 + j, y = cl),   ya[j] = (x = cl, y = 4 g4 + j)
template <int SH>
__device__ __forceinline__ void pair_addrs(const int* opw, uint32_t fo, int lane, uint32_t* xa, uint32_t* ya) {
  const int g4 = lane >> 4, cl = lane & 15;
  const uint32_t ox = (uint32_t)opw[W_OFF + cl], oy = (uint32_t)opw[W_OFF2 + cl];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    xa[j] = ((uint32_t)opw[W_OFF + 4 * g4 + j] ^ oy ^ fo) << SH;
    ya[j] = (ox ^ (uint32_t)opw[W_OFF2 + 4 * g4 + j] ^ fo) << SH;
  }
}

// block blk's coset base (byte offset)
template <int SH>
__device__ __forceinline__ uint32_t pair_base(const int* opw, int blk) {
  return ((uint32_t)opw[W_BL + (blk & 31)] ^ (uint32_t)opw[W_BH + (blk >> 5)]) << SH;
}

__device__ __forceinline__ uint4 pack4(const f4& re, const f4& im) {
  return make_uint4(pack_h2(re[0], im[0]), pack_h2(re[1], im[1]), pack_h2(re[2], im[2]), pack_h2(re[3], im[3]));
}

// Forward pair: Y U_Y (U_X X) on the psi image.  Read at (x = 4 g4 + j, y = cl), written at (x = cl, y = 4 g4 + i).
// A wave owns blocks blk = wave + NW i; the next block's reads are issued before the current block computes (all of
// a block's addresses belong to its coset, so blocks are disjoint).
template <int NW, int TB>
__device__ __forceinline__ void group_pair_fwd(uint32_t* tile, const uint4* FX, const uint4* FY, const int* opw,
                                               uint32_t fo, int lane, int wave, int nbw) {
  constexpr int MAXB = (1 << (TB - 8)) / NW;
  uint32_t xa[4], ya[4];
  pair_addrs<2>(opw, fo, lane, xa, ya);
  auto load = [&](int i) {
    const uint32_t b = pair_base<2>(opw, wave + NW * i);
    return make_uint4(lds_ld(tile, b ^ xa[0]), lds_ld(tile, b ^ xa[1]), lds_ld(tile, b ^ xa[2]), lds_ld(tile, b ^ xa[3]));
  };
  if (nbw <= 0) return;
  uint4 X = load(0);
#pragma unroll
  for (int i = 0; i < MAXB; ++i) {
    if (i >= nbw) break;
    uint4 Xn = X;
    if (i + 1 < MAXB && i + 1 < nbw) Xn = load(i + 1 < MAXB ? i + 1 : 0);
    const f4 z = {0.f, 0.f, 0.f, 0.f};
    f4 pr = mfma(X, FX[0], z), pi = mfma(X, FX[1], z);          // X transposed: lane holds x = cl, y = 4 g4 + r
    if (QFX_HEA_GATE_LO) {
      pr = mfma(X, FX[2], pr);
      pi = mfma(X, FX[3], pi);
    }
    const uint4 P = pack4(pr, pi);
    f4 d0 = mfma(FY[0], P, z), d1 = mfma(FY[1], P, z);           // Y over y, column x = cl
    if (QFX_HEA_GATE_LO) {
      d0 = mfma(FY[2], P, d0);
      d1 = mfma(FY[3], P, d1);
    }
    const uint32_t b = pair_base<2>(opw, wave + NW * i);
#pragma unroll
    for (int r = 0; r < 4; ++r) lds_st(tile, b ^ ya[r], pack_h2(d0[r], d1[r]));
    X = Xn;
  }
}

// Adjoint pair: U_X^H then U_Y^H on psi and lambda (interleaved image), both transposed, each op's gradient cross
// matrix taken from its rounded results (the op input side, as group_back_t): acc[0..1] for X, acc[2..3] for Y.  Read
// and written at the same addresses (x = 4 g4 + j, y = cl): after Y the lane holds y = cl for x = 4 g4 + r.
template <int NW, int TB>
__device__ __forceinline__ void group_pair_back(uint32_t* tile, const uint4* FX, const uint4* FY, const int* opw,
                                                uint32_t fo, int lane, int wave, int nbw, f4* acc) {
  constexpr int MAXB = (1 << (TB - 8)) / NW;
  uint32_t xa[4], ya[4];
  pair_addrs<3>(opw, fo, lane, xa, ya);
  auto load = [&](int i, uint4* X) {
    const uint32_t b = pair_base<3>(opw, wave + NW * i);
    const uint2 p0 = lds_ld2(tile, b ^ xa[0]), p1 = lds_ld2(tile, b ^ xa[1]), p2 = lds_ld2(tile, b ^ xa[2]),
                p3 = lds_ld2(tile, b ^ xa[3]);
    X[0] = make_uint4(p0.x, p1.x, p2.x, p3.x);
    X[1] = make_uint4(p0.y, p1.y, p2.y, p3.y);
  };
  // one transposed un-apply of both states + the cross matrix of the results.  The im-row fragments are formed
  // here from the re rows (frag_regs' identity, 4 VALU each): two groups' full fragment sets held across the block
  // loop pushed the kernel past 128 VGPRs into scratch.
  auto imrow = [](uint4 v) {        // opaque copy first: hoisted out of the block loop, the im rows stay live again
    __asm__ volatile("" : "+v"(v.x), "+v"(v.y), "+v"(v.z), "+v"(v.w));
    return make_uint4(mul_i(v.x), mul_i(v.y), mul_i(v.z), mul_i(v.w));
  };
  auto back = [&](const uint4& Ps, const uint4& Ls, const uint4* F, f4* ac, uint4& Po, uint4& Lo) {
    const f4 z = {0.f, 0.f, 0.f, 0.f};
    uint4 Fi = imrow(F[0]);
    f4 pr = mfma(Ps, F[0], z), pi = mfma(Ps, Fi, z), lr = mfma(Ls, F[0], z), li = mfma(Ls, Fi, z);
    if (QFX_HEA_GATE_LO) {
      Fi = imrow(F[2]);
      pr = mfma(Ps, F[2], pr);
      pi = mfma(Ps, Fi, pi);
      lr = mfma(Ls, F[2], lr);
      li = mfma(Ls, Fi, li);
    }
    Po = pack4(pr, pi);
    Lo = pack4(lr, li);
#if QFX_HEA_BF16
    const uint4 Li = make_uint4(pack_h2(-li[0], lr[0]), pack_h2(-li[1], lr[1]), pack_h2(-li[2], lr[2]), pack_h2(-li[3], lr[3]));
#else
    const uint4 Li = make_uint4(mul_i(Lo.x), mul_i(Lo.y), mul_i(Lo.z), mul_i(Lo.w));
#endif
    ac[0] = mfma(Po, Lo, ac[0]);
    ac[1] = mfma(Po, Li, ac[1]);
  };
  if (nbw <= 0) return;
  uint4 Xc[2];
  load(0, Xc);
#pragma unroll
  for (int i = 0; i < MAXB; ++i) {
    if (i >= nbw) break;
    uint4 P1, L1, P2, L2;
    back(Xc[0], Xc[1], FX, acc, P1, L1);
    // the next block's reads go into the registers X's products have just consumed (a separate prefetch set pushed
    // the kernel past 128 VGPRs into scratch); they stay in flight during Y's products and the writes
    if (i + 1 < MAXB && i + 1 < nbw) load(i + 1 < MAXB ? i + 1 : 0, Xc);
    back(P1, L1, FY, acc + 2, P2, L2);
    const uint32_t b = pair_base<3>(opw, wave + NW * i);
    const uint32_t* Pw = (const uint32_t*)&P2;
    const uint32_t* Lw = (const uint32_t*)&L2;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      // (psi, lambda) of one amplitude from two unpaired registers in one ds_write2_b32 (as group_back_t)
      const uint32_t la = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) char*)((char*)tile + (b ^ xa[r]));
      __asm__ volatile("ds_write2_b32 %0, %1, %2 offset1:1" ::"v"(la), "v"(Pw[r]), "v"(Lw[r]) : "memory");
    }
  }
}

// Cross-matrix-only pair (layer-1 gradient groups): N_X from the reads at (x = cl, y = 4 g4 + j) (columns y in K),
// N_Y from (x = 4 g4 + j, y = cl); read-only, so both address patterns read the same coset with no barrier between.
template <int NW, int TB>
__device__ __forceinline__ void group_pair_cross(const uint32_t* tile, const int* opw, uint32_t fo, int lane, int wave,
                                                 int nbw, f4* acc) {
  constexpr int MAXB = (1 << (TB - 8)) / NW;
  uint32_t xa[4], ya[4];
  pair_addrs<3>(opw, fo, lane, xa, ya);
#pragma unroll
  for (int i = 0; i < MAXB; ++i) {
    if (i >= nbw) break;
    const uint32_t b = pair_base<3>(opw, wave + NW * i);
#pragma unroll
    for (int g = 0; g < 2; ++g) {
      const uint32_t* ad = g == 0 ? ya : xa;
      uint32_t pv[4], lv[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const uint2 v = lds_ld2(tile, b ^ ad[j]);
        pv[j] = v.x;
        lv[j] = v.y;
      }
      const uint4 A = make_uint4(pv[0], pv[1], pv[2], pv[3]);
      const uint4 Br = make_uint4(lv[0], lv[1], lv[2], lv[3]);
      const uint4 Bi = make_uint4(mul_i(lv[0]), mul_i(lv[1]), mul_i(lv[2]), mul_i(lv[3]));
      acc[2 * g] = mfma(A, Br, acc[2 * g]);
      acc[2 * g + 1] = mfma(A, Bi, acc[2 * g + 1]);
    }
  }
}

// Readout / observable ops walk the tile words w = tid + NT i (i < T / NT).  The sign of class c at word w is
// parity(w & om[c]) ^ parity(fixed & of[c]): a per-thread part (tid bits) and a wave-uniform part (NT i bits,
// scalar).  The words are read in chunks of RCH with every read of a chunk issued before the first use (one
// LDS wait per chunk instead of one per word), and NC, the class count, is a template parameter so the class
// loop has no per-word branches.  Reads are never predicated (a predicated read serialises on the mask
// register): words past the tile wrap to in-bounds addresses and their contributions are masked.
constexpr int RCH = 8;

// Per-op class sign state, kept small in scalar registers (this kernel runs at the SGPR limit, and the class
// masks are dead after setup): words w = tid + NT (i0 + j), i0 = k CH a chunk start, j < CH, have the sign
//   parity(tid & om_c) ^ parity(fixed & of_c)   per lane    -> bit c of sgn0 (VGPR)
// ^ parity(NT k CH & om_c)                       per chunk   -> bit k NC + c of fu (one SGPR)
// ^ parity(NT j & om_c)                          per word    -> bit j NC + c of jb (two SGPRs)
// The word part becomes a +-1 table in registers (0 for words past a partial tile) while NC x CH <= 32.
template <int NC, int CH>
struct ClassSigns {
  static constexpr bool TAB = NC * CH <= 32;
  uint32_t sgn0;
  uint32_t fu;
  uint64_t jb;
  int iters;
  float f[TAB ? CH : 1][TAB ? NC : 1];
  __device__ __forceinline__ bool flip(int c, int k) const { return (((sgn0 >> c) ^ (fu >> (k * NC + c))) & 1u) != 0u; }
  __device__ __forceinline__ float mul(float x, int j, int c) const {
    if constexpr (TAB) return x * f[j][c];
    return j < iters ? (((jb >> (j * NC + c)) & 1u) ? -x : x) : 0.f;
  }
};

template <int NC, int NT, int CH, int TB = TMAX>
__device__ __forceinline__ ClassSigns<NC, CH> class_signs(const int* opw, int tid, uint32_t fixed, int iters) {
  constexpr int QI = (1 << TB) / NT;
  static_assert((QI / CH) * NC <= 32 && CH * NC <= 64, "class sign masks must fit one / two dwords");
  ClassSigns<NC, CH> cs;
  cs.sgn0 = 0;
  cs.fu = 0;
  cs.jb = 0;
  cs.iters = iters;
#pragma unroll
  for (int c = 0; c < NC; ++c) {
    const uint32_t om = (uint32_t)__builtin_amdgcn_readfirstlane(opw[W_OFF + c]);
    const uint32_t of = (uint32_t)__builtin_amdgcn_readfirstlane(opw[W_RFULL + 2 * c]);
    cs.sgn0 |= (uint32_t)(par((uint32_t)tid & om) ^ par(fixed & of)) << c;
#pragma unroll
    for (int k = 0; k < QI / CH; ++k) cs.fu |= (uint32_t)par((uint32_t)(NT * CH * k) & om) << (k * NC + c);
#pragma unroll
    for (int j = 0; j < CH; ++j) cs.jb |= (uint64_t)par((uint32_t)(NT * j) & om) << (j * NC + c);
  }
  if constexpr (ClassSigns<NC, CH>::TAB) {
#pragma unroll
    for (int j = 0; j < CH; ++j)
#pragma unroll
      for (int c = 0; c < NC; ++c) cs.f[j][c] = j < iters ? (((cs.jb >> (j * NC + c)) & 1u) ? -1.f : 1.f) : 0.f;
  }
  return cs;
}

// <Z_c> partial sums of the tile (forward image: one fp16 (re, im) word per amplitude).
template <int NC, int NT>
__device__ __forceinline__ void readout_op(const uint32_t* psi_t, const PassArgs& a, const int* opw, int tid,
                                           int lane, int wave, int T, uint32_t fixed, float* red, size_t pidx) {
  constexpr int QI = (1 << TMAX) / NT, NW = NT / 64;
  constexpr int CH = QI < RCH ? QI : RCH;
  const int iters = T >= NT ? T / NT : 1;
  const ClassSigns<NC, CH> cs = class_signs<NC, NT, CH>(opw, tid, fixed, iters);
  float acc[NC];
#pragma unroll
  for (int c = 0; c < NC; ++c) acc[c] = 0.f;
#pragma unroll 1
  for (int i0 = 0; i0 < QI; i0 += CH) {
    if (i0 >= iters) break;
    uint32_t v[CH];
#pragma unroll
    for (int j = 0; j < CH; ++j) v[j] = psi_t[(tid + NT * (i0 + j)) & (T - 1)];   // in bounds; masked by the sign table
    float sum[NC];
#pragma unroll
    for (int c = 0; c < NC; ++c) sum[c] = 0.f;
#pragma unroll
    for (int j = 0; j < CH; ++j) {
      const float p = norm2_h2(v[j]);
#pragma unroll
      for (int c = 0; c < NC; ++c) sum[c] += cs.mul(p, j, c);
    }
#pragma unroll
    for (int c = 0; c < NC; ++c) acc[c] += cs.flip(c, i0 / CH) ? -sum[c] : sum[c];
  }
#pragma unroll
  for (int c = 0; c < NC; ++c) {
    float v = tid < T ? acc[c] : 0.f;     // T < NT: lanes past the tile read wrapped words
    for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
    if (lane == 0) red[wave * CMAX + c] = v;
  }
  lds_barrier();
  if (tid < a.C) {
    float v = 0.f;
    for (int w = 0; w < NW; ++w) v += red[w * CMAX + tid];
    a.part[pidx + tid] = v / (a.scale * a.scale);
  }
}

// Adjoint seed lambda = sum_c r_c Z_c psi on the interleaved adjoint image (psi word 2w, lambda word 2w + 1).
template <int NC, int NT, int TB = TMAX>
__device__ __forceinline__ void obs_op(uint32_t* tile, const int* opw, int tid, int T, uint32_t fixed,
                                       const float* rsc_s) {
  constexpr int QI = (1 << TB) / NT;
  constexpr int CH = QI < RCH ? QI : RCH;
  const int iters = T >= NT ? T / NT : 1;
  const ClassSigns<NC, CH> cs = class_signs<NC, NT, CH, TB>(opw, tid, fixed, iters);
  float r[NC];
#pragma unroll
  for (int c = 0; c < NC; ++c) r[c] = rsc_s[c];
#pragma unroll 1
  for (int i0 = 0; i0 < QI; i0 += CH) {
    if (i0 >= iters) break;
    uint32_t v[CH];
#pragma unroll
    for (int j = 0; j < CH; ++j) v[j] = tile[2 * ((tid + NT * (i0 + j)) & (T - 1))];   // in bounds
    float rr[NC];
#pragma unroll
    for (int c = 0; c < NC; ++c) rr[c] = cs.flip(c, i0 / CH) ? -r[c] : r[c];
#pragma unroll
    for (int j = 0; j < CH; ++j) {
      float fsum = 0.f;
#pragma unroll
      for (int c = 0; c < NC; ++c) fsum += cs.mul(rr[c], j, c);
      const float2 f = unpack_h2(v[j]);
      const int w = tid + NT * (i0 + j);
      if (i0 + j < iters && w < T) tile[2 * w + 1] = pack_h2(fsum * f.x, fsum * f.y);
    }
  }
}

// Class-count specialisations of the pass kernel: NCK >= C classes (1, 2, 3, 4 or 8).  Classes C..NCK-1 are
// inert padding (zero observable masks, zero adjoint weights, no readout output).  One kernel per count, not a
// switch inside one kernel: the arms of such a switch keep their uniform values live across the op loop and
// push this kernel, which runs at the SGPR limit, into spilling scalars inside the group-op loops.
__host__ __device__ constexpr int class_kernel(int C) { return C <= 4 ? C : 8; }

// This wave's own LDS operations complete (no workgroup barrier).
__device__ __forceinline__ void lds_barrier_wave() { __asm__ volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); }


// Op barrier: wave 0 (the fragment DMA) and waves 0..1 (the next op record's global load, tid < OPW) wait for their
// vector memory; every other wave only for its LDS operations.  A wave that stored gradient partials to the slab
// (or anything else) thus never waits for those stores' completion at a barrier (each store stays counted in
// vmcnt for ~1-3K cycles under load).
__device__ __forceinline__ void op_barrier(int wave) {
  if (wave < 2) __asm__ volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __asm__ volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
}

// Memory bits of tile tile_id outside the tile.
__device__ __forceinline__ uint32_t tile_fixed(const PassArgs& a, int tile_id) {
  const int w1 = a.lo - a.c;
  return ((uint32_t)(tile_id & ((1 << w1) - 1)) << a.c) | ((uint32_t)(tile_id >> w1) << a.hi);
}

// The op's OFF base for the tile's fixed bits (their parities with the op's frame row masks).  The kernels read it from
// the host table (PassArgs::fo_tab, hea_plan.fo_table: one load per op); the debug build checks the table against this.
// Computed in the kernel it was a dependent chain of record loads on wave 0 before its share of the tile load (stall
// table, round 5: wave 0's prologue 5-10K cycles against < 1K for the other waves, every wave waiting at the first
// barrier).
__device__ __forceinline__ uint32_t op_fo_global(const int* ow, uint32_t fixed) {
  const int code = ow[W_CODE];
  if (code == OP_OBS || code == OP_READOUT) return 0u;
  const bool pair = code == OP_APPLY2 || code == OP_BACK2 || code == OP_GRAD2;
  const int nreal = ow[W_NREAL];
  int fpb = 0, fpy = 0;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    if (j < nreal) fpb |= par(fixed & (uint32_t)ow[W_RFULL + j]) << j;
    if (pair) fpy |= par(fixed & (uint32_t)ow[W_RFULL2 + j]) << j;
  }
  // a pair's OFF tables are linear: one word for both groups' fixed-bit offsets
  return (uint32_t)ow[W_OFF + fpb] ^ (pair ? (uint32_t)ow[W_OFF2 + fpy] : 0u);
}

// ------------------------------------------------------------------------------------------- forward pass
// One workgroup per tile of 2^t <= 2^14 amplitudes: 8 waves and 64 KB of LDS, so two workgroups share a CU and
// one's tile load overlaps the other's group ops (minimum waves per SIMD 4: <= 128 VGPRs).
template <int NCK, bool FULL>
__device__ __forceinline__ void fwd_pass(const PassArgs& a, int bid) {
  constexpr int NT = NT_FWD, NW = NT / 64;
  __shared__ __attribute__((aligned(16))) uint32_t psi_t[1 << TMAX];   // fp16 (re, im), swizzled
  __shared__ int opw2[2][OPW];                          // op records, double buffered (one barrier per op)
  __shared__ int fidx_s[MAXOPS][2];                     // per-op fragment indices (pair ops: two), staged once
  __shared__ uint32_t fo_s[MAXOPS];                     // per-op OFF base of this tile (fo_tab)
  __shared__ __attribute__((aligned(16))) uint4 frag_s[2][256];   // op unitary fragments, double buffered
  __shared__ float red[NW * CMAX];
  __shared__ float2 wv[32][2];
  __shared__ float2 tabA[128];
  __shared__ float2 tabB[128];
  __shared__ float2 outer_s;                            // scale x product of the out-of-tile layer-1 factors

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int s = bid / a.n_tiles, tile_id = bid % a.n_tiles;
  const int k = s / a.spc;
  // in_rep > 1: in_rep consecutive parameter rows (clients) share each input sample - a parameter-shift branch
  // starts from the stored unshifted state of its client's sample (sample s reads input row s_in)
  const int s_in = a.in_rep > 1 ? (s / (a.in_rep * a.spc)) * a.spc + s % a.spc : s;
  const int T = 1 << a.t;
  const size_t N = (size_t)1 << a.n;
  const uint32_t fixed = tile_fixed(a, tile_id);
  const float* prm = a.params + (size_t)k * a.p_stride;
  Stamps st;
  st.init();
  const uint32_t h_q = swz(a, (uint32_t)tid >> 3);        // for quads 4 (tid + NT i)

  // op records and unitary fragments are prefetched one op ahead (their global latency hides behind an op); op 0's
  // are requested before the initial tile, so their latency hides behind the tile load / layer-1 generation
  if (tid < a.nops) {                            // LDS copies: the prefetch below never waits on a global load
    fidx_s[tid][0] = a.fidx[2 * tid];
    fidx_s[tid][1] = a.fidx[2 * tid + 1];
    fo_s[tid] = a.fo_tab[(size_t)tile_id * a.nops + tid];
    QFX_DCHECK(fo_s[tid] == op_fo_global(a.ops + (size_t)tid * OPW, fixed));
  }
  if (tid < OPW && a.nops > 0) opw2[0][tid] = a.ops[tid];
  int nxt = (tid < OPW && a.nops > 1) ? a.ops[OPW + tid] : 0;
  if (a.nops > 0) dma_frags(a, k, a.fidx, lane, wave, frag_s[0]);
  st.mark(PH_PRO);

  // ---------------------------------------------------------------- initial psi tile
  if (a.gen) {
    // Product state of layer 1: wave 0 computes every qubit's 2-vector (lane q) and, by a complex product over
    // the wave, the factor of the qubits outside the tile (their bits are fixed over the tile).  Then the two
    // half-index tables: each entry is a product of <= 7 factors, all read from LDS before the first multiply
    // (one LDS round trip instead of one per factor).
    if (wave == 0) {
      float2 w[2] = {make_float2(1.f, 0.f), make_float2(1.f, 0.f)};
      if (tid < a.n) {
        l1_factor(a.xang[(size_t)s_in * a.x_stride + tid], prm[2 * tid], prm[2 * tid + 1], a.feature, w);
        wv[tid][0] = w[0];
        wv[tid][1] = w[1];
      }
      const bool outq = tid < a.n && !(tid < a.c || (tid >= a.lo && tid < a.hi));
      // value select, not w[bit]: a run-time index put w in scratch (a global round trip per workgroup)
      const float2 w0 = w[0], w1 = w[1];
      float2 f = outq ? (((fixed >> (tid & 31)) & 1) ? w1 : w0) : make_float2(1.f, 0.f);
#pragma unroll
      for (int off = 1; off < 64; off <<= 1) f = cmul(f, make_float2(__shfl_xor(f.x, off, 64), __shfl_xor(f.y, off, 64)));
      if (tid == 0) outer_s = make_float2(a.scale * f.x, a.scale * f.y);
    }
    lds_barrier();
    st.mark(PH_GEN1);
    const int ta = a.t >> 1, tb = a.t - ta;
    constexpr int JMAX = TMAX - (TMAX >> 1);
    const bool lowt = tid < (1 << ta), hight = tid >= 256 && tid < 256 + (1 << tb);
    if (lowt || hight) {                            // [0, 2^ta): low-half products; [256, ..): high half
      const int i = lowt ? tid : tid - 256, j0 = lowt ? 0 : ta, nj = lowt ? ta : tb;
      float2 fac[JMAX];
#pragma unroll
      for (int j = 0; j < JMAX; ++j) {
        const int tj = j0 + j, mb = tj < a.c ? tj : a.lo + tj - a.c;
        fac[j] = wv[j < nj ? mb : 0][(i >> j) & 1];
      }
      float2 v = lowt ? make_float2(1.f, 0.f) : outer_s;
#pragma unroll
      for (int j = 0; j < JMAX; ++j)
        if (j < nj) v = cmul(v, fac[j]);
      if (lowt)
        tabA[i] = v;
      else
        tabB[i] = v;
    }
    lds_barrier();
    st.mark(PH_GEN2);
    const uint32_t am = (1u << ta) - 1u;
    // quad q = tid + NT i holds LDS words 4q .. 4q+3 = amplitudes tau_e = (4q + e) ^ h, h = h(q >> 3);
    // the swizzle only flips bits < 5 and ta >= 4, so the four words share one high-half factor.  Table reads
    // are never predicated (quads past a small tile read quad 0); only the stores are.
    // All quads are computed before the first store: a store to the tile between them kept the compiler from
    // issuing the next quad's table reads early (one LDS round trip per quad).
    constexpr int QI = (1 << TMAX) / (4 * NT);
    uint4 out[QI];
#pragma unroll
    for (int i = 0; i < QI; ++i) {
      const uint32_t q = (uint32_t)(tid + NT * i);
      const uint32_t qq = 4 * q < (uint32_t)T ? q : 0u;
      const uint32_t h = h_q ^ swz(a, (uint32_t)(4 * NT / 32) * i);
      const float2 vb = tabB[((4 * qq) ^ h) >> ta];          // same high half for the whole quad
      uint32_t* ow = (uint32_t*)&out[i];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const float2 v = cmul(tabA[((4 * qq + e) ^ h) & am], vb);
        ow[e] = pack_h2(v.x, v.y);
      }
    }
#pragma unroll
    for (int i = 0; i < QI; ++i) {
      const uint32_t q = (uint32_t)(tid + NT * i);
      if (4 * q < (uint32_t)T) *(uint4*)&psi_t[4 * q] = out[i];
    }
  } else {
    load_tile<NT>(a, a.psi_in + (size_t)s_in * N, psi_t, tid, T, h_q, fixed);
  }

  // ---------------------------------------------------------------- op list
  const int ncol = T >> 4, nblk = ncol >> 4;
  const int nbw = FULL ? (1 << (TMAX - 8)) / NW : (wave < nblk ? (nblk - wave + NW - 1) / NW : 0);   // (uniform)
  st.mark(PH_LOAD);
  op_barrier(wave);   // (waves 0-1 wait for op 0's fragment DMA and record loads; the readout wave's stores never)
  st.mark(PH_BAR);
  for (int o = 0; o < a.nops; ++o) {
    // op o's record and fragments were written during op o - 1; the other buffers were last read at the
    // start of op o - 1, which every wave has finished at this barrier, so op o + 1's go there right away
    if (o > 0) {
      op_barrier(wave);
      st.mark(PH_BAR);
    }
    const int* opw = opw2[o & 1];
    uint4 F[4], FY[4];
    if (fidx_s[o][0] >= 0) frag_regs(frag_s[o & 1], 0, lane, F);
    if (fidx_s[o][1] >= 0) frag_regs(frag_s[o & 1], 1, lane, FY);
    if (o + 1 < a.nops) {
      if (tid < OPW) opw2[(o + 1) & 1][tid] = nxt;
      if (o + 2 < a.nops && tid < OPW) nxt = a.ops[(size_t)(o + 2) * OPW + tid];
      dma_frags(a, k, fidx_s[o + 1], lane, wave, frag_s[(o + 1) & 1]);
    }
    const int code = opw[W_CODE];
#if QFX_CHECKS_ON
    QFX_DCHECK(code == OP_APPLY || code == OP_APPLY2 || code == OP_READOUT);
    if (code != OP_READOUT) {
      QFX_DCHECK(opw[W_NREAL] >= 0 && opw[W_NREAL] <= 4);
      QFX_DCHECK((uint32_t)opw[W_OFF + (lane & 15)] < (uint32_t)T);
      QFX_DCHECK((uint32_t)opw[W_BL + (lane & 31)] < (uint32_t)T);
      QFX_DCHECK((uint32_t)opw[W_BH + (lane & 31)] < (uint32_t)T);
      QFX_DCHECK(fidx_s[o][0] >= 0 && fidx_s[o][0] < 4 * a.n_slots);
      if (code == OP_APPLY2) {
        QFX_DCHECK((uint32_t)opw[W_OFF2 + (lane & 15)] < (uint32_t)T);
        QFX_DCHECK(fidx_s[o][1] >= 0 && fidx_s[o][1] < 4 * a.n_slots && a.t >= 11);
      }
    } else {
      QFX_DCHECK(opw[W_NREAL] >= 1 && opw[W_NREAL] <= a.C);
    }
#endif
    st.mark(PH_SETUP);
    if (code == OP_APPLY) {
      group_apply<NW, false>(psi_t, F, opw, fo_s[o], lane, wave, nbw);
      st.mark(PH_APPLY);
    } else if (code == OP_APPLY2) {
      group_pair_fwd<NW, TMAX>(psi_t, F, FY, opw, fo_s[o], lane, wave, nbw);
      st.mark(PH_APPLY);
    } else if (code == OP_READOUT) {
      const size_t pidx = ((size_t)s * a.n_tiles + tile_id) * a.C;
      readout_op<NCK, NT>(psi_t, a, opw, tid, lane, wave, T, fixed, red, pidx);
      st.mark(PH_OTHER);
    }
    if constexpr (QFX_HEA_STAMPS) ++st.nops;
  }
  lds_barrier();
  if (a.store_psi) store_tile<NT>(a, a.psi_out + (size_t)s * N, psi_t, tid, T, h_q, fixed);
  st.mark(PH_TAIL);
  st.write(a.dbg, bid, NW, wave, lane);
}

// ------------------------------------------------------------------------------------------- adjoint pass
// One workgroup per tile of 2^t <= 2^TB amplitudes holding psi and lambda interleaved (2^(TB+3) bytes of LDS),
// 2^(TB-4) threads: TB = 14 is a 16-wave workgroup on 128 KB (one per CU); TB = 13 an 8-wave workgroup on
// 64 KB, two per CU, so one workgroup's tile load (the HBM latency of a fresh 64 KB tile) overlaps the other's
// group ops and the two workgroups' per-op barriers are independent.  Both have 4 column blocks per wave per
// op.  Gradient ops accumulate their cross-matrix entries into per-op LDS regions.  TB = 14 has room for one
// region per gradient op of the pass, reduced to partial traces once at the end.  TB = 13 alternates two
// regions: at the start of the op after a gradient op, ONE wave reduces that op's region to partial traces and
// zeroes it, while the other waves go on with the op (its region is next used two gradient ops later, after
// at least one more barrier).  Measured: spreading that flush over all waves delays every wave by its LDS
// round trip and was slower (16q adjoint 0.67 -> 0.72 ms).
// 2^(TB - 10) waves give each wave 4 column blocks per op (a 4-wave 2^13 workgroup with 8 blocks per wave halves the
// per-op setup per MFMA but halves the waves per SIMD: measured 18% slower, round 4).
template <int NCK, int TB, bool FULL>
__device__ __forceinline__ void adj_pass(const PassArgs& a, int bid) {
  constexpr int NT = 1 << (TB - 4), NW = NT / 64;
  static_assert(NW % 2 == 0 && (1 << (TB - 8)) % NW == 0, "column blocks per wave must be whole, block pairs aligned");
  // (psi, lambda) pairs (fp16 re, im), swizzled; 16-byte aligned for the b64 / b128 accesses
  __shared__ __attribute__((aligned(16))) uint32_t tile[2 << TB];
  __shared__ int opw2[2][OPW];                          // op records, double buffered (one barrier per op)
  __shared__ int fidx_s[MAXOPS][2];                     // per-op fragment indices (pair ops: two), staged once
  __shared__ uint32_t fo_s[MAXOPS];                     // per-op OFF base of this tile (fo_tab)
  __shared__ __attribute__((aligned(16))) uint4 frag_s[2][256];   // op unitary fragments, double buffered
  // the 80 cross-matrix entries a partial trace can use (b = a, and b = a ^ e_j) x (re, im), 2^-32 fixed point
  // One region per gradient record of the pass, reduced by all waves after the op loop - up to NREG (2^13 tiles: 9,
  // which still fits two workgroups per CU).  A pass with more records cycles through a ring of 4 regions instead,
  // one wave flushing a region at the start of the op after its use (an op uses at most two, so consecutive ops never
  // share one) - that flush put the flushing wave on every barrier's critical path (stall table, round 5).
  constexpr int NREG = TB < 14 ? 9 : MAXGRAD;
  const bool ring = TB < 14 && a.n_regions > NREG;   // (2^14 tiles: MAXGRAD regions, never a ring)
  __shared__ unsigned long long red64[NREG * RSTR];
  __shared__ int gmeta_s[NREG][2];                      // (slab index, nreal) of the region's gradient op
  __shared__ float rsc[CMAX + 2];

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int s = bid / a.n_tiles, tile_id = bid % a.n_tiles;
  const int k = s / a.spc;
  const int T = 1 << a.t;
  const size_t N = (size_t)1 << a.n;
  const uint32_t fixed = tile_fixed(a, tile_id);
  Stamps st;
  st.init();
  const uint32_t h_q = swz(a, (uint32_t)tid >> 3);        // for quads 4 (tid + NT i)
  long long* slab = a.gslab + ((size_t)s * a.slab_tiles + tile_id) * a.n_gradops * 32;
  QFX_DCHECK(tile_id < a.slab_tiles);

  // op 0's record and fragments are requested before the tile load (their latency hides behind it)
  if (tid < a.nops) {
    fidx_s[tid][0] = a.fidx[2 * tid];
    fidx_s[tid][1] = a.fidx[2 * tid + 1];
    fo_s[tid] = a.fo_tab[(size_t)tile_id * a.nops + tid];
    QFX_DCHECK(fo_s[tid] == op_fo_global(a.ops + (size_t)tid * OPW, fixed));
  }
  if (tid < OPW && a.nops > 0) opw2[0][tid] = a.ops[tid];
  int nxt = (tid < OPW && a.nops > 1) ? a.ops[OPW + tid] : 0;
  if (a.nops > 0) dma_frags(a, k, a.fidx, lane, wave, frag_s[0]);
  // Fused readout (the last wave): its lanes load the sample's readout partials, label, loss weight and readout
  // parameters BEFORE the tile load is issued, so their latency overlaps the tile's; lane 0 sums the partials in tile
  // order after the load (the readout kernel's order and arithmetic, qfx_readout.h).
  const bool ro_wave = a.ro_fuse && wave == NW - 1;
  const int ro_np = a.ro_fuse ? a.ro_tps * a.C : 0;   // partials per sample (<= 64: host-checked)
  float ro_v = 0.f, ro_ab = 0.f, ro_ws = 0.f;
  int ro_yy = 0;
  if (ro_wave) {
    if (lane < ro_np) ro_v = a.part[(size_t)s * ro_np + lane];
    if (lane < 2 * a.C) ro_ab = a.params[(size_t)k * a.p_stride + a.n_theta + lane];
    if (lane == 0) {
      ro_ws = a.ro_wts[s];
      ro_yy = (int)a.ro_y[s];
    }
  }
  st.mark(PH_PRO);
  load_tile_il<NT, TB>(a, a.psi_in + (size_t)s * N, a.load_lam ? a.lam_in + (size_t)s * N : nullptr, tile, tid, T, h_q,
                       fixed);

  if (a.ro_fuse ? tid == NT - 64 : tid == 0) {
    float wv[CMAX];
    if (a.ro_fuse) {
      // lane 0 of the last wave: partials and parameters gathered from its wave's lanes (one load round trip); every
      // per-class array is indexed by unrolled constants (a run-time class index would put them in scratch)
      float z[qfx_ro::RO_CMAX], ra[2 * qfx_ro::RO_CMAX], dl[qfx_ro::RO_CMAX], lterm, hit;
#pragma unroll
      for (int c = 0; c < qfx_ro::RO_CMAX; ++c) z[c] = 0.f;
      for (int u = 0; u < a.ro_tps; ++u) {
#pragma unroll
        for (int c = 0; c < qfx_ro::RO_CMAX; ++c)
          if (c < a.C) z[c] += __int_as_float(__builtin_amdgcn_readlane(__float_as_int(ro_v), u * a.C + c));
      }
#pragma unroll
      for (int c = 0; c < 2 * qfx_ro::RO_CMAX; ++c)
        ra[c] = c < 2 * a.C ? __int_as_float(__builtin_amdgcn_readlane(__float_as_int(ro_ab), c)) : 0.f;
      float rb[qfx_ro::RO_CMAX];
#pragma unroll
      for (int c = 0; c < qfx_ro::RO_CMAX; ++c) rb[c] = c < a.C ? __int_as_float(__builtin_amdgcn_readlane(
                                                                 __float_as_int(ro_ab), a.C + c)) : 0.f;
      qfx_ro::ce_sample(z, ra, rb, a.C, ro_yy, ro_ws, dl, lterm, hit);
      const bool out = tile_id == 0;
      float* rec = a.ro_rec + (size_t)s * (2 * a.C + 2);
#pragma unroll
      for (int c = 0; c < CMAX; ++c) {
        if (c >= a.C) break;
        wv[c] = dl[c] * ra[c];
        if (out) {
          a.ro_expz[(size_t)s * a.C + c] = z[c];
          a.ro_w[(size_t)s * a.C + c] = wv[c];
          rec[c] = dl[c] * z[c];
          rec[a.C + c] = dl[c];
        }
      }
      if (out) {
        rec[2 * a.C] = lterm;
        rec[2 * a.C + 1] = hit;
      }
    } else {
#pragma unroll
      for (int c = 0; c < CMAX; ++c) {
        if (c >= a.C) break;
        wv[c] = a.wread[(size_t)s * a.C + c];
      }
    }
    float rho = 0.f;
#pragma unroll
    for (int c = 0; c < CMAX; ++c) {
      if (c >= a.C) break;
      rho = fmaxf(rho, fabsf(wv[c]));
    }
    if (rho == 0.f) rho = 1.f;
#pragma unroll
    for (int c = 0; c < NCK; ++c) rsc[c] = c < a.C ? wv[c] / rho : 0.f;
    rsc[CMAX] = rho;
    rsc[CMAX + 1] = PK_SCALE / (a.scale * a.scale);
  }
  for (int e = tid; e < (ring ? 4 : min(a.n_regions, NREG)) * RSTR; e += NT) red64[e] = 0ull;

  // Partial traces of a finished gradient op's region (read after a barrier): output r = (j, y, x, comp) sums the
  // 8 entries with b_j = y, a_j = x (the whole workgroup at the end of the pass, or lanes 0..31 of the flushing
  // wave).
  auto reduce_region = [&](int reg, int r) {
    const int j = r >> 3, y = (r >> 2) & 1, x = (r >> 1) & 1, comp = r & 1;
    const unsigned long long* rg = red64 + reg * RSTR;
    long long v = 0;
    if (j < gmeta_s[reg][1]) {
      const int lowm = (1 << j) - 1;
      for (int o8 = 0; o8 < 8; ++o8) {    // the other three bits of b
        const int bb = ((o8 & ~lowm) << 1) | (o8 & lowm) | (y << j);
        const unsigned long long u = rg[red_slot(x == y ? bb : 16 + 16 * j + bb)];
        v += (long long)(uint32_t)(comp ? (u >> 32) : u) - (long long)NW * PK_BIAS;
      }
    }
    // 2^-22 units of N / rho -> the slab's 2^-32 units of N (one exact integer sum per tile: deterministic)
    slab[(size_t)gmeta_s[reg][0] * 32 + r] = __double2ll_rn((double)v * (double)rsc[CMAX] * (FIX / (double)PK_SCALE));
  };
  auto flush = [&](int reg) {                           // one wave: reduce, then zero the region
    if (lane < 32) reduce_region(reg, lane);
    lds_barrier_wave();
    for (int e = lane; e < RSTR; e += 64) red64[reg * RSTR + e] = 0ull;
  };

  // ---------------------------------------------------------------- op list
  const int ncol = T >> 4, nblk = ncol >> 4;
  // FULL (t == TB): every wave owns exactly (2^(TB - 8)) / NW column blocks - a compile-time count, so the block
  // loops of the group ops carry no bounds checks or branches
  const int nbw = FULL ? (1 << (TB - 8)) / NW : (wave < nblk ? (nblk - wave + NW - 1) / NW : 0);
  st.mark(PH_LOAD);
  op_barrier(wave);   // (waves 0-1 wait for op 0's fragment DMA and record loads; the readout wave's stores never)
  st.mark(PH_BAR);
  int ngrad = 0;
  int pending = -1, npend = 0;                         // ring: first region / count of the previous op's regions
  // Partial-trace entries this lane adds per gradient op: lane (g4, cl) holds N[4 g4 + i][cl]; byte i of epi is the
  // entry's region slot (b == a -> b, b ^ a == e_j -> 16 + 16 j + b, skewed by red_slot) or 0xFF if no partial
  // trace uses it.  One VGPR for the whole op loop (the per-op predicates had been SGPR pairs spilled to VGPR lanes,
  // and the four slot addresses four more VGPRs).
  uint32_t epi = 0;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const uint32_t bb = 4u * (lane >> 4) + i, aa = lane & 15, d = bb ^ aa;
    const uint32_t sl = __builtin_popcount(d) <= 1 ? (uint32_t)red_slot(d == 0 ? (int)bb : 16 + 16 * __builtin_ctz(d) + (int)bb)
                                                    : 0xFFu;
    epi |= sl << (8 * i);
  }
  for (int o = 0; o < a.nops; ++o) {
    // op o's record and fragments were written during op o - 1; the other buffers were last read at the
    // start of op o - 1, which every wave has finished at this barrier, so op o + 1's go there right away
    if (o > 0) {
      op_barrier(wave);
      st.mark(PH_BAR);
    }
    if (ring && npend > 0) {                           // one wave per region, the last waves
      for (int q = 0; q < npend; ++q)
        if (wave == NW - 1 - q) flush((pending + q) & 3);
      npend = 0;
    }
    const int* opw = opw2[o & 1];
    uint4 F[4], FY[4];
    if (fidx_s[o][0] >= 0) frag_regs(frag_s[o & 1], 0, lane, F);
    if (fidx_s[o][1] >= 0) frag_regs(frag_s[o & 1], 1, lane, FY);
    if (o + 1 < a.nops) {
      if (tid < OPW) opw2[(o + 1) & 1][tid] = nxt;
      if (o + 2 < a.nops && tid < OPW) nxt = a.ops[(size_t)(o + 2) * OPW + tid];
      dma_frags(a, k, fidx_s[o + 1], lane, wave, frag_s[(o + 1) & 1]);
    }
    const int code = opw[W_CODE];
#if QFX_CHECKS_ON
    QFX_DCHECK(code == OP_BACK || code == OP_GRAD_L1 || code == OP_OBS || code == OP_BACK2 || code == OP_GRAD2);
    if (code != OP_OBS) {
      const bool pr2 = code == OP_BACK2 || code == OP_GRAD2;
      QFX_DCHECK(opw[W_NREAL] >= 0 && opw[W_NREAL] <= 4);
      QFX_DCHECK((uint32_t)opw[W_OFF + (lane & 15)] < (uint32_t)T);
      QFX_DCHECK((uint32_t)opw[W_BL + (lane & 31)] < (uint32_t)T);
      QFX_DCHECK((uint32_t)opw[W_BH + (lane & 31)] < (uint32_t)T);
      // -1 = no unitary (cross-matrix-only gradient ops); every op that applies one names a fragment
      QFX_DCHECK(fidx_s[o][0] >= -1 && fidx_s[o][0] < 4 * a.n_slots);
      QFX_DCHECK(fidx_s[o][0] >= 0 || code == OP_GRAD_L1 || code == OP_GRAD2);
      QFX_DCHECK(opw[W_GIDX] >= 0 && opw[W_GIDX] < a.n_gradops);
      if (pr2) {
        QFX_DCHECK((uint32_t)opw[W_OFF2 + (lane & 15)] < (uint32_t)T && a.t >= 11);
        QFX_DCHECK(opw[W_GIDX2] >= 0 && opw[W_GIDX2] < a.n_gradops);
        QFX_DCHECK(code == OP_GRAD2 || (fidx_s[o][1] >= 0 && fidx_s[o][1] < 4 * a.n_slots));
      }
    } else {
      QFX_DCHECK(opw[W_NREAL] >= 1 && opw[W_NREAL] <= a.C);
    }
#endif
    st.mark(PH_SETUP);
    if (code == OP_OBS) {
      obs_op<NCK, NT, TB>(tile, opw, tid, T, fixed, rsc);
      st.mark(PH_OTHER);
    } else {   // OP_BACK / OP_GRAD_L1 / OP_BACK2 / OP_GRAD2
      const uint32_t fo = fo_s[o];
      f4 acc[4] = {{0.f, 0.f, 0.f, 0.f}, {0.f, 0.f, 0.f, 0.f}, {0.f, 0.f, 0.f, 0.f}, {0.f, 0.f, 0.f, 0.f}};
      int ng = 1;
      if (code == OP_BACK && (opw[W_FLAGS] & F_BACK_PSI)) {
        // U^H on psi and lambda, cross matrix at the op input from the results (hea_grad_reduce: input side)
        group_back_t<NW, TB>(tile, F, opw, fo, lane, wave, nbw, acc);
        st.mark(PH_BACK);
      } else if (code == OP_BACK) {
        // U^H on lambda only, cross matrix from the apply's own registers (one pass over the blocks)
        group_apply<NW, true, TB>(tile, F, opw, fo, lane, wave, nbw, acc);
        st.mark(PH_BACK);
      } else if (code == OP_BACK2) {
        group_pair_back<NW, TB>(tile, F, FY, opw, fo, lane, wave, nbw, acc);
        ng = 2;
        st.mark(PH_BACK);
      } else if (code == OP_GRAD2) {
        group_pair_cross<NW, TB>(tile, opw, fo, lane, wave, nbw, acc);
        ng = 2;
        st.mark(PH_GRADL1);
      } else {
        group_cross<NW, TB>(tile, opw, fo, lane, wave, nbw, acc[0], acc[1]);
        st.mark(PH_GRADL1);
      }
      // Cross-wave sum of the partial-trace entries of N / rho into the op's region(s): packed biased fixed point
      // (PK_*), one u64 LDS atomic per entry.  Integer addition is associative, so the sums are bitwise
      // independent of the order the waves (and, in hea_grad_reduce, samples and tiles) arrive.
      // Lane (g4, cl) holds N[4 g4 + i][cl]; entry slot: b == a -> b, b ^ a == e_j -> 16 + 16 j + b.
      const float sc = rsc[CMAX + 1];
      // opaque to the optimiser: kept packed in one VGPR (hoisted out of the op loop, the per-entry predicates and
      // slot addresses had taken eight SGPRs - spilled to VGPR lanes - and four VGPRs)
      uint32_t ep = epi;
      __asm__ volatile("" : "+v"(ep));
      if (ring) pending = ngrad & 3;
#pragma unroll
      for (int g = 0; g < 2; ++g) {
        if (g >= ng) break;
        const int reg = ring ? ngrad & 3 : ngrad;
        unsigned long long* rg = red64 + reg * RSTR;
        const f4 accR = acc[2 * g], accI = acc[2 * g + 1];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const uint32_t sl = (ep >> (8 * i)) & 0xFFu;
          if (sl != 0xFFu) {
            // round half up (floor(x + 0.5), one instruction): unbiased for these continuous values - truncation
            // biased every add toward zero, and a tile's sum has thousands
            const uint32_t lo = (uint32_t)cvt_rpi(accR[i] * sc) + PK_BIAS, hi = (uint32_t)cvt_rpi(accI[i] * sc) + PK_BIAS;
            atomicAdd(&rg[sl], ((unsigned long long)hi << 32) | lo);
          }
        }
        if (tid == 0) {
          gmeta_s[reg][0] = opw[g ? W_GIDX2 : W_GIDX];
          gmeta_s[reg][1] = opw[g ? W_NREAL2 : W_NREAL];   // (a layer-1 pair's groups may be short)
        }
        ++ngrad;
      }
      npend = ng;
      st.mark(PH_EPI);
    }
    if constexpr (QFX_HEA_STAMPS) ++st.nops;
  }
  lds_barrier();
  if (ring) {
    for (int q = 0; q < npend; ++q)
      if (wave == NW - 1 - q && lane < 32) reduce_region((pending + q) & 3, lane);
  } else {
    for (int e = tid; e < ngrad * 32; e += NT) reduce_region(e >> 5, e & 31);
  }
  if (a.store_lam) store_lam_il<NT, TB>(a, a.lam_out + (size_t)s * N, tile, tid, T, h_q, fixed);
  st.mark(PH_TAIL);
  st.write(a.dbg, bid, NW, wave, lane);
}

// ------------------------------------------------------------------------------------------- launches
template <int NCK, bool FULL>
__global__ void __launch_bounds__(NT_FWD, 4) hea_fwd_kernel(PassArgs a) { fwd_pass<NCK, FULL>(a, blockIdx.x); }

template <int NCK, int TB, bool FULL>
__global__ void __launch_bounds__(1 << (TB - 4), (1 << (TB - 4)) * 2 / 256) hea_adj_kernel(PassArgs a) {
  adj_pass<NCK, TB, FULL>(a, blockIdx.x);
}

}  // namespace HEA_NS

// adjoint: 2^13 tiles (8 waves, two workgroups per CU) up to t = 13, else one 16-wave 2^14 workgroup per CU
#define HEA_LAUNCH(NCK, KF, KA, ARG)                                                                         \
  do {                                                                                                      \
    if (!adjoint && t == HEA_NS::TMAX)                                                                       \
      hipLaunchKernelGGL((HEA_NS::KF<NCK, true>), dim3(grid), dim3(HEA_NS::NT_FWD), 0, st, ARG);             \
    else if (!adjoint)                                                                                      \
      hipLaunchKernelGGL((HEA_NS::KF<NCK, false>), dim3(grid), dim3(HEA_NS::NT_FWD), 0, st, ARG);            \
    else if (t <= 13)                                                                                       \
      hipLaunchKernelGGL((HEA_NS::KA<NCK, 13, false>), dim3(grid), dim3(512), 0, st, ARG);                   \
    else                                                                                                    \
      hipLaunchKernelGGL((HEA_NS::KA<NCK, 14, true>), dim3(grid), dim3(1024), 0, st, ARG);                   \
  } while (0)
#define HEA_SWITCH(KF, KA, ARG)                 \
  switch (HEA_NS::class_kernel(C)) {            \
    case 1: HEA_LAUNCH(1, KF, KA, ARG); break;  \
    case 2: HEA_LAUNCH(2, KF, KA, ARG); break;  \
    case 3: HEA_LAUNCH(3, KF, KA, ARG); break;  \
    case 4: HEA_LAUNCH(4, KF, KA, ARG); break;  \
    default: HEA_LAUNCH(8, KF, KA, ARG); break; \
  }

static bool hea_args_ok(const HEA_NS::PassArgs& a) {
  return !(a.t > HEA_NS::TMAX || a.t < 8 || a.C > HEA_NS::CMAX || a.n > 30 || a.c < 2);
}

extern "C" int HEA_EXT(qfx_hea_pass)(int adjoint, const HEA_NS::PassArgs* args, int n_samples, hipStream_t st) {
  const HEA_NS::PassArgs& a = *args;
  if (!hea_args_ok(a)) return -2;
  const unsigned grid = (unsigned)(n_samples * a.n_tiles);
  if (grid == 0) return 0;
  const int t = a.t, C = a.C;
  HEA_SWITCH(hea_fwd_kernel, hea_adj_kernel, a);
  return (int)hipGetLastError();
}

#undef HEA_SWITCH
#undef HEA_LAUNCH


// Debug build: synchronise the stream and return (and clear) the first failed device-check line, 0 if none;
// -1 in the release build (no checks compiled).  A launch recorded into a graph under capture is not checked here
// (a synchronise would invalidate the capture): its checks fire when the graph replays and are read at the next
// eager launch's check.
extern "C" int HEA_EXT(qfx_hea_check_status)(hipStream_t st) {
#if QFX_CHECKS_ON
  hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
  if (hipStreamIsCapturing(st, &cs) != hipSuccess) return -2;
  if (cs != hipStreamCaptureStatusNone) return 0;
  if (hipStreamSynchronize(st) != hipSuccess) return -2;
  unsigned int v = 0, z = 0;
  if (hipMemcpyFromSymbol(&v, HIP_SYMBOL(qfx_check_word), sizeof(v)) != hipSuccess) return -2;
  if (v && hipMemcpyToSymbol(HIP_SYMBOL(qfx_check_word), &z, sizeof(z)) != hipSuccess) return -2;
  return (int)v;
#else
  (void)st;
  return -1;
#endif
}
