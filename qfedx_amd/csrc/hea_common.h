// Definitions shared by the MFMA statevector engine's translation units: hea_mfma.hip (pass kernels) and
// hea_step.hip (per-step fragment build and gradient reduction), each also built for bf16 storage via
// hea_mfma_bf16.hip.  Storage-type primitives, op / record enums, fixed-point constants, stall-attribution stamps.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdlib>
#include <cstring>

// Storage type of the states and unitary fragments: fp16 (this translation unit) or bf16 (hea_mfma_bf16.hip includes
// this file with QFX_HEA_BF16=1: the same kernels in namespace hea_bf16, entry points suffixed _bf16).  Only the
// pack / unpack / MFMA / i-multiply primitives and the fragment split below depend on it.
#ifndef QFX_HEA_BF16
#define QFX_HEA_BF16 0
#endif
#if QFX_HEA_BF16
#define HEA_NS hea_bf16
#define HEA_EXT(name) name##_bf16
#define qfx_check_word qfx_check_word_bf16
#else
#define HEA_NS hea
#define HEA_EXT(name) name
#endif

#include "hea_args.h"
#include "qfx_readout.h"
#include "qfx_adam.h"
#include "qfx_check.h"


// Gate precision: 1 (default) applies every unitary as its fp16 hi + lo halves (exact to ~2^-22), 0 as the hi half
// only (fp16-rounded gate: half the apply MFMAs).
#ifndef QFX_HEA_GATE_LO
#define QFX_HEA_GATE_LO 1
#endif
// Stall attribution (diagnostic build only: python -m qfedx_amd._build --stamps -> _qfedx_C_stamps, -DQFX_HEA_STAMPS=1).
// Every wave of the first STAMP_WG workgroups of a pass adds the s_memtime cycles of each phase (enum Ph) into its own
// row of a.dbg; scripts/hea_stamps.py turns the rows into the per-op-phase table.  In the release build no stamp
// executes and the bookkeeping folds away.
#ifndef QFX_HEA_STAMPS
#define QFX_HEA_STAMPS 0
#endif


namespace HEA_NS {

constexpr int OPW = 128;
// APPLY2 / BACK2 / GRAD2: chained pairs of two commuting 4-qubit groups X, Y of one layer (group_pair_*)
enum { OP_APPLY = 1, OP_APPLY2 = 2, OP_BACK2 = 3, OP_GRAD2 = 4, OP_GRAD_L1 = 5, OP_OBS = 6, OP_READOUT = 7, OP_BACK = 8 };
enum { W_CODE = 0, W_SLOT = 1, W_NREAL = 2, W_FLAGS = 3, W_RFULL = 4, W_RT = 8, W_TH = 12, W_PH = 16, W_OFF = 20,
       W_BL = 36, W_BH = 68, W_GIDX = 100,
       // pair records (hea_plan.pair_table): group Y's row masks in the W_RT words, its records / OFF table here
       W_RFULL2 = 8, W_GIDX2 = 101, W_SLOT2 = 102, W_NREAL2 = 103, W_OFF2 = 104 };
constexpr double FIX = 4294967296.0;   // 2^32: fixed point of the scaled gradient partial traces
constexpr int F_BACK_PSI = 1;
constexpr int F_BACK_TRANS = 2;   // OP_BACK (with F_BACK_PSI) in the transposed form: cross matrix at the op input
constexpr int TMAX = 14;
constexpr int NT_FWD = 512;    // forward: 8 waves, 64 KB LDS -> 2 workgroups per CU
constexpr int NT_ADJ = 1024;   // adjoint: 16 waves, 128 KB LDS (psi + lambda) -> 1 workgroup per CU
constexpr int CMAX = 8;
constexpr int MAXOPS = 32;     // ops per pass program (host-checked)
constexpr int MAXGRAD = 12;    // gradient ops per pass program (host-checked)
// Per gradient op, 80 cross-matrix entries e = 16 k + b (k = 0: b == a, k = 1 + j: b ^ a = e_j), each one u64
// LDS atomic holding (re, im) as two biased 32-bit fixed-point halves (PK_*).  A half-wave's active lanes add
// entries {b + 16 k} with b in {i, i + 4}: unskewed they all sit on one bank pair (5-way conflicts);
// slot(e) = e + s(k), s = 0, 1, 2, 3, 8, spreads them over distinct 8-byte bank pairs (b + s(k) distinct mod 16).
constexpr int RIM = 88, RSTR = RIM;
// Packed entry halves: N / rho in 2^-22 units plus a bias of 2^26 per add.  |N / rho| <= C <= 8 (Cauchy-Schwarz
// on the tile's psi and lambda / rho, rho = max |w_c|), so each add lies in [2^25, 2^27) and the sum of <= 16
// waves' adds stays below 2^31: no carry ever crosses into the other half, and integer addition keeps the
// cross-wave sums independent of arrival order.  One atomic and ~4 VALU per entry and component instead of
// two int64 atomics with a 7-op fp32 -> int64 split each.
constexpr float PK_SCALE = 0x1p22f;
constexpr uint32_t PK_BIAS = 1u << 26;
__device__ __forceinline__ int red_slot(int e) {
  const int k = e >> 4;
  return e + (k < 4 ? k : 8);
}

#if QFX_HEA_BF16
typedef __bf16 st_t;
#else
typedef _Float16 st_t;
#endif
typedef st_t half8 __attribute__((ext_vector_type(8)));
typedef st_t half2v __attribute__((ext_vector_type(2)));
// 1.0 in the storage type, in the low / high half of a packed (re, im) word
constexpr uint32_t ONE_LO = QFX_HEA_BF16 ? 0x00003F80u : 0x00003C00u;
constexpr uint32_t ONE_HI = ONE_LO << 16;
typedef float f4 __attribute__((ext_vector_type(4)));
typedef uint32_t u4v __attribute__((ext_vector_type(4)));

using PassArgs = HeaPassArgs;

__device__ __forceinline__ uint32_t pack_h2(float re, float im) {
  half2v h = {(st_t)re, (st_t)im};
  return __builtin_bit_cast(uint32_t, h);
}

// |amplitude|^2 of one packed word: one v_dot2_f32_f16 for fp16 (the fp16 products are exact in fp32) instead of two
// converts, a multiply and an fma
__device__ __forceinline__ float norm2_h2(uint32_t u);

__device__ __forceinline__ float2 unpack_h2(uint32_t u) {
#if QFX_HEA_BF16
  return make_float2(__uint_as_float(u << 16), __uint_as_float(u & 0xFFFF0000u));   // bf16 -> fp32 is a shift
#else
  half2v h = __builtin_bit_cast(half2v, u);
  return make_float2((float)h.x, (float)h.y);
#endif
}

__device__ __forceinline__ float norm2_h2(uint32_t u) {
#if QFX_HEA_BF16
  const float2 f = unpack_h2(u);
  return f.x * f.x + f.y * f.y;
#else
  const half2v h = __builtin_bit_cast(half2v, u);
  return __builtin_amdgcn_fdot2(h, h, 0.f, false);
#endif
}

__device__ __forceinline__ int par(uint32_t x) { return __builtin_popcount(x) & 1; }

// Workgroup barrier for LDS hand-offs only.  __syncthreads() is a workgroup fence and so also drains every
// outstanding GLOBAL load (vmcnt(0)) - including the next op's prefetched record and unitary fragments.
// Cross-wave data here only moves through LDS, so completing this wave's LDS (and scalar) operations before
// the s_barrier is sufficient; global results (gslab, stored tiles) are never read back inside the kernel.
__device__ __forceinline__ void lds_barrier() { __asm__ volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

// Stall-attribution phases: per wave, the cycles between consecutive marks go to the phase named by the LATER mark.
//   PRO     kernel start -> tile-load issue (record / fragment staging, readout inputs)
//   LOAD    tile load or product-state generation, up to the first op barrier's arrival
//   BAR     op barriers: arrival -> release (waiting for the slowest wave of the workgroup)
//   SETUP   after release: fragment registers, next op's record / fragment DMA, gradient-region flush
//   BACK    adjoint BACK op bodies (LDS reads, MFMAs, writes)      GRADL1  cross-matrix-only (layer-1) op bodies
//   APPLY   forward group-op bodies                                OTHER   OBS / READOUT op bodies
//   EPI     gradient epilogue (fixed-point packing, u64 LDS atomics)
//   TAIL    after the op loop: last barrier, region reduction, tile store
// Slots NPH - 2 / NPH - 1 hold the op count and the wave's total cycles.
//   GEN1 / GEN2  the first forward pass's layer-1 generation: factors + outer product (wave 0) and its barrier / the
//           half-index tables and their barrier (LOAD then covers the quads)
enum { PH_PRO = 0, PH_LOAD, PH_BAR, PH_SETUP, PH_BACK, PH_GRADL1, PH_APPLY, PH_OTHER, PH_EPI, PH_TAIL, PH_GEN1, PH_GEN2,
       PH_COUNT, NPH = 16 };
static_assert(PH_COUNT <= NPH - 2, "stamp row: phases + op count + total");
constexpr int STAMP_WG = HEA_STAMP_ROWS / 16;   // workgroups stamped per pass (a.dbg: STAMP_WG x waves x NPH u64)
struct Stamps {
  unsigned long long acc[PH_COUNT];
  unsigned long long t0, last;
  int nops;
  __device__ __forceinline__ static unsigned long long now() {
    unsigned long long t;
    __builtin_amdgcn_sched_barrier(0);
    __asm__ volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
    __builtin_amdgcn_sched_barrier(0);
    return t;
  }
  __device__ __forceinline__ void init() {
    if constexpr (QFX_HEA_STAMPS) {
#pragma unroll
      for (int i = 0; i < PH_COUNT; ++i) acc[i] = 0;
      nops = 0;
      t0 = last = now();
    }
  }
  __device__ __forceinline__ void mark(int ph) {
    if constexpr (QFX_HEA_STAMPS) {
      const unsigned long long t = now();
      acc[ph] += t - last;
      last = t;
    }
  }
  // lane 0 of every wave of the first STAMP_WG workgroups writes its row
  __device__ __forceinline__ void write(long long* dbg, int bid, int nw, int wave, int lane) {
    if constexpr (QFX_HEA_STAMPS) {
      if (!dbg || bid >= STAMP_WG || lane != 0) return;
      long long* row = dbg + ((size_t)bid * nw + wave) * NPH;
#pragma unroll
      for (int i = 0; i < PH_COUNT; ++i) row[i] = (long long)acc[i];
      row[NPH - 2] = nops;
      row[NPH - 1] = (long long)(last - t0);
    }
  }
};

__device__ __forceinline__ float2 cmul(float2 a, float2 b) {
  return make_float2(a.x * b.x - a.y * b.y, a.x * b.y + a.y * b.x);
}

__device__ __forceinline__ f4 mfma(uint4 a, uint4 b, f4 c) {
#if QFX_HEA_BF16
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(half8, a), __builtin_bit_cast(half8, b), c, 0,
                                                  0, 0);
#else
  return __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(half8, a), __builtin_bit_cast(half8, b), c, 0,
                                                 0, 0);
#endif
}

}  // namespace HEA_NS
