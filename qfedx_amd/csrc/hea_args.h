// Launch arguments of the MFMA statevector pass kernel (csrc/hea_mfma.hip); shared by the host
// bindings (csrc/hea_bindings.cpp) so both sides agree on the layout.
#pragma once
#include <cstdint>

// Rows of the stall-attribution buffer (stamps build): STAMP_WG = 2048 workgroups x up to 16 waves.
constexpr int HEA_STAMP_ROWS = 2048 * 16;

struct HeaPassArgs {
  const int* ops;            // [nops][128] op records (hea_plan.py)
  const int* fidx;           // [nops][2] unitary fragment indices (slot * 4 + 0 | 2) or -1
  const uint32_t* fo_tab;    // [n_tiles][nops] per-op OFF base of each tile (hea_plan.fo_table)
  int nops;
  int n, t, c, lo, hi, n_tiles;   // tile = memory bits [0, c) u [lo, hi), 2^(n - t) tiles per sample
  int gen, load_lam, store_psi, store_lam;
  int spc, C, n_theta, p_stride, feature;
  float scale;               // stored amplitudes = scale * true amplitudes (fp16 range)
  const uint32_t* psi_in;    // fp16 (re, im) states [S][2^n]
  uint32_t* psi_out;
  const uint32_t* lam_in;
  uint32_t* lam_out;
  const float* xang;         // [S][x_stride] feature angles
  int x_stride;
  const float* params;       // [K][p_stride]
  const void* frags;         // uint4 unitary fragments (hea_frag.h)
  int n_slots;
  int frag_shared;           // 1: one fragment set for every client (a round's first step, built by the prologue)
  const float* wread;        // [S][C] dL/d<Z_c>
  float* part;               // [S][n_tiles][C] readout partials
  long long* gslab;          // [S][slab_tiles][n_gradops][32] 2^-32 fixed-point partial traces
  int slab_tiles;
  int n_gradops;
  int n_regions;             // adjoint: gradient records of this pass program (LDS partial-trace regions it fills)
  int hrow[5];               // LDS swizzle: dword(tau) = tau ^ h(tau >> 5), h bit b = parity(hrow[b] & x)
  long long* dbg;            // stamps build only (QFX_HEA_STAMPS): per-wave phase cycles, [HEA_STAMP_ROWS][16]
  int in_rep;                // forward: shifted parameter rows per stored input sample (param-shift prefix reuse)
  int nt_store;              // 1: pass-output tiles stored with the non-temporal hint (a pass's states exceed the MALL)
  // Fused readout (first adjoint pass, noiseless): every workgroup computes its sample's <Z>, cross entropy and
  // dL/d<Z> from the readout partials (part, ro_tps tiles) instead of reading wread; the tile-0 workgroup writes
  // ro_expz / ro_w [S][C] (the later passes' wread) and the per-sample reduction record ro_rec [S][2C + 2]
  // (dl_c z_c, dl_c, loss term, hit) that hea_grad_reduce sums per client.
  int ro_fuse, ro_tps;
  const long long* ro_y;
  const float* ro_wts;
  float* ro_expz;
  float* ro_w;
  float* ro_rec;
};

// Launch arguments of a fused Adam epilogue (m == nullptr: none); each gradient block steps the parameters it owns.
// cnt: per-client counters of the earlier last-block epilogue, unused since round 6 (kept zero).
struct QfxAdamArgs {
  float* m;
  float* v;
  const float* t_in;
  float* t_out;
  const float* active;
  unsigned* cnt;
  float lr, b1, b2, eps;
};

// The round's FedAvg folded into hea_grad_reduce's Adam epilogue (a round's last local step, plain FedAvg: no DP, no
// SecAgg; buf == nullptr: none).  Each block, right after the Adam step of the parameters it owns, adds client k's
// exact fixed-point terms round(2^32 w_k wrap(theta_k - theta_g)) of them (block (k, 0) also the weight
// round(2^32 w_k)) into the all-reduce buffer head with int64 atomics (integer sums: any arrival order gives the same
// bits, as the FedAvg reduce's own sums), which the round prologue zeroed; the last block of the launch packs the
// round metrics and, on a single rank, applies the round to theta_g (the FedAvg launch's FusedApply).
struct QfxFedTail {
  long long* buf;            // [P + 6 + n_norms] all-reduce buffer
  const float* theta_g;      // [P]
  const unsigned char* mask; // [P] angle mask (wrapped entries)
  const double* weights;     // [K] FedAvg weights
  int wrap;
  const float *loss, *correct, *nvalid, *act;   // round metric tables (n_metrics entries each)
  int n_metrics;
  unsigned* cnt;             // zero-initialised arrival counter of the launch's blocks (the last one resets it)
  float* apply_theta;        // single rank: theta_g updated in place (nullptr: the all-reduce + apply follow)
  double* apply_out;         // [6 + n_norms] metrics / saturation / weight sum read back by the host
  int n_norms;
};

// Per-client readout reduction in hea_grad_reduce (fused readout): one more block per client sums its samples' ro_rec
// records in sample order into the loss / hit outputs and the readout-parameter gradients (a, b) of grad.
struct QfxReadoutRed {
  const float* rec;          // [S][2C + 2] (nullptr: no readout block)
  float* loss;               // [K]
  float* correct;            // [K]
  int C, n_theta;
};
