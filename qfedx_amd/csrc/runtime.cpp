// Native round scheduler (host runtime): the per-round minibatch plan of a rank's clients.
//
// For client k with n_k samples, step s and slot t of a B-sample minibatch:
//   epoch mode  (local_steps = 0): steps_k = epochs * ceil(n_k / B) (the reference's epochs x
//               len(dataloader), Classical_FL.py:56-62); step s reads epoch s / nb_k, batch s % nb_k; the
//               last batch of an epoch is partial (valid slots only, weights renormalised);
//   fixed steps (local_steps > 0): the epoch orders are walked cyclically, every slot valid.
// Epoch e's order is a keyed partial Fisher-Yates shuffle of 0..n_k-1 driven by Philox words with the
// client key = Philox(round key, client id) - so the plan depends on (seed, round, client id) only and
// is identical however clients are sharded over ranks.  Outputs (all host tensors):
//   idx int64 [S, K, B] (0 where invalid), wts float32 [S, K, B] (1 / #valid of the row),
//   active float32 [S, K] (s < steps_k), steps int64 [K];  S = max_k steps_k.
// Python oracle: fl/trainer.py BatchPlan._plan_torch.
#include <torch/extension.h>

#include <algorithm>
#include <numeric>
#include <stdexcept>
#include <vector>

#include "philox_core.h"

namespace qfx_runtime {

std::vector<torch::Tensor> batch_plan(torch::Tensor counts, torch::Tensor client_ids, int64_t B, int64_t rk0,
                                      int64_t rk1, int64_t local_epochs, int64_t local_steps, bool shuffle) {
  if (B <= 0) throw std::invalid_argument("batch_plan: batch size must be > 0");
  auto cn = counts.to(torch::kInt64).contiguous();
  auto ci = client_ids.to(torch::kInt64).contiguous();
  const int64_t K = cn.numel();
  if (ci.numel() != K) throw std::invalid_argument("batch_plan: counts / client_ids size mismatch");
  const int64_t* n = cn.data_ptr<int64_t>();
  const int64_t* id = ci.data_ptr<int64_t>();
  std::vector<int64_t> steps(K), epochs(K), nb(K);
  int64_t S = 0, E = 1, N = 1;
  for (int64_t k = 0; k < K; ++k) {
    nb[k] = (n[k] + B - 1) / B;
    if (local_steps > 0) {
      const int64_t nk = std::max<int64_t>(n[k], 1);
      steps[k] = local_steps;
      epochs[k] = (local_steps * B + nk - 1) / nk;
    } else {
      steps[k] = local_epochs * nb[k];
      epochs[k] = local_epochs;
    }
    S = std::max(S, steps[k]);
    E = std::max(E, epochs[k]);
    N = std::max(N, n[k]);
  }
  // per-client epoch orders perm[k][e][0:n_k] (only the first n_k entries are ever read)
  // Only the first m_e entries of epoch e's order are read (all n_k in epoch mode; the cyclic walk of
  // fixed-step mode stops after steps * B positions): a partial Fisher-Yates shuffle draws exactly those,
  // j-th swap partner r = j + (w_j * (n_k - j)) >> 32 with w_j the raw Philox word of element e*N + j
  // (Lemire's multiply-shift: integer-exact, no comparisons, no sort).
  std::vector<int32_t> perm((size_t)K * E * N);
  for (int64_t k = 0; k < K; ++k) {
    const int64_t nk = n[k];
    uint32_t ck0 = 0, ck1 = 0;
    if (shuffle) {
      const qfx::u32x4 o = qfx::philox4x32_10({(uint32_t)(id[k] & 0xFFFFFFFF), (uint32_t)((uint64_t)id[k] >> 32), 0u, 0u},
                                              (uint32_t)rk0, (uint32_t)rk1);
      ck0 = o.x;
      ck1 = o.y;
    }
    const int64_t used = local_steps > 0 ? steps[k] * B : epochs[k] * std::max<int64_t>(nk, 1);
    for (int64_t e = 0; e < E; ++e) {
      int32_t* pe = perm.data() + ((size_t)k * E + e) * N;
      const int64_t m = std::min<int64_t>(nk, used - e * std::max<int64_t>(nk, 1));
      if (m <= 0) continue;
      std::iota(pe, pe + nk, 0);
      if (!shuffle || nk <= 1) continue;
      uint64_t cur = ~0ull;
      uint32_t w[4] = {0, 0, 0, 0};
      const int64_t jmax = std::min<int64_t>(m, nk - 1);   // the last position has no choice left
      for (int64_t j = 0; j < jmax; ++j) {
        const uint64_t el = (uint64_t)(e * N + j);
        if ((el >> 2) != cur) {
          cur = el >> 2;
          const qfx::u32x4 o = qfx::philox4x32_10({(uint32_t)cur, (uint32_t)(cur >> 32), 0u, 0u}, ck0, ck1);
          w[0] = o.x; w[1] = o.y; w[2] = o.z; w[3] = o.w;
        }
        const int64_t r = j + (int64_t)(((uint64_t)w[el & 3] * (uint64_t)(nk - j)) >> 32);
        std::swap(pe[j], pe[r]);
      }
    }
  }
  auto idx = torch::zeros({S, K, B}, torch::kInt64);
  auto wts = torch::zeros({S, K, B}, torch::kFloat32);
  auto act = torch::zeros({S, K}, torch::kFloat32);
  auto stp = torch::empty({K}, torch::kInt64);
  int64_t* pi = idx.data_ptr<int64_t>();
  float* pw = wts.data_ptr<float>();
  float* pa = act.data_ptr<float>();
  for (int64_t k = 0; k < K; ++k) stp.data_ptr<int64_t>()[k] = steps[k];
  for (int64_t s = 0; s < S; ++s) {
    for (int64_t k = 0; k < K; ++k) {
      if (s >= steps[k]) continue;  // inactive: zeros
      pa[s * K + k] = 1.f;
      const int64_t nk = std::max<int64_t>(n[k], 1);
      int64_t* row = pi + (s * K + k) * B;
      float* wrow = pw + (s * K + k) * B;
      int64_t cnt = 0;
      for (int64_t t = 0; t < B; ++t) {
        int64_t ep, i;
        bool valid;
        if (local_steps > 0) {
          const int64_t pos = (s * B + t) % (epochs[k] * nk);
          ep = pos / nk;
          i = pos % nk;
          valid = true;
        } else {
          const int64_t nbk = std::max<int64_t>(nb[k], 1);
          ep = s / nbk;
          i = (s % nbk) * B + t;
          valid = i < n[k];
          if (!valid) i = 0;
        }
        ep = std::min(ep, E - 1);
        if (valid) {
          row[t] = perm[((size_t)k * E + ep) * N + i];
          ++cnt;
        }
        wrow[t] = valid ? 1.f : 0.f;
      }
      const float c = (float)std::max<int64_t>(cnt, 1);
      for (int64_t t = 0; t < B; ++t) wrow[t] = wrow[t] / c;
    }
  }
  return {idx, wts, act, stp};
}

}  // namespace qfx_runtime
