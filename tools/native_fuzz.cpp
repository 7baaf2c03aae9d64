// Host-side fuzz harness for the native planner + JIT code generator (no GPU).  Built with
// AddressSanitizer + UndefinedBehaviorSanitizer by tools/sanitize_host.sh: random circuits (all gate
// kinds incl. noise Paulis, random qubit counts / readouts / register sizes) go through
// plan_circuit() for the forward, loading and adjoint modes, every pass is code-generated (fp32 and
// bf16 storage), and the blob invariants the kernels rely on are checked.  GPU AddressSanitizer and
// XNACK are not available on the GPU pool, so the host code is where memory errors are hunted.
#include <cstdio>
#include <cstdlib>
#include <random>
#include <stdexcept>
#include <string>
#include <vector>

#include "../qfedx_amd/csrc/qfx_plan.h"

namespace qfx {
std::vector<int> plan_circuit(int n, int R, int kmax, const std::vector<int>& ops_i, const std::vector<float>& coef,
                              const std::vector<int>& readout, int n_theta, int mode, int final_flags);
std::string jit_source(const std::vector<int>& blob, int p, bool adjoint, bool bf16);
}

using namespace qfx;

static void require(bool c, const char* what, int it) {
  if (!c) {
    std::fprintf(stderr, "invariant failed at iteration %d: %s\n", it, what);
    std::exit(1);
  }
}

int main(int argc, char** argv) {
  const int iters = argc > 1 ? std::atoi(argv[1]) : 300;
  std::mt19937 rng(12345);
  auto U = [&](int a, int b) { return std::uniform_int_distribution<int>(a, b)(rng); };
  long passes = 0, chars = 0;
  for (int it = 0; it < iters; ++it) {
    const int n = U(1, 18);
    const int R = n >= 4 ? 16 : 4;
    const int kmax = U(std::min(n, 4), 12);
    const int G = U(1, 60);
    const int n_theta = U(0, 12);
    std::vector<int> ops;
    std::vector<float> coef;
    int n_slots = n_theta + n;
    for (int g = 0; g < G; ++g) {
      int kind = U(0, 15);
      if (kind == K_SWAP) kind = K_CX;
      if (U(0, 9) == 0) kind = K_PAULI;
      const bool two = kind == K_CX || kind == K_CZ;
      if (two && n < 2) kind = K_H;
      const int q0 = U(0, n - 1);
      int q1 = -1;
      if (kind == K_CX || kind == K_CZ) {
        do { q1 = U(0, n - 1); } while (q1 == q0);
      }
      int slot = -1;
      if (kind <= K_P || kind == K_PAULI) slot = U(-1, n_slots - 1);
      ops.insert(ops.end(), {kind, q0, q1, slot});
      coef.insert(coef.end(), {1.0f, 0.25f * (float)U(-8, 8)});
    }
    std::vector<int> readout;
    const int C = U(1, std::min(n, 8));
    for (int c = 0; c < C; ++c) readout.push_back(c);
    for (int mode = 0; mode < 3; ++mode) {
      const int fin = mode == 2 ? 0 : U(1, 3);
      std::vector<int> blob;
      try {
        blob = qfx::plan_circuit(n, R, kmax, ops, coef, readout, n_theta, mode, fin);
      } catch (const std::invalid_argument&) {
        continue;   // rejected configurations are fine; memory errors are not
      }
      require(blob.size() > (size_t)HF_PASSES, "blob header", it);
      const int np = blob[1];
      require(np >= 1 && np < 1000, "pass count", it);
      for (int p = 0; p < np; ++p) {
        const int off = blob[HF_PASSES + p];
        require(off > 0 && off < (int)blob.size(), "pass offset", it);
        for (int bf = 0; bf < 2; ++bf) {
          const std::string src = qfx::jit_source(blob, p, mode == 2, bf == 1);
          require(src.find("qfx_jit_pass") != std::string::npos, "kernel entry", it);
          chars += (long)src.size();
        }
        ++passes;
      }
    }
  }
  std::printf("native fuzz ok: %d circuits, %ld passes, %ld chars of generated source\n", iters, passes, chars);
  return 0;
}
