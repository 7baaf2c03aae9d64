// Bindings of the CNOT-chain MPS kernel (mps_chain.hip).  Launches go on torch's current HIP stream.
#include <c10/hip/HIPStream.h>
#include <torch/extension.h>

#include <cstdint>
#include <stdexcept>
#include <vector>

#include "mps_args.h"

extern "C" {
int qfx_mps_chain(const QfxMpsArgs* args, hipStream_t st);
}

namespace {

void need(bool ok, const std::string& msg) {
  if (!ok) throw std::invalid_argument("mps_chain: " + msg);
}

float* fp(const torch::Tensor& t, const char* name, int64_t numel) {
  need(t.defined() && t.is_cuda() && t.is_contiguous() && t.scalar_type() == torch::kFloat32,
       std::string(name) + ": expected a contiguous float32 CUDA tensor");
  need(t.numel() >= numel, std::string(name) + ": too small");
  return t.data_ptr<float>();
}

// x [S, >= n] angles, theta [K, >= 2 n L] per-client rows (spc samples each), readout qubit list; w [S, C] (or an
// empty tensor: <Z> only).  z [S, C] out; grad [S, 2 n L] out (gradient mode); rp / ro float32 scratch.
void mps_chain(torch::Tensor x, torch::Tensor theta, int64_t spc, int64_t n, int64_t L, int64_t feature,
               std::vector<int64_t> readout, torch::Tensor w, torch::Tensor z, torch::Tensor grad, torch::Tensor rp,
               torch::Tensor ro) {
  need(x.dim() == 2 && theta.dim() == 2, "x [S, F] and theta [K, P] expected");
  const int64_t S = x.size(0), C = (int64_t)readout.size();
  need(n >= 2 && L >= 1 && L <= 3 && x.size(1) >= n && theta.size(1) >= 2 * n * L, "shape / layer range");
  need(spc >= 1 && S == theta.size(0) * spc, "samples must be clients x spc");
  need(C >= 1 && C <= QFX_MPS_RMAX && feature >= 0 && feature <= 2, "1..8 readout qubits, feature 0..2");
  QfxMpsArgs a{};
  int qmax = 0;
  for (int64_t i = 0; i < C; ++i) {
    need(readout[i] >= 0 && readout[i] < n, "readout qubit out of range");
    a.readout[i] = (int)readout[i];
    qmax = std::max(qmax, (int)readout[i]);
  }
  const bool gmode = w.defined() && w.numel() > 0;
  a.x = fp(x, "x", S * x.size(1));
  a.theta = fp(theta, "theta", theta.numel());
  a.w = gmode ? fp(w, "w", S * C) : nullptr;
  a.z = fp(z, "z", S * C);
  a.grad = gmode ? fp(grad, "grad", S * 2 * n * L) : nullptr;
  a.rp = fp(rp, "rp", S * n * 64 * 2);
  a.ro = gmode ? fp(ro, "ro", S * (qmax + 1) * 64 * 2) : nullptr;
  a.x_stride = (int)x.size(1);
  a.t_stride = (int)theta.size(1);
  a.spc = (int)spc;
  a.S = (int)S;
  a.n = (int)n;
  a.L = (int)L;
  a.feature = (int)feature;
  a.C = (int)C;
  a.qmax = qmax;
  const int rc = qfx_mps_chain(&a, c10::hip::getCurrentHIPStream().stream());
  if (rc != 0) throw std::runtime_error("qfx_mps_chain failed: " + std::to_string(rc));
}

}  // namespace

void register_mps(pybind11::module& m) {
  m.def("mps_chain", &mps_chain, pybind11::arg("x"), pybind11::arg("theta"), pybind11::arg("spc"), pybind11::arg("n"),
        pybind11::arg("L"), pybind11::arg("feature"), pybind11::arg("readout"), pybind11::arg("w"), pybind11::arg("z"),
        pybind11::arg("grad"), pybind11::arg("rp"), pybind11::arg("ro"));
}
