// Bindings of the CNOT-chain MPS kernel (mps_chain.hip).  Launches go on torch's current HIP stream.
#include <c10/hip/HIPStream.h>
#include <torch/extension.h>

#include <cstdint>
#include <stdexcept>
#include <vector>

#include "mps_args.h"

extern "C" {
int qfx_mps_chain(const QfxMpsArgs* args, hipStream_t st);
int qfx_mps_mpo(const QfxMpoArgs* args, hipStream_t st);
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
// Fused readout (y defined, non-empty; w then empty): theta rows hold the readout a / b at ro_off / ro_off + C, y [S]
// int64 labels, wts [S] loss weights; out dl [S, C] (dL/dlogit), lossv / hitv [S]; z [S, C] and grad as usual.
void mps_chain(torch::Tensor x, torch::Tensor theta, int64_t spc, int64_t n, int64_t L, int64_t feature,
               std::vector<int64_t> readout, torch::Tensor w, torch::Tensor z, torch::Tensor grad, torch::Tensor rp,
               torch::Tensor ro, c10::optional<torch::Tensor> y, c10::optional<torch::Tensor> wts, int64_t ro_off,
               c10::optional<torch::Tensor> dl, c10::optional<torch::Tensor> lossv, c10::optional<torch::Tensor> hitv) {
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
  const bool fused = y.has_value() && y->defined() && y->numel() > 0;
  const bool gmode = (w.defined() && w.numel() > 0) || fused;
  a.x = fp(x, "x", S * x.size(1));
  a.theta = fp(theta, "theta", theta.numel());
  a.w = (gmode && !fused) ? fp(w, "w", S * C) : nullptr;
  if (fused) {
    need(y->is_cuda() && y->is_contiguous() && y->scalar_type() == torch::kInt64 && y->numel() >= S, "y: int64 [S]");
    need(ro_off >= 2 * n * L && ro_off + 2 * C <= theta.size(1), "readout a / b outside the theta rows");
    a.y = reinterpret_cast<const long long*>(y->data_ptr<int64_t>());
    a.wts = fp(*wts, "wts", S);
    a.ro_off = (int)ro_off;
    a.dl = fp(*dl, "dl", S * C);
    a.lossv = fp(*lossv, "lossv", S);
    a.hitv = fp(*hitv, "hitv", S);
  }
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

const int* ip(const torch::Tensor& t, const char* name, int64_t numel) {
  need(t.defined() && t.is_cuda() && t.is_contiguous() && t.scalar_type() == torch::kInt32,
       std::string(name) + ": expected a contiguous int32 CUDA tensor");
  need(t.numel() >= numel, std::string(name) + ": too small");
  return t.data_ptr<int>();
}

// Generic MPO-product MPS (mps_mpo.hip): ang [S, G] gate angles, tables from quantum/mps_mpo.compile_mpo (gkind [G],
// events, sinfo [n, 8], nbits [n - 1]), readout qubits; w [S, C] or empty (<Z> only).  z [S, C] out; dang [S, G]
// (gradient mode: RX / RY / RZ / P entries written); rp / ro float32 scratch (complex [S, n, 256] / [S, qmax + 1, 256]).
void mps_mpo(torch::Tensor ang, torch::Tensor gkind, torch::Tensor events, torch::Tensor sinfo, torch::Tensor nbits,
             torch::Tensor sinfo_host, torch::Tensor nbits_host, std::vector<int64_t> readout, torch::Tensor w, torch::Tensor z, torch::Tensor dang, torch::Tensor rp,
             torch::Tensor ro) {
  need(ang.dim() == 2 && sinfo.dim() == 2 && sinfo.size(1) == 8, "ang [S, G], sinfo [n, 8] expected");
  const int64_t S = ang.size(0), G = ang.size(1), n = sinfo.size(0), C = (int64_t)readout.size();
  need(n >= 2 && nbits.numel() == n - 1 && gkind.numel() == G, "table shapes");
  need(C >= 1 && C <= QFX_MPS_RMAX, "1..8 readout qubits");
  // the same tables on the host (no device sync): every bond <= 16, every site's event range inside the list
  need(!sinfo_host.is_cuda() && !nbits_host.is_cuda() && sinfo_host.scalar_type() == torch::kInt32 &&
           nbits_host.scalar_type() == torch::kInt32 && sinfo_host.is_contiguous() && nbits_host.is_contiguous() &&
           sinfo_host.numel() == n * 8 && nbits_host.numel() == n - 1, "host tables");
  const int* si = sinfo_host.data_ptr<int>();
  const int* nb = nbits_host.data_ptr<int>();
  for (int64_t c = 0; c < n - 1; ++c) need(nb[c] >= 0 && (1 << nb[c]) <= QFX_MPO_DMAX, "bond over 16");
  for (int64_t q = 0; q < n; ++q)
    need(si[8 * q] >= 0 && si[8 * q] + si[8 * q + 1] <= events.numel() && si[8 * q + 3] <= 4 &&
             si[8 * q + 4] <= QFX_MPO_MAXPG, "site table");
  QfxMpoArgs a{};
  int qmax = 0;
  for (int64_t i = 0; i < C; ++i) {
    need(readout[i] >= 0 && readout[i] < n, "readout qubit out of range");
    a.readout[i] = (int)readout[i];
    qmax = std::max(qmax, (int)readout[i]);
  }
  const bool gmode = w.defined() && w.numel() > 0;
  a.ang = fp(ang, "ang", S * G);
  a.gkind = ip(gkind, "gkind", G);
  a.events = ip(events, "events", events.numel());
  a.sinfo = ip(sinfo, "sinfo", n * 8);
  a.nbits = ip(nbits, "nbits", n - 1);
  a.w = gmode ? fp(w, "w", S * C) : nullptr;
  a.z = fp(z, "z", S * C);
  a.dang = gmode ? fp(dang, "dang", S * G) : nullptr;
  a.rp = fp(rp, "rp", S * n * 256 * 2);
  a.ro = gmode ? fp(ro, "ro", S * (qmax + 1) * 256 * 2) : nullptr;
  a.S = (int)S;
  a.G = (int)G;
  a.n = (int)n;
  a.C = (int)C;
  a.qmax = qmax;
  const int rc = qfx_mps_mpo(&a, c10::hip::getCurrentHIPStream().stream());
  if (rc != 0) throw std::runtime_error("qfx_mps_mpo failed: " + std::to_string(rc));
}

}  // namespace

void register_mps(pybind11::module& m) {
  m.def("mps_chain", &mps_chain, pybind11::arg("x"), pybind11::arg("theta"), pybind11::arg("spc"), pybind11::arg("n"),
        pybind11::arg("L"), pybind11::arg("feature"), pybind11::arg("readout"), pybind11::arg("w"), pybind11::arg("z"),
        pybind11::arg("grad"), pybind11::arg("rp"), pybind11::arg("ro"), pybind11::arg("y") = pybind11::none(),
        pybind11::arg("wts") = pybind11::none(), pybind11::arg("ro_off") = 0, pybind11::arg("dl") = pybind11::none(),
        pybind11::arg("lossv") = pybind11::none(), pybind11::arg("hitv") = pybind11::none());
  m.def("mps_mpo", &mps_mpo, pybind11::arg("ang"), pybind11::arg("gkind"), pybind11::arg("events"),
        pybind11::arg("sinfo"), pybind11::arg("nbits"), pybind11::arg("sinfo_host"), pybind11::arg("nbits_host"),
        pybind11::arg("readout"), pybind11::arg("w"), pybind11::arg("z"),
        pybind11::arg("dang"), pybind11::arg("rp"), pybind11::arg("ro"));
}
