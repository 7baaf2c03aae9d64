// Bindings of the client-batched TinyCNN kernels (cnn_kernels.hip).  All launches go on torch's current
// HIP stream (composable with graphs / stream semantics like the statevector ops).
#include <c10/hip/HIPStream.h>
#include <torch/extension.h>

#include <cstdint>
#include <stdexcept>
#include <vector>

#include "cnn_args.h"

extern "C" {
int qfx_cnn_mfma_probe(const float* A, const float* B, float* D, int K, hipStream_t st);
int qfx_cnn_forward(const float* X, const float* params, int P, int K, int B, const int* off4, float* pool1,
                    uint8_t* am1, float* pool2, uint8_t* am2, hipStream_t st);
int qfx_cnn_backward(const float* X, const float* params, int pstride, int P, int K, int B, const int* off4,
                     const float* pool1, const uint8_t* am1, const float* pool2, const uint8_t* am2, const float* dP2,
                     float* part, const CnnSgd* sink, hipStream_t st);
int qfx_cnn_head(const float* h1, int off_b1, const float* mask, const long long* dkeys, unsigned drop_stream,
                 float drop_p, float drop_scale, const float* params, int pstride, int P, int off_w, int off_b, int C,
                 int K, int B, const long long* y, const float* wts, float* dh1, float* dlog, float* loss,
                 float* correct, const CnnSgd* sink, hipStream_t st);
int qfx_cnn_partial_size();
int qfx_cnn_fc1_wgrad(const float* dh1, const float* pool2, int K, int B, const CnnSgd* sink, int P, int off_w1,
                      hipStream_t st);
int qfx_cnn_bwd_groups(int K, int B);
int qfx_cnn_fc1_forward(const float* pool2, const float* params, int P, int off_w1, int K, int B, float* h1p,
                        hipStream_t st);
int qfx_cnn_fc1_dgrad(const float* dh1, const float* params, int P, int off_w1, int K, int B, float* dP2,
                      hipStream_t st);
int qfx_cnn_eval_head(const float* h1p, const float* params, int P, int off_b1, int off_w, int off_b, int C, int K,
                      int B, const long long* y, float* logits, double* stats, hipStream_t st);
int qfx_cnn_fc1_splits();
int qfx_cnn_eval_blocks(int B);
}

namespace {

hipStream_t stream() { return c10::hip::getCurrentHIPStream().stream(); }

template <typename T>
T* dptr(const torch::Tensor& t, torch::ScalarType dt, const char* name, int64_t min_numel) {
  if (!t.defined() || t.scalar_type() != dt || !t.is_contiguous() || !t.is_cuda())
    throw std::invalid_argument(std::string("cnn: bad tensor ") + name);
  if (t.numel() < min_numel) throw std::invalid_argument(std::string("cnn: tensor too small: ") + name);
  return reinterpret_cast<T*>(t.data_ptr());
}

void check(int rc, const char* what) {
  if (rc != 0) throw std::runtime_error(std::string(what) + " failed: " + std::to_string(rc));
}

constexpr int64_t IMG = 28 * 28, POOL1 = 16 * 14 * 14, POOL2 = 32 * 7 * 7;

// Parameter rows the step kernels READ: a contiguous [K, P] tensor (row stride P) or the global parameters broadcast
// as theta.expand(K, P) (row stride 0: the first local step of a round reads theta, no per-client row copies).
const float* prm_rows(const torch::Tensor& p, int64_t K, int* stride, int* P) {
  if (!p.defined() || p.scalar_type() != torch::kFloat32 || !p.is_cuda() || p.dim() != 2 || p.size(0) < K ||
      p.stride(1) != 1 || !(p.stride(0) == 0 || p.stride(0) == p.size(1)) ||
      (p.stride(0) == p.size(1) && !p.is_contiguous()))
    throw std::invalid_argument("cnn: params must be a contiguous [K, P] fp32 CUDA tensor or theta.expand(K, P)");
  *stride = (int)p.stride(0);
  *P = (int)p.size(1);
  return p.data_ptr<float>();
}

// Gradient sink: the gradient rows ``grad`` [K, P], or (``sgd`` = [pin, pout, buf, t_in, t_out, act] tensors and
// ``hyper`` = [lr, mu, keep]) the fused SGD-momentum step of cnn_args.h - pin as prm_rows, pout / buf [K, P], t_in /
// t_out / act [K]; ``grad`` may then be empty.
CnnSgd make_sink(const torch::Tensor& grad, const c10::optional<std::vector<torch::Tensor>>& sgd,
                 const c10::optional<std::vector<double>>& hyper, int64_t K, int64_t P) {
  CnnSgd sk{};
  if (!sgd.has_value() || sgd->empty()) {
    if (grad.dim() != 2 || grad.size(0) < K || grad.size(1) != P)
      throw std::invalid_argument("cnn: grad must be [K, P]");
    sk.grad = dptr<float>(grad, torch::kFloat32, "grad", K * P);
    return sk;
  }
  const auto& v = *sgd;
  if (v.size() != 6 || !hyper.has_value() || hyper->size() != 3)
    throw std::invalid_argument("cnn: sgd = [pin, pout, buf, t_in, t_out, act], hyper = [lr, mu, keep]");
  int ps = 0, pp = 0;
  sk.pin = prm_rows(v[0], K, &ps, &pp);
  if (pp != P) throw std::invalid_argument("cnn: sgd pin row length");
  sk.pstride = ps;
  sk.pout = dptr<float>(v[1], torch::kFloat32, "pout", K * P);
  if (v[1].size(-1) != P) throw std::invalid_argument("cnn: sgd pout row length");
  sk.buf = dptr<float>(v[2], torch::kFloat32, "buf", K * P);
  sk.t_in = dptr<float>(v[3], torch::kFloat32, "t_in", K);
  sk.t_out = dptr<float>(v[4], torch::kFloat32, "t_out", K);
  sk.act = dptr<float>(v[5], torch::kFloat32, "act", K);
  sk.lr = (float)(*hyper)[0];
  sk.mu = (float)(*hyper)[1];
  sk.keep = (*hyper)[2] != 0.0;
  return sk;
}

void mfma_probe(torch::Tensor A, torch::Tensor B, torch::Tensor D, int64_t K) {
  check(qfx_cnn_mfma_probe(dptr<float>(A, torch::kFloat32, "A", 16 * K), dptr<float>(B, torch::kFloat32, "B", 16 * K),
                           dptr<float>(D, torch::kFloat32, "D", 256), (int)K, stream()),
        "mfma_probe");
}

void forward(torch::Tensor X, torch::Tensor params, int64_t K, int64_t B, std::vector<int64_t> off, torch::Tensor pool1,
             torch::Tensor am1, torch::Tensor pool2, torch::Tensor am2) {
  const int64_t S = K * B;
  int ps = 0, P = 0;
  const float* prm = prm_rows(params, K, &ps, &P);
  if (off.size() != 4) throw std::invalid_argument("cnn_forward: params/off");
  std::vector<int> o(off.begin(), off.end());
  check(qfx_cnn_forward(dptr<float>(X, torch::kFloat32, "X", S * IMG), prm,
                        ps, (int)K, (int)B, o.data(), dptr<float>(pool1, torch::kFloat32, "pool1", S * POOL1),
                        dptr<uint8_t>(am1, torch::kUInt8, "am1", S * POOL1), dptr<float>(pool2, torch::kFloat32, "pool2", S * POOL2),
                        dptr<uint8_t>(am2, torch::kUInt8, "am2", S * POOL2), stream()),
        "cnn_forward");
}

void backward(torch::Tensor X, torch::Tensor params, int64_t K, int64_t B, std::vector<int64_t> off, torch::Tensor pool1,
              torch::Tensor am1, torch::Tensor pool2, torch::Tensor am2, torch::Tensor dP2, torch::Tensor part,
              torch::Tensor grad, c10::optional<std::vector<torch::Tensor>> sgd,
              c10::optional<std::vector<double>> hyper) {
  const int64_t S = K * B;
  int ps = 0, P = 0;
  const float* prm = prm_rows(params, K, &ps, &P);
  const CnnSgd sink = make_sink(grad, sgd, hyper, K, P);
  std::vector<int> o(off.begin(), off.end());
  const int64_t G = qfx_cnn_bwd_groups((int)K, (int)B);
  check(qfx_cnn_backward(dptr<float>(X, torch::kFloat32, "X", S * IMG), prm,
                         ps, P, (int)K, (int)B, o.data(), dptr<float>(pool1, torch::kFloat32, "pool1", S * POOL1),
                         dptr<uint8_t>(am1, torch::kUInt8, "am1", S * POOL1), dptr<float>(pool2, torch::kFloat32, "pool2", S * POOL2),
                         dptr<uint8_t>(am2, torch::kUInt8, "am2", S * POOL2), dptr<float>(dP2, torch::kFloat32, "dP2", S * POOL2),
                         dptr<float>(part, torch::kFloat32, "part", K * G * qfx_cnn_partial_size()), &sink,
                         stream()),
        "cnn_backward");
}

// h1: the fc1 forward's split partial sums [K, FC_KS, B, 64] (cnn_fc1_forward); off_b1: fc1 bias offset in the parameter row (its gradient is written here).
// Dropout: ``mask`` [K*B, 64], or (mask undefined) per-client Philox keys ``dkeys`` [K, 2] (int64 words) whose
// uniforms of stream ``drop_stream`` are kept (x drop_scale) where u >= drop_p.
void head(torch::Tensor h1, int64_t off_b1, c10::optional<torch::Tensor> mask, c10::optional<torch::Tensor> dkeys,
          int64_t drop_stream, double drop_p, double drop_scale, torch::Tensor params, int64_t off_w, int64_t off_b, int64_t C, int64_t K,
          int64_t B, torch::Tensor y, torch::Tensor wts, torch::Tensor dh1, torch::Tensor dlog, torch::Tensor loss,
          torch::Tensor correct, torch::Tensor grad, c10::optional<std::vector<torch::Tensor>> sgd,
          c10::optional<std::vector<double>> hyper) {
  const int64_t S = K * B;
  int ps = 0, P = 0;
  const float* prm = prm_rows(params, K, &ps, &P);
  const CnnSgd sink = make_sink(grad, sgd, hyper, K, P);
  const bool hm = mask.has_value() && mask->defined(), hu = dkeys.has_value() && dkeys->defined();
  if (hm == hu) throw std::invalid_argument("cnn_head: pass exactly one of mask / dkeys");
  check(qfx_cnn_head(dptr<float>(h1, torch::kFloat32, "h1", S * 64 * qfx_cnn_fc1_splits()), (int)off_b1,
                     hm ? dptr<float>(*mask, torch::kFloat32, "mask", S * 64) : nullptr,
                     hu ? dptr<long long>(*dkeys, torch::kInt64, "dkeys", 2 * K) : nullptr, (unsigned)drop_stream,
                     (float)drop_p, (float)drop_scale,
                     prm, ps, P, (int)off_w, (int)off_b, (int)C, (int)K,
                     (int)B, dptr<long long>(y, torch::kInt64, "y", S), dptr<float>(wts, torch::kFloat32, "wts", S),
                     dptr<float>(dh1, torch::kFloat32, "dh1", S * 64), dptr<float>(dlog, torch::kFloat32, "dlog", S * 16),
                     dptr<float>(loss, torch::kFloat32, "loss", K), dptr<float>(correct, torch::kFloat32, "correct", K),
                     &sink, stream()),
        "cnn_head");
}

void fc1_wgrad(torch::Tensor dh1, torch::Tensor pool2, int64_t K, int64_t B, torch::Tensor grad, int64_t off_w1,
               c10::optional<std::vector<torch::Tensor>> sgd, c10::optional<std::vector<double>> hyper) {
  const int64_t S = K * B;
  const bool fused = sgd.has_value() && !sgd->empty();
  const int P = (int)(fused ? (*sgd)[1].size(-1) : grad.size(1));
  if (off_w1 < 0 || off_w1 + 64 * POOL2 > P) throw std::invalid_argument("cnn_fc1_wgrad: grad/offset");
  const CnnSgd sink = make_sink(grad, sgd, hyper, K, P);
  check(qfx_cnn_fc1_wgrad(dptr<float>(dh1, torch::kFloat32, "dh1", S * 64), dptr<float>(pool2, torch::kFloat32, "pool2", S * POOL2),
                          (int)K, (int)B, &sink, P, (int)off_w1, stream()),
        "cnn_fc1_wgrad");
}

void check_w1(const torch::Tensor& params, int64_t K, int64_t off_w1) {
  if (params.dim() != 2 || params.size(0) < K || off_w1 < 0 || off_w1 + 64 * POOL2 > params.size(1))
    throw std::invalid_argument("cnn fc1: params [K, P] / fc1 weight offset");
}

// h1p [K, FC_KS, B, 64]: per input-chunk partial sums of pool2 W1^T (no bias), summed in fixed order by the heads
void fc1_forward(torch::Tensor pool2, torch::Tensor params, int64_t off_w1, int64_t K, int64_t B, torch::Tensor h1p) {
  check_w1(params, K, off_w1);
  int ps = 0, P = 0;
  const float* prm = prm_rows(params, K, &ps, &P);
  check(qfx_cnn_fc1_forward(dptr<float>(pool2, torch::kFloat32, "pool2", K * B * POOL2),
                            prm, ps, (int)off_w1, (int)K, (int)B,
                            dptr<float>(h1p, torch::kFloat32, "h1p", K * B * 64 * qfx_cnn_fc1_splits()), stream()),
        "cnn_fc1_forward");
}

void fc1_dgrad(torch::Tensor dh1, torch::Tensor params, int64_t off_w1, int64_t K, int64_t B, torch::Tensor dP2) {
  check_w1(params, K, off_w1);
  int ps = 0, P = 0;
  const float* prm = prm_rows(params, K, &ps, &P);
  check(qfx_cnn_fc1_dgrad(dptr<float>(dh1, torch::kFloat32, "dh1", K * B * 64),
                          prm, ps, (int)off_w1, (int)K, (int)B,
                          dptr<float>(dP2, torch::kFloat32, "dP2", K * B * POOL2), stream()),
        "cnn_fc1_dgrad");
}

// logits [K*B, C]; with labels y [K*B] (int64), stats [K * eval_blocks(B), 2] float64 = per-block (CE sum, hits)
void eval_head(torch::Tensor h1p, torch::Tensor params, int64_t off_b1, int64_t off_w, int64_t off_b, int64_t C,
               int64_t K, int64_t B, c10::optional<torch::Tensor> y, torch::Tensor logits, torch::Tensor stats) {
  const int P = (int)params.size(1);
  const bool hy = y.has_value() && y->defined();
  check(qfx_cnn_eval_head(dptr<float>(h1p, torch::kFloat32, "h1p", K * B * 64 * qfx_cnn_fc1_splits()),
                          dptr<float>(params, torch::kFloat32, "params", K * P), P, (int)off_b1, (int)off_w, (int)off_b,
                          (int)C, (int)K, (int)B, hy ? dptr<long long>(*y, torch::kInt64, "y", K * B) : nullptr,
                          dptr<float>(logits, torch::kFloat32, "logits", K * B * C),
                          hy ? dptr<double>(stats, torch::kFloat64, "stats", 2 * K * qfx_cnn_eval_blocks((int)B))
                             : nullptr,
                          stream()),
        "cnn_eval_head");
}

}  // namespace

void register_cnn(pybind11::module& m) {
  m.def("cnn_mfma_probe", &mfma_probe);
  m.def("cnn_forward", &forward, "fused conv1/conv2 + bias + ReLU + maxpool (MFMA implicit GEMM)");
  m.def("cnn_backward", &backward, "conv stack backward -> deterministic per-client weight/bias grads",
        pybind11::arg("X"), pybind11::arg("params"), pybind11::arg("K"), pybind11::arg("B"), pybind11::arg("off"),
        pybind11::arg("pool1"), pybind11::arg("am1"), pybind11::arg("pool2"), pybind11::arg("am2"),
        pybind11::arg("dP2"), pybind11::arg("part"), pybind11::arg("grad"), pybind11::arg("sgd") = pybind11::none(),
        pybind11::arg("hyper") = pybind11::none());
  m.def("cnn_head", &head, "ReLU + dropout + fc2 + weighted CE fwd/bwd per client (+ fc1 bias gradient)",
        pybind11::arg("h1"), pybind11::arg("off_b1"), pybind11::arg("mask"), pybind11::arg("dkeys"),
        pybind11::arg("drop_stream"), pybind11::arg("drop_p"), pybind11::arg("drop_scale"), pybind11::arg("params"),
        pybind11::arg("off_w"), pybind11::arg("off_b"), pybind11::arg("C"), pybind11::arg("K"), pybind11::arg("B"),
        pybind11::arg("y"), pybind11::arg("wts"), pybind11::arg("dh1"), pybind11::arg("dlog"), pybind11::arg("loss"),
        pybind11::arg("correct"), pybind11::arg("grad"), pybind11::arg("sgd") = pybind11::none(),
        pybind11::arg("hyper") = pybind11::none());
  m.def("cnn_partial_size", []() { return qfx_cnn_partial_size(); });
  m.def("cnn_fc1_wgrad", &fc1_wgrad, "fc1 weight gradient into the flat [K, P] gradient rows (MFMA)",
        pybind11::arg("dh1"), pybind11::arg("pool2"), pybind11::arg("K"), pybind11::arg("B"), pybind11::arg("grad"),
        pybind11::arg("off_w1"), pybind11::arg("sgd") = pybind11::none(), pybind11::arg("hyper") = pybind11::none());
  m.def("cnn_bwd_groups", [](int64_t K, int64_t B) { return qfx_cnn_bwd_groups((int)K, (int)B); });
  m.def("cnn_fc1_forward", &fc1_forward, "fc1 pre-activation partial sums [K, FC_KS, B, 64] (MFMA, split inputs)");
  m.def("cnn_fc1_dgrad", &fc1_dgrad, "fc1 input gradient dL/dpool2 [K*B, 1568] (MFMA)");
  m.def("cnn_eval_head", &eval_head, "eval: fc1 partials + bias + ReLU + fc2 -> logits, fused CE / argmax-hit sums");
  m.def("cnn_fc1_splits", []() { return qfx_cnn_fc1_splits(); });
  m.def("cnn_eval_blocks", [](int64_t B) { return qfx_cnn_eval_blocks((int)B); });
}
