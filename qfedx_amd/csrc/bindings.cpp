// Python bindings of the qfedx_amd native runtime (pybind11 + torch tensors).
//
// Host planner (planner.cpp) and launchers of the gfx950 kernels (statevec.hip, train_kernels.hip,
// cnn_kernels.hip).  Every launch goes on torch's CURRENT HIP stream, so the ops compose with
// torch's stream semantics, ``torch.cuda.graph`` capture (hipGraph) and the comm-stream overlap of
// the federated runtime.  Shapes are validated here, on the host, before any kernel is launched.
#include <c10/hip/HIPStream.h>
#include <torch/extension.h>

#include <stdexcept>
#include <string>
#include <vector>

namespace py = pybind11;

namespace qfx {
std::vector<int> plan_circuit(int n, int R, int kmax, const std::vector<int>& ops_i,
                              const std::vector<float>& coef, const std::vector<int>& readout,
                              int n_theta, int mode, int final_flags);
}

namespace qfx {
struct PassArgsHost {
  const int* blob;
  int pass_off;
  void* psi;
  void* lam;
  const float* params;
  int p_stride;
  int spc;
  const float* xang;
  int x_stride;
  const float* w_read;
  float* out_read;
  float* gslab;
  int n_samples;
  int n_grad;
};
int jit_prepare(const std::vector<int>& blob, int p, bool adjoint, const std::string& cache_dir,
                const std::string& include_dir, const std::string& arch, std::string* key_out, bool bf16);
int jit_launch(int handle, const PassArgsHost& args, hipStream_t stream);
std::string jit_source(const std::vector<int>& blob, int p, bool adjoint, bool bf16);
long jit_state_bytes(int handle, bool* bf16);
}  // namespace qfx

extern "C" {
int qfx_launch_pass(int R, int adjoint, const int* blob, int pass_off, int k, int n, int n_ops, int n_gates, void* psi, void* lam,
                    const float* params, int p_stride, int spc, const float* xang, int x_stride,
                    const float* w_read, float* out_read, float* gslab, int n_samples, int n_grad_ops,
                    hipStream_t stream);
int qfx_launch_readout_ce(const float* part, int tps, int C, int spc, int K, const long long* y, const float* wts,
                          const float* params, int p_stride, int n_theta, float* expz, float* w_out, float* loss,
                          float* correct, float* grad, int write_grad, float p01, float p10, int shots,
                          const long long* keys, unsigned stream, hipStream_t st);
int qfx_launch_readout_noise(float* expz, int C, int spc, long n_samples, float p01, float p10, int shots,
                             const long long* keys, unsigned stream, hipStream_t st);
int qfx_launch_philox_uniform(const long long* keys, int K, long n, unsigned stream, float* out, hipStream_t st);
int qfx_launch_readout_sum(const float* part, int tps, int C, long n_samples, float* expz, hipStream_t st);
int qfx_amp_scratch(long F);
int qfx_launch_amp_init(const float* x, long F, long ld, int n_samples, int n, double* part, void* psi, int bf16,
                        hipStream_t stream);
int qfx_launch_grad_reduce(const float* slab, int tps, int spc, int K, int G, const int* blob, const int* csr,
                           float* grad,
                           int p_stride, float* gpart, hipStream_t st);
int qfx_grad_split(int tps, int spc);
int qfx_launch_round_pack(long long* buf, int P, const float* loss, const float* correct, const float* nvalid,
                          const float* act, int n, hipStream_t st);
int qfx_launch_round_apply(long long* buf, int P, float* theta, double lr, double* out, int bits,
                           double ring_scale, int n_norms, hipStream_t st);
int qfx_fedavg_norm_scratch(int K, int P);
int qfx_launch_adam(float* p, const float* g, float* m, float* v, const float* t_in, float* t_out,
                    const float* active, int K, int P, float lr, float b1, float b2, float eps, hipStream_t st);
int qfx_launch_sgdm(float* p, const float* g, float* buf, const float* t_in, float* t_out, const float* active,
                    int K, int P, float lr, float mu, int keep, hipStream_t st);
int qfx_launch_host_upload(const void* host_src, void* dst, long nbytes, long long* ctr, long long* host_flag,
                           hipStream_t st);
int qfx_launch_ps_combine(const float* f0, const float* fpi, const float* jac, const float* w, const long long* keys,
                          float p01, float p10, int shots, unsigned stream, int K, int P, int B, int C, int noisy,
                          float* out, hipStream_t st);
int qfx_launch_round_init(const float* theta, int K, int P, float* params, float* m, float* v, float* t, int nt,
                          hipStream_t st);
int qfx_launch_round_prologue(const float* theta, int K, int P, float* params, float* m, float* v, float* t, int nt,
                              const float* X, const long long* Y, const long long* lid, const long long* idx,
                              int steps, int B, long nmax, int F, int mode, float alpha, float* xo, int x_stride,
                              long long* yo, const int* slot_tab, int n_slots, void* frags, int bf16, long long* zero,
                              int nzero, const void* up_host, void* up_dst, long up_nbytes, long long* up_ctr,
                              long long* up_flag, hipStream_t st);
int qfx_prologue_gather_lanes(int F);
int qfx_launch_batch_gather(const float* X, const long long* Y, const long long* lid, const long long* idx, int K,
                            int B, long nmax, int F, int mode, float alpha, float* xo, int x_stride, long long* yo,
                            hipStream_t st);
int qfx_launch_fedavg(const float* theta_k, const float* theta_g, const unsigned char* angle_mask,
                      const double* weights, double* norms, const uint32_t* keys, int K, int P, int wrap, int dp,
                      float clip, float sigma, long long* out, long long* pack_buf, const float* loss,
                      const float* correct, const float* nvalid, const float* act, int n_metrics, long long* sat,
                      const uint32_t* sa_seeds, const int* sa_sign, const int* sa_round, int sa_n, double sa_scale,
                      int sa_bits, long long* sa_masks, const int* norm_cid, float* fa_theta, double* fa_out,
                      unsigned* fa_cnt, int fa_bits, double fa_ring_scale, int fa_n_norms, const float* dp_scale,
                      int sa_pairsym, hipStream_t st);
}

namespace qfx_runtime {
std::vector<torch::Tensor> batch_plan(torch::Tensor counts, torch::Tensor client_ids, int64_t B, int64_t rk0,
                                      int64_t rk1, int64_t local_epochs, int64_t local_steps, bool shuffle);
}

namespace {

hipStream_t cur_stream() { return c10::hip::getCurrentHIPStream().stream(); }

void check(int rc, const char* what) {
  if (rc != 0) throw std::runtime_error(std::string(what) + " failed: hip error " + std::to_string(rc));
}

template <typename T>
T* ptr(const torch::Tensor& t) { return t.defined() && t.numel() > 0 ? reinterpret_cast<T*>(t.data_ptr()) : nullptr; }

void need(const torch::Tensor& t, torch::ScalarType dt, const char* name) {
  if (!t.defined()) throw std::invalid_argument(std::string(name) + " is undefined");
  if (t.scalar_type() != dt) throw std::invalid_argument(std::string(name) + " has wrong dtype");
  if (!t.is_contiguous()) throw std::invalid_argument(std::string(name) + " must be contiguous");
  if (!t.is_cuda()) throw std::invalid_argument(std::string(name) + " must be a GPU tensor");
}

torch::Tensor plan(torch::Tensor ops, torch::Tensor coef, int64_t n, int64_t R, int64_t kmax,
                   std::vector<int64_t> readout, int64_t n_theta, int64_t mode, int64_t final_flags) {
  auto o = ops.to(torch::kInt32).contiguous().cpu();
  auto c = coef.to(torch::kFloat32).contiguous().cpu();
  std::vector<int> oi(o.data_ptr<int>(), o.data_ptr<int>() + o.numel());
  std::vector<float> cf(c.data_ptr<float>(), c.data_ptr<float>() + c.numel());
  std::vector<int> ro(readout.begin(), readout.end());
  auto blob = qfx::plan_circuit((int)n, (int)R, (int)kmax, oi, cf, ro, (int)n_theta, (int)mode, (int)final_flags);
  auto out = torch::empty({(int64_t)blob.size()}, torch::kInt32);
  std::copy(blob.begin(), blob.end(), out.data_ptr<int>());
  return out;
}

void pass_launch(int64_t R, bool adjoint, torch::Tensor blob, int64_t pass_off, int64_t k, int64_t n, int64_t n_ops, int64_t n_gates,
                 torch::Tensor psi, c10::optional<torch::Tensor> lam, torch::Tensor params, int64_t spc,
                 torch::Tensor xang, c10::optional<torch::Tensor> w_read, c10::optional<torch::Tensor> out_read,
                 c10::optional<torch::Tensor> gslab, int64_t n_samples, int64_t n_grad_ops) {
  need(blob, torch::kInt32, "blob");
  need(psi, torch::kComplexFloat, "psi");
  need(params, torch::kFloat32, "params");
  need(xang, torch::kFloat32, "xang");
  if (psi.numel() < (n_samples << n)) throw std::invalid_argument("psi too small for n_samples x 2^n");
  if (xang.size(0) < n_samples) throw std::invalid_argument("xang rows < n_samples");
  if (params.size(0) * spc < n_samples) throw std::invalid_argument("params rows * spc < n_samples");
  torch::Tensor lt = lam.has_value() ? *lam : torch::Tensor();
  torch::Tensor wt = w_read.has_value() ? *w_read : torch::Tensor();
  torch::Tensor ot = out_read.has_value() ? *out_read : torch::Tensor();
  torch::Tensor gs = gslab.has_value() ? *gslab : torch::Tensor();
  if (adjoint) {
    need(lt, torch::kComplexFloat, "lam");
    need(gs, torch::kFloat32, "gslab");
    if (lt.numel() < psi.numel()) throw std::invalid_argument("lam smaller than psi");
  }
  check(qfx_launch_pass((int)R, adjoint ? 1 : 0, ptr<int>(blob), (int)pass_off, (int)k, (int)n, (int)n_ops, (int)n_gates, ptr<float2>(psi),
                        ptr<float2>(lt), ptr<float>(params), (int)params.size(1), (int)spc, ptr<float>(xang),
                        (int)xang.size(1), ptr<float>(wt), ptr<float>(ot), ptr<float>(gs), (int)n_samples,
                        (int)n_grad_ops, cur_stream()),
        "qfx_pass");
}

void readout_ce(torch::Tensor part, int64_t tps, int64_t C, int64_t spc, int64_t K, torch::Tensor y,
                torch::Tensor wts, torch::Tensor params, int64_t n_theta, torch::Tensor expz, torch::Tensor w_out,
                torch::Tensor loss, torch::Tensor correct, torch::Tensor grad, bool write_grad, double p01,
                double p10, int64_t shots, torch::Tensor keys, int64_t stream) {
  need(part, torch::kFloat32, "part");
  need(y, torch::kInt64, "y");
  need(wts, torch::kFloat32, "wts");
  need(params, torch::kFloat32, "params");
  if (y.numel() < K * spc || wts.numel() < K * spc) throw std::invalid_argument("y/wts too small");
  check(qfx_launch_readout_ce(ptr<float>(part), (int)tps, (int)C, (int)spc, (int)K, ptr<long long>(y),
                              ptr<float>(wts), ptr<float>(params), (int)params.size(1), (int)n_theta,
                              ptr<float>(expz), ptr<float>(w_out), ptr<float>(loss), ptr<float>(correct),
                              ptr<float>(grad), write_grad ? 1 : 0, (float)p01, (float)p10, (int)shots,
                              keys.numel() ? ptr<long long>(keys) : nullptr, (unsigned)stream, cur_stream()),
        "qfx_readout_ce");
}

void readout_noise(torch::Tensor expz, int64_t C, int64_t spc, int64_t n_samples, double p01, double p10,
                   int64_t shots, torch::Tensor keys, int64_t stream) {
  need(expz, torch::kFloat32, "expz");
  if (shots > 0) need(keys, torch::kInt64, "keys");
  check(qfx_launch_readout_noise(ptr<float>(expz), (int)C, (int)spc, (long)n_samples, (float)p01, (float)p10,
                                 (int)shots, keys.numel() ? ptr<long long>(keys) : nullptr, (unsigned)stream,
                                 cur_stream()),
        "qfx_readout_noise");
}

void philox_uniform(torch::Tensor keys, int64_t n, int64_t stream, torch::Tensor out) {
  need(keys, torch::kInt64, "keys");
  need(out, torch::kFloat32, "out");
  if (out.numel() < keys.size(0) * n) throw std::invalid_argument("philox_uniform: out too small");
  check(qfx_launch_philox_uniform(ptr<long long>(keys), (int)keys.size(0), (long)n, (unsigned)stream,
                                  ptr<float>(out), cur_stream()),
        "qfx_philox_uniform");
}

// amplitude encoding straight into pass storage: x [S, F] fp32 (row stride ld), psi complex64 [S, 2^n] or
// int32 [S, 2^n] (packed bf16x2)
void amp_init(torch::Tensor x, int64_t n, torch::Tensor part, torch::Tensor psi) {
  need(x, torch::kFloat32, "x");
  need(part, torch::kFloat64, "part");
  if (x.dim() != 2 || x.stride(1) != 1) throw std::invalid_argument("amp_init: x must be [S, F] with unit inner stride");
  const int64_t S = x.size(0), F = x.size(1);
  if (n < 1 || n > 34 || F > (int64_t(1) << n)) throw std::invalid_argument("amp_init: need F <= 2^n");
  const bool bf16 = psi.scalar_type() == torch::kInt32;
  if (!bf16 && psi.scalar_type() != torch::kComplexFloat)
    throw std::invalid_argument("amp_init: psi must be complex64 or int32 (bf16x2)");
  if (!psi.is_contiguous() || psi.numel() < (S << n)) throw std::invalid_argument("amp_init: psi too small");
  if (part.numel() < S * qfx_amp_scratch((long)F)) throw std::invalid_argument("amp_init: scratch too small");
  check(qfx_launch_amp_init(ptr<float>(x), (long)F, (long)x.stride(0), (int)S, (int)n, ptr<double>(part),
                            psi.data_ptr(), bf16 ? 1 : 0, cur_stream()),
        "qfx_amp_init");
}

int64_t amp_scratch(int64_t F) { return qfx_amp_scratch((long)F); }

void readout_sum(torch::Tensor part, int64_t tps, int64_t C, int64_t n_samples, torch::Tensor expz) {
  need(part, torch::kFloat32, "part");
  need(expz, torch::kFloat32, "expz");
  check(qfx_launch_readout_sum(ptr<float>(part), (int)tps, (int)C, (long)n_samples, ptr<float>(expz), cur_stream()),
        "qfx_readout_sum");
}

int64_t grad_split(int64_t tps, int64_t spc) { return qfx_grad_split((int)tps, (int)spc); }

void round_pack(torch::Tensor buf, int64_t P, torch::Tensor loss, torch::Tensor correct, torch::Tensor nvalid,
                torch::Tensor act) {
  need(buf, torch::kInt64, "buf");
  for (auto* x : {&loss, &correct, &nvalid, &act}) need(*x, torch::kFloat32, "round_pack metric");
  const int64_t n = loss.numel();
  if (buf.numel() < P + 5 || correct.numel() < n || nvalid.numel() < n || act.numel() < n)
    throw std::invalid_argument("round_pack: sizes");
  check(qfx_launch_round_pack(ptr<long long>(buf), (int)P, ptr<float>(loss), ptr<float>(correct), ptr<float>(nvalid),
                              ptr<float>(act), (int)n, cur_stream()),
        "qfx_round_pack");
}

// bits > 0: the update / weight entries are SecAgg ring elements (Z_2^bits, scale ring_scale)
// n_norms: per-client norm slots buf[P + 6 ..] (CC6) copied to out[6 ..] and zeroed
void round_apply(torch::Tensor buf, int64_t P, torch::Tensor theta, double lr, torch::Tensor out, int64_t bits,
                 double ring_scale, int64_t n_norms) {
  need(buf, torch::kInt64, "buf");
  need(theta, torch::kFloat32, "theta");
  need(out, torch::kFloat64, "out");
  if (buf.numel() < P + 6 + n_norms || theta.numel() < P || out.numel() < 6 + n_norms)
    throw std::invalid_argument("round_apply: sizes");
  check(qfx_launch_round_apply(ptr<long long>(buf), (int)P, ptr<float>(theta), lr, ptr<double>(out), (int)bits,
                               ring_scale, (int)n_norms, cur_stream()),
        "qfx_round_apply");
}

// csr: int32 [n_theta + 1 + n_entries] slot -> gradient-gate CSR (ops/statevec_hip.py slot_csr)
void grad_reduce(torch::Tensor slab, int64_t tps, int64_t spc, int64_t K, int64_t G, torch::Tensor blob,
                 torch::Tensor csr, torch::Tensor grad, torch::Tensor gpart) {
  need(slab, torch::kFloat32, "slab");
  need(csr, torch::kInt32, "csr");
  need(grad, torch::kFloat32, "grad");
  need(gpart, torch::kFloat32, "gpart");
  if (slab.numel() < K * spc * tps * G) throw std::invalid_argument("grad slab too small");
  if (gpart.numel() < K * grad_split(tps, spc) * G) throw std::invalid_argument("gpart too small");
  check(qfx_launch_grad_reduce(ptr<float>(slab), (int)tps, (int)spc, (int)K, (int)G, ptr<int>(blob),
                               ptr<int>(csr), ptr<float>(grad), (int)grad.size(1), ptr<float>(gpart), cur_stream()),
        "qfx_grad_reduce");
}

void check_counters(const torch::Tensor& p, const torch::Tensor& t_in, const torch::Tensor& t_out,
                    const torch::Tensor& active) {
  for (auto* x : {&t_in, &t_out, &active}) need(*x, torch::kFloat32, "optimizer counter/mask");
  if (t_in.numel() < p.size(0) || t_out.numel() < p.size(0) || active.numel() < p.size(0))
    throw std::invalid_argument("optimizer: counters / mask need one entry per client row");
  if (t_in.data_ptr() == t_out.data_ptr()) throw std::invalid_argument("optimizer: t_in and t_out must differ");
}

void adam(torch::Tensor p, torch::Tensor g, torch::Tensor m, torch::Tensor v, torch::Tensor t_in, torch::Tensor t_out,
          torch::Tensor active, double lr, double b1, double b2, double eps) {
  for (auto* x : {&p, &g, &m, &v}) need(*x, torch::kFloat32, "adam tensor");
  check_counters(p, t_in, t_out, active);
  check(qfx_launch_adam(ptr<float>(p), ptr<float>(g), ptr<float>(m), ptr<float>(v), ptr<float>(t_in),
                        ptr<float>(t_out), ptr<float>(active), (int)p.size(0), (int)p.size(1), (float)lr, (float)b1,
                        (float)b2, (float)eps, cur_stream()),
        "qfx_adam");
}

void sgdm(torch::Tensor p, torch::Tensor g, torch::Tensor buf, torch::Tensor t_in, torch::Tensor t_out,
          torch::Tensor active, double lr, double mu, bool keep_state) {
  for (auto* x : {&p, &g, &buf}) need(*x, torch::kFloat32, "sgd tensor");
  check_counters(p, t_in, t_out, active);
  check(qfx_launch_sgdm(ptr<float>(p), ptr<float>(g), ptr<float>(buf), ptr<float>(t_in), ptr<float>(t_out),
                        ptr<float>(active), (int)p.size(0), (int)p.size(1), (float)lr, (float)mu, keep_state ? 1 : 0,
                        cur_stream()),
        "qfx_sgdm");
}

// params[k, :] = theta; optional m, v (same shape) and t (any length) zeroed
// Pinned host staging memory allocated mapped + portable (device-readable from every GPU of the process, whatever
// the current device was at allocation), as a CPU uint8 tensor that frees itself with hipHostFree.
// ``coherent``: fine-grained (device writes are visible to the host without a kernel-boundary flush; the round
// signal word).
torch::Tensor host_alloc(int64_t nbytes, bool coherent) {
  if (nbytes <= 0) throw std::invalid_argument("host_alloc: size");
  void* p = nullptr;
  const unsigned flags = hipHostMallocMapped | hipHostMallocPortable | (coherent ? hipHostMallocCoherent : 0u);
  if (hipHostMalloc(&p, (size_t)nbytes, flags) != hipSuccess || !p)
    throw std::runtime_error("host_alloc: hipHostMalloc failed");
  return torch::from_blob(p, {nbytes}, [](void* q) { (void)hipHostFree(q); },
                          torch::TensorOptions().dtype(torch::kUInt8).device(torch::kCPU));
}

// dst (device, uint8) <- src (host_alloc memory, uint8) by a copy kernel that reads the host memory directly.
// Optional round signal (ctr: device int64 [2] = round counter + block arrival count, zero-initialised; flag: coherent
// host_alloc memory holding one int64): the kernel's last block bumps ctr[0] and publishes it to flag.
void host_upload(torch::Tensor src, torch::Tensor dst, c10::optional<torch::Tensor> ctr,
                 c10::optional<torch::Tensor> flag) {
  if (src.device().is_cuda()) throw std::invalid_argument("host_upload: src must be host memory from host_alloc");
  if (!dst.device().is_cuda()) throw std::invalid_argument("host_upload: dst must be a device tensor");
  if (src.scalar_type() != torch::kUInt8 || dst.scalar_type() != torch::kUInt8 || !src.is_contiguous() ||
      !dst.is_contiguous())
    throw std::invalid_argument("host_upload: contiguous uint8 tensors expected");
  const int64_t n = src.numel();
  if (dst.numel() < n || n % 16) throw std::invalid_argument("host_upload: size (16-byte multiple, dst >= src)");
  long long* cp = nullptr;
  long long* fp = nullptr;
  if (ctr && ctr->defined()) {
    need(*ctr, torch::kInt64, "ctr");
    if (ctr->numel() < 2) throw std::invalid_argument("host_upload: ctr needs 2 int64 words (count, arrivals)");
    if (!flag || flag->device().is_cuda() || flag->numel() < 8 || flag->scalar_type() != torch::kUInt8)
      throw std::invalid_argument("host_upload: flag must be >= 8 bytes of host_alloc memory");
    cp = ptr<long long>(*ctr);
    fp = (long long*)flag->data_ptr();
  }
  check(qfx_launch_host_upload(src.data_ptr(), dst.data_ptr(), (long)n, cp, fp, cur_stream()), "qfx_host_upload");
}

// f0 [K,B,C], fpi [K,P,B,C] (empty: no mean term), jac [K,B,C,P], w [K,B,C], keys [K,2] int64 (shots > 0) -> out [K,P]
void ps_combine(torch::Tensor f0, torch::Tensor fpi, torch::Tensor jac, torch::Tensor w, torch::Tensor keys,
                double p01, double p10, int64_t shots, int64_t stream, int64_t noisy, torch::Tensor out) {
  need(jac, torch::kFloat32, "jac");
  need(w, torch::kFloat32, "w");
  need(out, torch::kFloat32, "out");
  const int64_t K = out.size(0), P = out.size(1);
  const int64_t B = w.size(1), C = w.size(2);
  if (w.dim() != 3 || w.size(0) != K || jac.numel() != K * B * C * P)
    throw std::invalid_argument("ps_combine: w [K,B,C] / jac [K,B,C,P] shapes");
  if (fpi.numel()) {
    need(f0, torch::kFloat32, "f0");
    need(fpi, torch::kFloat32, "fpi");
    if (f0.numel() != K * B * C || fpi.numel() != K * P * B * C) throw std::invalid_argument("ps_combine: f0 / fpi");
  }
  if (noisy && shots > 0) {
    need(keys, torch::kInt64, "keys");
    if (keys.numel() < 2 * K) throw std::invalid_argument("ps_combine: keys [K, 2]");
  }
  check(qfx_launch_ps_combine(fpi.numel() ? ptr<float>(f0) : nullptr, ptr<float>(fpi), ptr<float>(jac), ptr<float>(w),
                              (noisy && shots > 0) ? ptr<long long>(keys) : nullptr, (float)p01, (float)p10,
                              (int)shots, (unsigned)stream, (int)K, (int)P, (int)B, (int)C, (int)noisy,
                              ptr<float>(out), cur_stream()),
        "qfx_ps_combine");
}

void round_init(torch::Tensor theta, torch::Tensor params, c10::optional<torch::Tensor> m,
                c10::optional<torch::Tensor> v, c10::optional<torch::Tensor> t) {
  need(theta, torch::kFloat32, "theta");
  need(params, torch::kFloat32, "params");
  const int64_t K = params.size(0), P = params.size(1);
  if (theta.numel() != P) throw std::invalid_argument("round_init: theta size != params row");
  torch::Tensor mt = m ? *m : torch::Tensor(), vt = v ? *v : torch::Tensor(), tt = t ? *t : torch::Tensor();
  for (auto* x : {&mt, &vt})
    if (x->defined()) {
      need(*x, torch::kFloat32, "round_init state");
      if (x->numel() != K * P) throw std::invalid_argument("round_init: state shape");
    }
  if (tt.defined()) need(tt, torch::kFloat32, "round_init t");
  check(qfx_launch_round_init(ptr<float>(theta), (int)K, (int)P, ptr<float>(params), ptr<float>(mt), ptr<float>(vt),
                              ptr<float>(tt), tt.defined() ? (int)tt.numel() : 0, cur_stream()),
        "qfx_round_init");
}

// X [Nc, nmax, F] fp32, Y [Nc, nmax] int64, lid [K] int64, idx [K, B] int64 (rows < nmax, checked by the
// planner on the host) -> x_out rows of stride x_stride (first F columns), y_out [K*B]
void batch_gather(torch::Tensor X, torch::Tensor Y, torch::Tensor lid, torch::Tensor idx, int64_t mode, double alpha,
                  torch::Tensor x_out, torch::Tensor y_out) {
  need(X, torch::kFloat32, "X");
  need(Y, torch::kInt64, "Y");
  need(lid, torch::kInt64, "lid");
  need(idx, torch::kInt64, "idx");
  need(x_out, torch::kFloat32, "x_out");
  need(y_out, torch::kInt64, "y_out");
  if (X.dim() != 3 || Y.dim() != 2 || idx.dim() != 2 || Y.size(1) != X.size(1))
    throw std::invalid_argument("batch_gather: shapes");
  const int64_t K = idx.size(0), B = idx.size(1), F = X.size(2);
  if (lid.numel() != K || x_out.dim() != 3 || x_out.size(0) != K || x_out.size(1) != B || x_out.size(2) < F ||
      !x_out.is_contiguous() || y_out.numel() < K * B || mode < 0 || mode > 2)
    throw std::invalid_argument("batch_gather: output shapes / mode");
  check(qfx_launch_batch_gather(ptr<float>(X), ptr<long long>(Y), ptr<long long>(lid), ptr<long long>(idx), (int)K,
                                (int)B, (long)X.size(1), (int)F, (int)mode, (float)alpha, ptr<float>(x_out),
                                (int)x_out.size(2), ptr<long long>(y_out), cur_stream()),
        "qfx_batch_gather");
}

// round_init + the minibatch gather of every local step in one launch: idx [steps, K, B] int64,
// x_out [steps, K, B, >= F] fp32, y_out [steps * K * B] int64 (same checks as round_init / batch_gather)
void round_prologue(torch::Tensor theta, torch::Tensor params, c10::optional<torch::Tensor> m,
                    c10::optional<torch::Tensor> v, c10::optional<torch::Tensor> t, torch::Tensor X, torch::Tensor Y,
                    torch::Tensor lid, torch::Tensor idx, int64_t mode, double alpha, torch::Tensor x_out,
                    torch::Tensor y_out, bool rows, c10::optional<std::vector<torch::Tensor>> frag_job, bool frag_bf16,
                    c10::optional<torch::Tensor> zero, c10::optional<std::vector<torch::Tensor>> upload) {
  need(theta, torch::kFloat32, "theta");
  need(params, torch::kFloat32, "params");
  const int64_t K = params.size(0), P = params.size(1);
  if (theta.numel() != P) throw std::invalid_argument("round_prologue: theta size != params row");
  torch::Tensor mt = m ? *m : torch::Tensor(), vt = v ? *v : torch::Tensor(), tt = t ? *t : torch::Tensor();
  for (auto* x : {&mt, &vt})
    if (x->defined()) {
      need(*x, torch::kFloat32, "round_prologue state");
      if (x->numel() != K * P) throw std::invalid_argument("round_prologue: state shape");
    }
  if (tt.defined()) need(tt, torch::kFloat32, "round_prologue t");
  need(X, torch::kFloat32, "X");
  need(Y, torch::kInt64, "Y");
  need(lid, torch::kInt64, "lid");
  need(idx, torch::kInt64, "idx");
  need(x_out, torch::kFloat32, "x_out");
  need(y_out, torch::kInt64, "y_out");
  if (X.dim() != 3 || Y.dim() != 2 || idx.dim() != 3 || Y.size(1) != X.size(1))
    throw std::invalid_argument("round_prologue: shapes");
  const int64_t S = idx.size(0), B = idx.size(2), F = X.size(2);
  if (idx.size(1) != K || lid.numel() != K || x_out.dim() != 4 || x_out.size(0) != S || x_out.size(1) != K ||
      x_out.size(2) != B || x_out.size(3) < F || y_out.numel() < S * K * B || mode < 0 || mode > 2)
    throw std::invalid_argument("round_prologue: output shapes / mode");
  // frag_job = (slot_tab int32 [n_slots, 9], frags int32 [n_slots * 4 * 128 * 4]): the MFMA engine's shared
  // fragments of the round's first step, built from theta by extra blocks of the same launch
  const int* slot_tab = nullptr;
  void* frags = nullptr;
  int n_slots = 0;
  if (frag_job && !frag_job->empty()) {
    if (frag_job->size() != 2) throw std::invalid_argument("round_prologue: frag_job = (slot_tab, frags)");
    const torch::Tensor& stab = (*frag_job)[0];
    const torch::Tensor& fr = (*frag_job)[1];
    need(stab, torch::kInt32, "slot_tab");
    need(fr, torch::kInt32, "frags");
    if (stab.dim() != 2 || stab.size(1) != 9) throw std::invalid_argument("round_prologue: slot_tab [n_slots, 9]");
    n_slots = (int)stab.size(0);
    if (fr.numel() < (int64_t)n_slots * 4 * 128 * 4) throw std::invalid_argument("round_prologue: frags too small");
    slot_tab = stab.data_ptr<int>();
    frags = fr.data_ptr();
  }
  // zero: int64 entries the prologue zeroes (the all-reduce buffer head the MFMA engine's FedAvg tail adds into)
  long long* zp = nullptr;
  int64_t nz = 0;
  if (zero && zero->defined() && zero->numel() > 0) {
    need(*zero, torch::kInt64, "zero");
    zp = reinterpret_cast<long long*>(zero->data_ptr<int64_t>());
    nz = zero->numel();
  }
  // upload = (src host_alloc uint8, dst device uint8, ctr int64 [2], flag host_alloc >= 8 bytes): the round's
  // host_upload folded into this launch (lid and idx must be views of dst; the launcher checks)
  const void* uh = nullptr;
  void* ud = nullptr;
  long un = 0;
  long long *uc = nullptr, *uf = nullptr;
  if (upload && !upload->empty()) {
    if (upload->size() != 4) throw std::invalid_argument("round_prologue: upload = (src, dst, ctr, flag)");
    const torch::Tensor &src = (*upload)[0], &dst = (*upload)[1], &ctr = (*upload)[2], &flag = (*upload)[3];
    if (src.device().is_cuda() || !dst.device().is_cuda() || src.scalar_type() != torch::kUInt8 ||
        dst.scalar_type() != torch::kUInt8 || !src.is_contiguous() || !dst.is_contiguous() ||
        dst.numel() < src.numel() || src.numel() % 16)
      throw std::invalid_argument("round_prologue: upload src (host_alloc) / dst (device) uint8, 16-byte multiple");
    need(ctr, torch::kInt64, "upload ctr");
    if (ctr.numel() < 2 || flag.device().is_cuda() || flag.numel() < 8 || flag.scalar_type() != torch::kUInt8)
      throw std::invalid_argument("round_prologue: upload ctr [2] int64 / flag >= 8 bytes host_alloc");
    uh = src.data_ptr();
    ud = dst.data_ptr();
    un = (long)src.numel();
    uc = ptr<long long>(ctr);
    uf = (long long*)flag.data_ptr();
  }
  // rows = false: params only gives the [K, P] shape (the first local step reads theta; CFed fused SGD)
  check(qfx_launch_round_prologue(ptr<float>(theta), (int)K, (int)P, rows ? ptr<float>(params) : nullptr, ptr<float>(mt),
                                  ptr<float>(vt),
                                  ptr<float>(tt), tt.defined() ? (int)tt.numel() : 0, ptr<float>(X),
                                  ptr<long long>(Y), ptr<long long>(lid), ptr<long long>(idx), (int)S, (int)B,
                                  (long)X.size(1), (int)F, (int)mode, (float)alpha, ptr<float>(x_out),
                                  (int)x_out.size(3), ptr<long long>(y_out), slot_tab, n_slots, frags,
                                  frag_bf16 ? 1 : 0, zp, (int)nz, uh, ud, un, uc, uf, cur_stream()),
        "qfx_round_prologue");
}

// pack_buf (optional, the round's [P + 6] all-reduce buffer): one more block of the same launch packs the round
// metrics (loss, correct, nvalid, act: float32 [n]) into its tail, as round_pack does.  sat: int64 [1] counter
// of saturated fixed-point terms (with pack_buf, it must be pack_buf[P + 5])
void fedavg(torch::Tensor theta_k, torch::Tensor theta_g, torch::Tensor angle_mask, torch::Tensor weights,
            torch::Tensor norms, torch::Tensor keys, bool wrap, bool dp, double clip, double sigma,
            torch::Tensor out, torch::Tensor pack_buf, torch::Tensor loss, torch::Tensor correct,
            torch::Tensor nvalid, torch::Tensor act, torch::Tensor sat, c10::optional<torch::Tensor> sa_seeds,
            c10::optional<torch::Tensor> sa_sign, c10::optional<torch::Tensor> sa_round, double sa_scale,
            int64_t sa_bits, c10::optional<torch::Tensor> sa_masks, c10::optional<torch::Tensor> norm_cid,
            c10::optional<torch::Tensor> fa_theta, c10::optional<torch::Tensor> fa_out,
            c10::optional<torch::Tensor> fa_cnt, int64_t fa_bits, double fa_scale, int64_t fa_n_norms,
            c10::optional<torch::Tensor> dp_scale, bool sa_pairsym) {
  need(theta_k, torch::kFloat32, "theta_k");
  need(sat, torch::kInt64, "sat");
  if (sat.numel() < 1) throw std::invalid_argument("fedavg: sat counter missing");
  need(theta_g, torch::kFloat32, "theta_g");
  need(weights, torch::kFloat64, "weights");
  need(norms, torch::kFloat64, "norms");
  need(out, torch::kInt64, "out");
  const int K = (int)theta_k.size(0), P = (int)theta_k.size(1);
  if (out.numel() < P + 1) throw std::invalid_argument("fedavg out too small");
  if (norms.numel() < qfx_fedavg_norm_scratch(K, P)) throw std::invalid_argument("fedavg norms scratch too small");
  if (dp && keys.numel() < 2 * K) throw std::invalid_argument("fedavg: DP needs 2 key words per client");
  const bool pack = pack_buf.defined() && pack_buf.numel() > 0;
  int64_t n = 0;
  if (pack) {
    need(pack_buf, torch::kInt64, "pack_buf");
    for (auto* x : {&loss, &correct, &nvalid, &act}) need(*x, torch::kFloat32, "fedavg metric");
    n = loss.numel();
    if (pack_buf.numel() < P + 6 || correct.numel() < n || nvalid.numel() < n || act.numel() < n)
      throw std::invalid_argument("fedavg: metric pack sizes");
    if (out.data_ptr() != pack_buf.data_ptr()) throw std::invalid_argument("fedavg: out must be the head of pack_buf");
    if (sat.data_ptr() != (void*)(ptr<long long>(pack_buf) + P + 5))
      throw std::invalid_argument("fedavg: sat must be pack_buf[P + 5]");
  }
  // SecAgg: pair-seed key words [K, N, 2] int32, signs [K, N] int32, round [1] int32 (all device tensors)
  const bool sa = sa_seeds.has_value() && sa_seeds->defined();
  int sa_n = 0;
  if (sa) {
    if (!sa_sign.has_value() || !sa_round.has_value()) throw std::invalid_argument("fedavg: SecAgg needs seeds, signs, round");
    need(*sa_seeds, torch::kInt32, "sa_seeds");
    need(*sa_sign, torch::kInt32, "sa_sign");
    need(*sa_round, torch::kInt32, "sa_round");
    if (sa_sign->dim() != 2 || sa_sign->size(0) < K) throw std::invalid_argument("fedavg: sa_sign must be [K, N]");
    sa_n = (int)sa_sign->size(1);
    if (sa_seeds->numel() < (int64_t)K * sa_n * 2 || sa_round->numel() < 1)
      throw std::invalid_argument("fedavg: SecAgg table sizes");
    if (sa_bits < 2 || sa_bits > 62 || !(sa_scale > 0)) throw std::invalid_argument("fedavg: SecAgg bits / scale");
    // pair-symmetric mask generation: the caller vouches that row k is client k and every client is a row
    if (sa_pairsym && (sa_n != K || K > 128 || sa_sign->size(0) != K))
      throw std::invalid_argument("fedavg: pair-symmetric SecAgg masks need a square [K, K] table, K <= 128");
    if (!sa_masks.has_value()) throw std::invalid_argument("fedavg: SecAgg needs a [K, P + 1] mask workspace");
    need(*sa_masks, torch::kInt64, "sa_masks");
    if (sa_masks->numel() < (int64_t)K * (P + 1)) throw std::invalid_argument("fedavg: SecAgg mask workspace size");
  }
  // CC6: global client ids [K] int32 of the rows; the pack block scatters the DP norms into buf[P + 6 + cid]
  const bool nc = norm_cid.has_value() && norm_cid->defined() && norm_cid->numel() > 0;
  if (nc) {
    need(*norm_cid, torch::kInt32, "norm_cid");
    if (!pack || !dp || norm_cid->numel() < K) throw std::invalid_argument("fedavg: norm slots need pack + DP + [K] ids");
  }
  // distributed DP: per-client noise scale [K] float32 (the round's 1 / sqrt(live participants))
  const bool ds = dp_scale.has_value() && dp_scale->defined() && dp_scale->numel() > 0;
  if (ds) {
    need(*dp_scale, torch::kFloat32, "dp_scale");
    if (!dp || dp_scale->numel() < K) throw std::invalid_argument("fedavg: dp_scale needs DP and [K] entries");
  }
  // single-rank round: the launch's last block also applies the round (round_apply's work) to fa_theta [P], writing
  // the [6 + n_norms] outputs to fa_out; fa_cnt is an int32 [1] zeroed arrival counter (self-resetting)
  const bool fa = fa_theta.has_value() && fa_theta->defined();
  if (fa) {
    if (!pack || !fa_out.has_value() || !fa_cnt.has_value()) throw std::invalid_argument("fedavg: fused apply needs pack, out, counter");
    need(*fa_theta, torch::kFloat32, "fa_theta");
    need(*fa_out, torch::kFloat64, "fa_out");
    need(*fa_cnt, torch::kInt32, "fa_cnt");
    if (fa_theta->numel() != P || fa_out->numel() < 6 + fa_n_norms || fa_cnt->numel() < 1 || fa_n_norms < 0 ||
        pack_buf.numel() < P + 6 + fa_n_norms || fa_bits < 0 || fa_bits > 62)
      throw std::invalid_argument("fedavg: fused apply sizes");
  }
  check(qfx_launch_fedavg(ptr<float>(theta_k), ptr<float>(theta_g), ptr<unsigned char>(angle_mask),
                          ptr<double>(weights), ptr<double>(norms), ptr<uint32_t>(keys), K, P, wrap ? 1 : 0,
                          dp ? 1 : 0, (float)clip, (float)sigma, ptr<long long>(out),
                          pack ? ptr<long long>(pack_buf) : nullptr, pack ? ptr<float>(loss) : nullptr,
                          pack ? ptr<float>(correct) : nullptr, pack ? ptr<float>(nvalid) : nullptr,
                          pack ? ptr<float>(act) : nullptr, (int)n, ptr<long long>(sat),
                          sa ? ptr<uint32_t>(*sa_seeds) : nullptr, sa ? ptr<int>(*sa_sign) : nullptr,
                          sa ? ptr<int>(*sa_round) : nullptr, sa_n, sa_scale, (int)sa_bits,
                          sa ? ptr<long long>(*sa_masks) : nullptr, nc ? ptr<int>(*norm_cid) : nullptr,
                          fa ? ptr<float>(*fa_theta) : nullptr, fa ? ptr<double>(*fa_out) : nullptr,
                          fa ? ptr<unsigned>(*fa_cnt) : nullptr, (int)fa_bits, fa_scale, (int)fa_n_norms,
                          ds ? ptr<float>(*dp_scale) : nullptr, sa_pairsym ? 1 : 0, cur_stream()),
        "qfx_fedavg");
}

std::vector<int> blob_vec(const torch::Tensor& blob) {
  auto b = blob.to(torch::kInt32).contiguous().cpu();
  return std::vector<int>(b.data_ptr<int>(), b.data_ptr<int>() + b.numel());
}

py::tuple jit_prepare(torch::Tensor blob, int64_t p, bool adjoint, std::string cache_dir, std::string include_dir,
                      std::string arch, bool bf16) {
  std::string key;
  int h = qfx::jit_prepare(blob_vec(blob), (int)p, adjoint, cache_dir, include_dir, arch, &key, bf16);
  return py::make_tuple(h, key);
}

std::string jit_source(torch::Tensor blob, int64_t p, bool adjoint, bool bf16) {
  return qfx::jit_source(blob_vec(blob), (int)p, adjoint, bf16);
}

void jit_launch(int64_t handle, torch::Tensor blob, int64_t pass_off, torch::Tensor psi, c10::optional<torch::Tensor> lam,
                torch::Tensor params, int64_t spc, torch::Tensor xang, c10::optional<torch::Tensor> w_read,
                c10::optional<torch::Tensor> out_read, c10::optional<torch::Tensor> gslab, int64_t n_samples,
                int64_t n_grad) {
  need(blob, torch::kInt32, "blob");
  bool bf16 = false;
  const long sbytes = qfx::jit_state_bytes((int)handle, &bf16);
  if (sbytes < 0) throw std::invalid_argument("jit_launch: bad kernel handle");
  need(psi, bf16 ? torch::kInt32 : torch::kComplexFloat, "psi (int32 = packed bf16x2 state)");
  // the kernel indexes [n_samples, 2^n] amplitudes: refuse buffers that would be overrun
  if ((long)(psi.numel() * psi.element_size()) < sbytes * n_samples) throw std::invalid_argument("psi too small");
  if (lam.has_value() && (long)(lam->numel() * lam->element_size()) < sbytes * n_samples)
    throw std::invalid_argument("lam too small");
  need(params, torch::kFloat32, "params");
  need(xang, torch::kFloat32, "xang");
  if (xang.size(0) < n_samples) throw std::invalid_argument("xang rows < n_samples");
  if (params.size(0) * spc < n_samples) throw std::invalid_argument("params rows * spc < n_samples");
  torch::Tensor lt = lam.has_value() ? *lam : torch::Tensor();
  torch::Tensor wt = w_read.has_value() ? *w_read : torch::Tensor();
  torch::Tensor ot = out_read.has_value() ? *out_read : torch::Tensor();
  torch::Tensor gs = gslab.has_value() ? *gslab : torch::Tensor();
  qfx::PassArgsHost a{ptr<int>(blob), (int)pass_off, psi.data_ptr(), lt.defined() ? lt.data_ptr() : nullptr,
                      ptr<float>(params), (int)params.size(1), (int)spc, ptr<float>(xang), (int)xang.size(1),
                      ptr<float>(wt), ptr<float>(ot), ptr<float>(gs), (int)n_samples, (int)n_grad};
  check(qfx::jit_launch((int)handle, a, cur_stream()), "qfx_jit_launch");
}

}  // namespace

void register_cnn(pybind11::module& m);

extern "C" {
int qfx_dm_gate_bytes();
int qfx_dm_run(const void* gates, int G, int n, const float* rows, int W, long S, const int* readout, int C,
               const float* superop, void* scratch, float* expz, hipStream_t st);
int qfx_dm_lds_qubits();
}

// Exact density-matrix run (density.hip): gates = lowered program bytes (ops/density.py), rows [S, W] slot values,
// superop [32] float (4 x 4 complex noise channel) or empty, scratch [S, 4^n] complex64 (n > LDS qubits), expz [S, C]
void dm_run(torch::Tensor gates, int64_t G, int64_t n, torch::Tensor rows, torch::Tensor readout, torch::Tensor superop,
            torch::Tensor scratch, torch::Tensor expz) {
  need(gates, torch::kInt32, "gates");
  need(rows, torch::kFloat32, "rows");
  need(readout, torch::kInt32, "readout");
  need(expz, torch::kFloat32, "expz");
  if (gates.numel() * 4 < G * qfx_dm_gate_bytes()) throw std::invalid_argument("dm_run: gate table too small");
  if (rows.dim() != 2) throw std::invalid_argument("dm_run: rows must be [S, W]");
  const int64_t S = rows.size(0), C = readout.numel();
  if (expz.numel() < S * C) throw std::invalid_argument("dm_run: expz too small");
  const bool noisy = superop.defined() && superop.numel() > 0;
  if (noisy) {
    need(superop, torch::kFloat32, "superop");
    if (superop.numel() != 32) throw std::invalid_argument("dm_run: superop must be 4 x 4 complex");
  }
  const bool global = n > qfx_dm_lds_qubits();
  if (global) {
    need(scratch, torch::kComplexFloat, "scratch");
    if (scratch.numel() < S * (int64_t(1) << (2 * n))) throw std::invalid_argument("dm_run: scratch too small");
  }
  check(qfx_dm_run(gates.data_ptr(), (int)G, (int)n, ptr<float>(rows), (int)rows.size(1), (long)S, ptr<int>(readout),
                   (int)C, noisy ? ptr<float>(superop) : nullptr, global ? scratch.data_ptr() : nullptr,
                   ptr<float>(expz), cur_stream()),
        "qfx_dm_run");
}
void register_hea(pybind11::module& m);
void register_mps(pybind11::module& m);

PYBIND11_MODULE(TORCH_EXTENSION_NAME, m) {
  m.doc() = "qfedx_amd native runtime: pass planner + gfx950 HIP kernels";
  m.def("plan", &plan, "plan circuit passes");
  m.def("pass_launch", &pass_launch);
  m.def("readout_ce", &readout_ce);
  m.def("readout_sum", &readout_sum);
  m.def("amp_init", &amp_init);
  m.def("round_init", &round_init);
  m.def("host_alloc", &host_alloc, py::arg("nbytes"), py::arg("coherent") = false);
  m.def("ps_combine", &ps_combine);
  m.def("host_upload", &host_upload, py::arg("src"), py::arg("dst"), py::arg("ctr") = py::none(),
        py::arg("flag") = py::none());
  m.def("batch_plan", &qfx_runtime::batch_plan);
  m.def("batch_gather", &batch_gather);
  m.def("round_prologue", &round_prologue, pybind11::arg("theta"), pybind11::arg("params"), pybind11::arg("m"),
        pybind11::arg("v"), pybind11::arg("t"), pybind11::arg("X"), pybind11::arg("Y"), pybind11::arg("lid"),
        pybind11::arg("idx"), pybind11::arg("mode"), pybind11::arg("alpha"), pybind11::arg("x_out"),
        pybind11::arg("y_out"), pybind11::arg("rows") = true, pybind11::arg("frag_job") = pybind11::none(),
        pybind11::arg("frag_bf16") = false, pybind11::arg("zero") = pybind11::none(),
        pybind11::arg("upload") = pybind11::none());
  m.def("amp_scratch", &amp_scratch);
  m.def("readout_noise", &readout_noise);
  m.def("philox_uniform", &philox_uniform);
  m.def("grad_reduce", &grad_reduce);
  m.def("grad_split", &grad_split);
  m.def("round_pack", &round_pack);
  m.def("fedavg_norm_scratch", [](int64_t K, int64_t P) { return qfx_fedavg_norm_scratch((int)K, (int)P); });
  m.def("round_apply", &round_apply);
  m.def("adam", &adam);
  m.def("sgdm", &sgdm);
  m.def("fedavg", &fedavg);
  m.def("prologue_gather_lanes", [](int64_t F) { return qfx_prologue_gather_lanes((int)F); });
  m.def("jit_prepare", &jit_prepare, "generate + hiprtc-compile (or load cached) a circuit-specialised pass kernel",
        py::arg("blob"), py::arg("p"), py::arg("adjoint"), py::arg("cache_dir"), py::arg("include_dir"),
        py::arg("arch"), py::arg("bf16") = false);
  m.def("jit_source", &jit_source, py::arg("blob"), py::arg("p"), py::arg("adjoint"), py::arg("bf16") = false);
  m.def("jit_launch", &jit_launch);
  register_cnn(m);
  m.def("dm_run", &dm_run, "exact density-matrix simulation of a lowered noisy program (one workgroup per row)");
  m.def("dm_gate_bytes", []() { return qfx_dm_gate_bytes(); });
  m.def("dm_lds_qubits", []() { return qfx_dm_lds_qubits(); });
  register_hea(m);
  register_mps(m);
}
