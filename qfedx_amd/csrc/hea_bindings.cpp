// Bindings of the MFMA statevector engine (hea_mfma.hip).  Every launch goes on torch's current HIP
// stream (composes with hipGraph capture).  Buffer extents are checked here against the geometry the
// kernel will index with, so a bad plan or a short buffer is a Python exception, never a GPU fault.
#include <c10/hip/HIPStream.h>
#include <torch/extension.h>

#include <algorithm>
#include <cstdint>
#include <cstdlib>
#include <stdexcept>
#include <string>
#include <vector>

#include "hea_args.h"

extern "C" {
int qfx_hea_pass(int adjoint, const HeaPassArgs* args, int n_samples, hipStream_t st);
int qfx_hea_frags(const float* params, int p_stride, const int* slot_tab, int n_slots, int K, void* frags,
                  hipStream_t st);
int qfx_hea_grad_reduce(const long long* gslab, int slab_tiles, int n_gradops, const int* gmeta, int spc, int K,
                        float* params, float* grad, int p_stride, const QfxAdamArgs* adam,
                        const QfxReadoutRed* readout, const QfxFedTail* fed, hipStream_t st);
int qfx_hea_args_size();
int qfx_hea_check_status(hipStream_t st);
// bf16 state storage (hea_mfma_bf16.hip)
int qfx_hea_pass_bf16(int adjoint, const HeaPassArgs* args, int n_samples, hipStream_t st);
int qfx_hea_frags_bf16(const float* params, int p_stride, const int* slot_tab, int n_slots, int K, void* frags,
                       hipStream_t st);
int qfx_hea_check_status_bf16(hipStream_t st);
}

namespace {

hipStream_t cur() { return c10::hip::getCurrentHIPStream().stream(); }

void need(bool ok, const std::string& msg) {
  if (!ok) throw std::invalid_argument("hea: " + msg);
}

template <typename T>
T* dp(const torch::Tensor& t, torch::ScalarType dt, const char* name, int64_t min_numel) {
  if (min_numel == 0 && (!t.defined() || t.numel() == 0)) return nullptr;
  need(t.defined() && t.is_cuda() && t.is_contiguous() && t.scalar_type() == dt, std::string(name) +
       ": expected a contiguous CUDA tensor of the right dtype");
  need(t.numel() >= min_numel, std::string(name) + ": buffer too small (" + std::to_string(t.numel()) + " < " +
       std::to_string(min_numel) + ")");
  return reinterpret_cast<T*>(t.data_ptr());
}

void check(int rc, const char* what) {
  if (rc != 0) throw std::runtime_error(std::string(what) + " failed: " + std::to_string(rc));
#if defined(QFX_DEVICE_CHECKS) && QFX_DEVICE_CHECKS
  // debug build: every launch is followed by a read of the device-check status word
  int line = qfx_hea_check_status(cur());
  if (line == 0) line = qfx_hea_check_status_bf16(cur());
  if (line != 0)
    throw std::runtime_error(std::string(what) + ": device check failed at hea_mfma.hip:" + std::to_string(line));
#endif
}

// geom = [n, t, c, lo, hi, n_tiles, gen, load_lam, store_psi, store_lam, spc, C, n_theta, p_stride, feature,
//         S, x_stride, n_slots, slab_tiles, K, H0..H4 (LDS swizzle rows), n_gradops, in_rep, bf16, n_regions,
//         frag_shared, nt_store]
// bf16: states and fragments in bf16 (hea_mfma_bf16.hip) instead of fp16.  dbg: the stall-attribution buffer of the
// stamps build (int64 [HEA_STAMP_ROWS * 16]; empty otherwise)
void hea_pass(bool adjoint, torch::Tensor ops, torch::Tensor fidx, torch::Tensor fo, std::vector<int64_t> geom, double scale,
              torch::Tensor psi_in,
              torch::Tensor psi_out, torch::Tensor lam_in, torch::Tensor lam_out, torch::Tensor xang,
              torch::Tensor params, torch::Tensor frags, torch::Tensor wread, torch::Tensor part,
              torch::Tensor gslab, torch::Tensor dbg, c10::optional<std::vector<torch::Tensor>> readout,
              int64_t ro_tps) {
  need(geom.size() == 31, "geometry vector must have 31 entries");
  const bool bf16 = geom[27] != 0;
  HeaPassArgs a{};
  a.n = (int)geom[0];
  a.t = (int)geom[1];
  a.c = (int)geom[2];
  a.lo = (int)geom[3];
  a.hi = (int)geom[4];
  a.n_tiles = (int)geom[5];
  a.gen = (int)geom[6];
  a.load_lam = (int)geom[7];
  a.store_psi = (int)geom[8];
  a.store_lam = (int)geom[9];
  a.spc = (int)geom[10];
  a.C = (int)geom[11];
  a.n_theta = (int)geom[12];
  a.p_stride = (int)geom[13];
  a.feature = (int)geom[14];
  const int64_t S = geom[15];
  a.x_stride = (int)geom[16];
  a.n_slots = (int)geom[17];
  a.slab_tiles = (int)geom[18];
  const int64_t K = geom[19];
  a.n_gradops = (int)geom[25];
  a.in_rep = (int)geom[26];
  a.n_regions = (int)geom[28];
  a.frag_shared = geom[29] != 0 ? 1 : 0;
  a.nt_store = geom[30] != 0 ? 1 : 0;
  need(a.n_regions >= 0 && a.n_regions <= 2 * 32, "gradient regions per pass out of range");
  a.scale = (float)scale;
  a.dbg = dbg.defined() && dbg.numel() > 0 ? dp<long long>(dbg, torch::kInt64, "dbg", (int64_t)HEA_STAMP_ROWS * 16)
                                           : nullptr;
  for (int b = 0; b < 5; ++b) {
    a.hrow[b] = (int)geom[20 + b];
    need(a.hrow[b] >= 0 && a.hrow[b] < (1 << (a.t - 5)), "swizzle row reads past the tile bits");
  }
  need(a.n >= 8 && a.n <= 30 && a.t >= 8 && a.t <= 14 && a.t <= a.n, "qubit / tile size out of range");
  need(a.c >= 2 && a.c <= a.lo && a.lo <= a.hi && a.hi <= a.n && a.c + a.hi - a.lo == a.t, "bad tile layout");
  need(a.n_tiles == (1 << (a.n - a.t)), "n_tiles must be 2^(n - t)");
  need(a.spc > 0 && S == K * a.spc, "samples must be K x spc");
  need(a.C >= 1 && a.C <= 8, "1..8 readout classes");
  need(a.n_theta >= 2 * a.n, "theta count below one layer");
  need(a.p_stride >= a.n_theta, "param stride too small");
  need(ops.dim() == 2 && ops.size(1) == 128 && ops.scalar_type() == torch::kInt32 && ops.is_cuda(),
       "ops must be int32 [nops, 128] on the device");
  a.nops = (int)ops.size(0);
  need(a.nops <= 32, "at most 32 ops per pass program");
  a.ops = dp<int>(ops, torch::kInt32, "ops", 0);
  a.fidx = a.nops ? dp<int>(fidx, torch::kInt32, "fidx", 2 * a.nops) : nullptr;
  a.fo_tab = a.nops ? reinterpret_cast<const uint32_t*>(dp<int>(fo, torch::kInt32, "fo", (int64_t)a.n_tiles * a.nops)) : nullptr;
  need(a.in_rep >= 1 && (!adjoint || a.in_rep == 1) && K % a.in_rep == 0,
       "in_rep: forward only, parameter rows a multiple of it");
  const int64_t states = S << a.n;
  a.psi_in = a.gen ? nullptr : dp<uint32_t>(psi_in, torch::kInt32, "psi_in", states / a.in_rep);
  need(!(adjoint && a.store_psi), "adjoint passes store lambda only");
  a.psi_out = a.store_psi ? dp<uint32_t>(psi_out, torch::kInt32, "psi_out", states) : nullptr;
  a.lam_in = (adjoint && a.load_lam) ? dp<uint32_t>(lam_in, torch::kInt32, "lam_in", states) : nullptr;
  a.lam_out = (adjoint && a.store_lam) ? dp<uint32_t>(lam_out, torch::kInt32, "lam_out", states) : nullptr;
  need(a.x_stride >= a.n, "x stride must cover n feature angles");
  // layer-1 factors: the product-state generation (forward gen passes)
  a.xang = a.gen ? dp<float>(xang, torch::kFloat32, "xang", S / a.in_rep * a.x_stride) : nullptr;
  a.params = dp<float>(params, torch::kFloat32, "params", K * a.p_stride);
  a.frags = a.n_slots ? (const void*)dp<int32_t>(frags, torch::kInt32, "frags",
                                                  (a.frag_shared ? 1 : K) * a.n_slots * 4 * 128 * 4)
                      : nullptr;
  a.part = dp<float>(part, torch::kFloat32, "part", 0);
  if (readout && !readout->empty()) {
    // fused readout (first adjoint pass): readout = (y int64 [S], wts [S], expz [S, C], w_out [S, C],
    // rec [S, 2C + 2]); part holds the readout pass's [S, ro_tps, C] partials
    const auto& r = *readout;
    need(adjoint && !a.load_lam && r.size() == 5 && ro_tps >= 1, "fused readout: first adjoint pass, 5 tensors");
    need(ro_tps * a.C <= 64, "fused readout: at most 64 readout partials per sample (one per lane)");
    need(a.part && part.numel() >= S * ro_tps * a.C, "fused readout: part buffer too small");
    a.ro_fuse = 1;
    a.ro_tps = (int)ro_tps;
    a.ro_y = dp<long long>(r[0], torch::kInt64, "ro_y", S);
    a.ro_wts = dp<float>(r[1], torch::kFloat32, "ro_wts", S);
    a.ro_expz = dp<float>(r[2], torch::kFloat32, "ro_expz", S * a.C);
    a.ro_w = dp<float>(r[3], torch::kFloat32, "ro_w", S * a.C);
    a.ro_rec = dp<float>(r[4], torch::kFloat32, "ro_rec", S * (2 * a.C + 2));
    need(a.n_theta + 2 * a.C <= a.p_stride, "fused readout: readout parameters past the parameter row");
    a.wread = nullptr;
  } else {
    a.wread = adjoint ? dp<float>(wread, torch::kFloat32, "wread", S * a.C) : nullptr;
    if (a.part) need(part.numel() >= S * a.n_tiles * a.C, "part buffer too small");
  }
  a.gslab = adjoint ? dp<long long>(gslab, torch::kInt64, "gslab", S * a.slab_tiles * a.n_gradops * 32) : nullptr;
  need(!adjoint || a.slab_tiles >= a.n_tiles, "gradient slab has fewer tiles than the pass");
  need(!a.gen || a.n <= 32, "product-state generation supports <= 32 qubits");
  if (bf16)
    check(qfx_hea_pass_bf16(adjoint ? 1 : 0, &a, (int)S, cur()), "qfx_hea_pass_bf16");
  else
    check(qfx_hea_pass(adjoint ? 1 : 0, &a, (int)S, cur()), "qfx_hea_pass");
}

// Validate a pass program once (host copy) when it is built: slot / gradient-slot ranges and op kinds.
void hea_check_ops(torch::Tensor ops, torch::Tensor fidx, int64_t n_slots, int64_t n_theta, bool adjoint, int64_t t,
                   int64_t n_gradops) {
  need(fidx.scalar_type() == torch::kInt32 && !fidx.is_cuda() && fidx.is_contiguous() && fidx.numel() == 2 * ops.size(0),
       "fidx must be a host int32 [nops, 2] tensor");
  const int* fi = fidx.data_ptr<int>();
  for (int64_t o = 0; o < 2 * ops.size(0); ++o) need(fi[o] >= -1 && fi[o] < 4 * n_slots, "fragment index out of range");
  need(ops.dim() == 2 && ops.size(1) == 128 && ops.scalar_type() == torch::kInt32 && !ops.is_cuda() &&
       ops.is_contiguous(), "ops must be a contiguous host int32 [nops, 128] tensor");
  const int* ow = ops.data_ptr<int>();
  int ngrad = 0;
  // op codes (hea_plan.py): 1 APPLY, 2 APPLY2, 3 BACK2, 4 GRAD2 (chained pairs), 5 GRAD_L1, 6 OBS, 7 READOUT, 8 BACK
  for (int64_t o = 0; o < ops.size(0); ++o) {
    const int c = ow[o * 128];
    ngrad += (c == 5 || c == 8) ? 1 : (c == 3 || c == 4) ? 2 : 0;
  }
  need(ngrad <= 12, "at most 12 gradient ops per pass program");
  need(ops.size(0) <= 32, "at most 32 ops per pass program");
  for (int64_t o = 0; o < ops.size(0); ++o) {
    const int* w = ow + o * 128;
    const int code = w[0];
    const bool pair = code >= 2 && code <= 4;
    need(code >= 1 && code <= 8, "unknown op code");
    need(adjoint ? (code >= 3 && code <= 6) || code == 8 : (code == 1 || code == 2 || code == 7),
         "op kind not valid in this pass");
    if (code == 1 || code == 2 || code == 3 || code == 8) need(w[1] >= 0 && w[1] < n_slots, "op names a missing unitary slot");
    if (code == 2 || code == 3) need(w[102] >= 0 && w[102] < n_slots, "pair op names a missing unitary slot");
    // fragment indices must be the op's own slots (the kernel DMAs them)
    if (code == 1 || code == 2) need(fi[2 * o] == 4 * w[1], "fragment index / slot mismatch");
    if (code == 3 || code == 8) need(fi[2 * o] == 4 * w[1] + 2, "fragment index / slot mismatch");
    if (code == 2) need(fi[2 * o + 1] == 4 * w[102], "fragment index / slot mismatch");
    if (code == 3) need(fi[2 * o + 1] == 4 * w[102] + 2, "fragment index / slot mismatch");
    if (!pair) need(fi[2 * o + 1] == -1, "a single op has one fragment set");
    if (code != 6 && code != 7) {
      // rotation pairs hold two 4-qubit groups; a layer-1 gradient pair (GRAD2) may have short groups (w[103]: Y's)
      if (pair) need(code == 4 ? (w[2] >= 1 && w[2] <= 4 && w[103] >= 1 && w[103] <= 4) : (w[2] == 4 && w[103] == 4),
                     "pair group sizes out of range");
      else need(w[2] >= 0 && w[2] <= 4, "group size out of range");
      for (int j = 0; j < w[2]; ++j)
        need(w[12 + j] >= 0 && w[12 + j] < n_theta && w[16 + j] >= 0 && w[16 + j] < n_theta,
             "gradient slot out of range");
      if (pair)
        for (int j = 0; j < w[103]; ++j)
          need(w[120 + j] >= 0 && w[120 + j] < n_theta && w[124 + j] >= 0 && w[124 + j] < n_theta,
               "gradient slot out of range");
      for (int i = 20; i < 100; ++i) need(w[i] >= 0 && w[i] < (1 << t), "tile address out of range");
      if (pair)
        for (int i = 104; i < 120; ++i) need(w[i] >= 0 && w[i] < (1 << t), "tile address out of range");
      if (pair) need(t >= 11, "pair ops need tiles of >= 2^11 amplitudes");
      if (code != 1 && code != 2) need(w[100] >= 0 && w[100] < n_gradops, "gradient op index out of range");
      if (code == 3 || code == 4) need(w[101] >= 0 && w[101] < n_gradops, "gradient op index out of range");
    }
    if (code == 6 || code == 7) need(w[2] >= 1 && w[2] <= 8, "observable count out of range");
  }
}

void hea_frags(torch::Tensor params, int64_t p_stride, torch::Tensor slot_tab, int64_t n_slots, int64_t K,
               torch::Tensor frags, bool bf16) {
  need(slot_tab.scalar_type() == torch::kInt32 && slot_tab.numel() >= n_slots * 9, "slot table [n_slots, 9] int32");
  check((bf16 ? qfx_hea_frags_bf16 : qfx_hea_frags)(dp<float>(params, torch::kFloat32, "params", K * p_stride), (int)p_stride,
                      dp<int>(slot_tab, torch::kInt32, "slot_tab", n_slots * 9), (int)n_slots, (int)K,
                      dp<int32_t>(frags, torch::kInt32, "frags", K * n_slots * 4 * 128 * 4), cur()),
        "qfx_hea_frags");
}

// adam: optional (m, v, t_in, t_out, active, cnt) device tensors [K, P] / [K] (cnt int32, zero-initialised) and
// lr, b1, b2, eps: the clients' Adam step fused into the reduction (the last block of each client updates its row)
// readout: optional (rec [K * spc, 2C + 2], loss [K], correct [K]) of a fused-readout step and ro_c = C, ro_ntheta:
// one more block per client reduces the records into loss / correct and the readout-parameter gradients
void hea_grad_reduce(torch::Tensor gslab, int64_t slab_tiles, int64_t n_gradops, torch::Tensor gmeta, int64_t spc,
                     int64_t K, torch::Tensor params, torch::Tensor grad, int64_t p_stride,
                     c10::optional<std::vector<torch::Tensor>> adam, c10::optional<std::vector<double>> hyper,
                     c10::optional<std::vector<torch::Tensor>> readout, int64_t ro_c, int64_t ro_ntheta,
                     c10::optional<std::vector<torch::Tensor>> fed, bool fed_wrap, int64_t fed_n_norms) {
  QfxReadoutRed ro{};
  if (readout && !readout->empty()) {
    const auto& r = *readout;
    need(r.size() == 3 && ro_c >= 1 && ro_c <= 8 && ro_ntheta + 2 * ro_c <= p_stride,
         "grad_reduce: readout = (rec, loss, correct) with 1..8 classes inside the parameter row");
    ro.rec = dp<float>(r[0], torch::kFloat32, "rec", K * spc * (2 * ro_c + 2));
    ro.loss = dp<float>(r[1], torch::kFloat32, "loss", K);
    ro.correct = dp<float>(r[2], torch::kFloat32, "correct", K);
    ro.C = (int)ro_c;
    ro.n_theta = (int)ro_ntheta;
  }
  QfxAdamArgs ad{};
  if (adam && !adam->empty()) {
    const auto& a = *adam;
    need(a.size() == 6 && hyper && hyper->size() == 4, "grad_reduce: adam = (m, v, t_in, t_out, active, cnt), hyper = (lr, b1, b2, eps)");
    need(params.size(1) == p_stride && params.is_contiguous(), "grad_reduce: fused Adam needs contiguous [K, P] params");
    ad.m = dp<float>(a[0], torch::kFloat32, "m", K * p_stride);
    ad.v = dp<float>(a[1], torch::kFloat32, "v", K * p_stride);
    ad.t_in = dp<float>(a[2], torch::kFloat32, "t_in", K);
    ad.t_out = dp<float>(a[3], torch::kFloat32, "t_out", K);
    ad.active = dp<float>(a[4], torch::kFloat32, "active", K);
    ad.cnt = dp<unsigned>(a[5], torch::kInt32, "cnt", K);
    ad.lr = (float)(*hyper)[0], ad.b1 = (float)(*hyper)[1], ad.b2 = (float)(*hyper)[2], ad.eps = (float)(*hyper)[3];
    need(n_gradops > 0 || ro.rec, "grad_reduce: fused Adam needs at least one reduction block");
  }
  // fed = (buf int64 [P + 6 + n_norms], theta_g f32 [P], mask u8 [P], weights f64 [K], loss, correct, nvalid, act
  // f32 [n], cnt int32 [1][, apply_theta f32 [P], apply_out f64 [6 + n_norms]]): the round's FedAvg in the Adam
  // epilogue (QfxFedTail)
  QfxFedTail ft{};
  const bool fused_fed = fed && !fed->empty();
  if (fused_fed) {
    const auto& f = *fed;
    need((f.size() == 9 || f.size() == 11) && ad.m, "grad_reduce: fed = 9 or 11 tensors, with the fused Adam step");
    need(fed_n_norms >= 0, "grad_reduce: fed norm slots");
    ft.buf = dp<long long>(f[0], torch::kInt64, "fed buf", p_stride + 6 + fed_n_norms);
    ft.theta_g = dp<float>(f[1], torch::kFloat32, "fed theta_g", p_stride);
    need(f[2].defined() && f[2].is_cuda() && f[2].scalar_type() == torch::kUInt8 && f[2].numel() >= p_stride,
         "grad_reduce: fed angle mask");
    ft.mask = f[2].data_ptr<uint8_t>();
    ft.weights = dp<double>(f[3], torch::kFloat64, "fed weights", K);
    const int64_t nm = f[4].numel();
    ft.loss = dp<float>(f[4], torch::kFloat32, "fed loss", nm);
    ft.correct = dp<float>(f[5], torch::kFloat32, "fed correct", nm);
    ft.nvalid = dp<float>(f[6], torch::kFloat32, "fed nvalid", nm);
    ft.act = dp<float>(f[7], torch::kFloat32, "fed act", nm);
    ft.n_metrics = (int)nm;
    ft.cnt = dp<unsigned>(f[8], torch::kInt32, "fed cnt", 1);
    ft.wrap = fed_wrap ? 1 : 0;
    ft.n_norms = (int)fed_n_norms;
    if (f.size() == 11) {
      ft.apply_theta = dp<float>(f[9], torch::kFloat32, "fed apply theta", p_stride);
      ft.apply_out = dp<double>(f[10], torch::kFloat64, "fed apply out", 6 + fed_n_norms);
      need(ft.apply_theta == ft.theta_g, "grad_reduce: the single-rank apply updates theta_g in place");
    }
  }
  check(qfx_hea_grad_reduce(dp<long long>(gslab, torch::kInt64, "gslab", K * spc * slab_tiles * n_gradops * 32),
                            (int)slab_tiles, (int)n_gradops, dp<int>(gmeta, torch::kInt32, "gmeta", n_gradops * 10),
                            (int)spc, (int)K, dp<float>(params, torch::kFloat32, "params", K * p_stride),
                            dp<float>(grad, torch::kFloat32, "grad", K * p_stride), (int)p_stride, &ad, &ro,
                            fused_fed ? &ft : nullptr, cur()),
        "qfx_hea_grad_reduce");
}

}  // namespace

void register_hea(pybind11::module& m) {
  m.def("hea_pass", &hea_pass, pybind11::arg("adjoint"), pybind11::arg("ops"), pybind11::arg("fidx"), pybind11::arg("fo"),
        pybind11::arg("geom"), pybind11::arg("scale"), pybind11::arg("psi_in"), pybind11::arg("psi_out"),
        pybind11::arg("lam_in"), pybind11::arg("lam_out"), pybind11::arg("xang"), pybind11::arg("params"),
        pybind11::arg("frags"), pybind11::arg("wread"), pybind11::arg("part"), pybind11::arg("gslab"),
        pybind11::arg("dbg"), pybind11::arg("readout") = pybind11::none(), pybind11::arg("ro_tps") = 0);
  m.def("hea_frags", &hea_frags, pybind11::arg("params"), pybind11::arg("p_stride"), pybind11::arg("slot_tab"),
        pybind11::arg("n_slots"), pybind11::arg("K"), pybind11::arg("frags"), pybind11::arg("bf16") = false);
  m.def("hea_check_ops", &hea_check_ops);
  m.def("hea_grad_reduce", &hea_grad_reduce, pybind11::arg("gslab"), pybind11::arg("slab_tiles"),
        pybind11::arg("n_gradops"), pybind11::arg("gmeta"), pybind11::arg("spc"), pybind11::arg("K"),
        pybind11::arg("params"), pybind11::arg("grad"), pybind11::arg("p_stride"),
        pybind11::arg("adam") = pybind11::none(), pybind11::arg("hyper") = pybind11::none(),
        pybind11::arg("readout") = pybind11::none(), pybind11::arg("ro_c") = 0, pybind11::arg("ro_ntheta") = 0,
        pybind11::arg("fed") = pybind11::none(), pybind11::arg("fed_wrap") = false, pybind11::arg("fed_n_norms") = 0);
  m.def("hea_args_size", []() { return qfx_hea_args_size(); });
  m.attr("HEA_STAMP_ROWS") = HEA_STAMP_ROWS;
  // -1: release build (no device checks); 0: no failure since the last read; else the failing source line
  m.def("hea_check_status", []() { return qfx_hea_check_status(cur()); });
}
