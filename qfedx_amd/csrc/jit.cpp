// Circuit-specialised kernels: plan pass -> straight-line HIP source -> hiprtc (gfx950) -> module.
//
// The ahead-of-time interpreter (statevec.hip) executes any plan, but it must allocate registers
// for the worst of all op variants and spend scalar instructions decoding micro-ops.  For a fixed
// circuit every op code, register bit, remap slot table, gate kind and address offset is known when
// the plan is built, so this generator emits one kernel per pass with all of them as literals: the
// compiler sees straight-line VALU/LDS code, allocates registers exactly, and no op is decoded at
// run time.  Gate ANGLES stay run-time (per-client theta, per-sample features) and are read by the
// same device helpers (qfx_device.h).  Code objects are cached on disk keyed by a hash of the
// generated source + target, so a circuit is compiled once per machine (or shipped pre-built).
#include <hip/hip_runtime.h>
#include <hip/hiprtc.h>

#include <algorithm>
#include <cstdint>
#include <cstdlib>
#include <cstdio>
#include <cstring>
#include <fstream>
#include <memory>
#include <mutex>
#include <sstream>
#include <stdexcept>
#include <string>
#include <sys/stat.h>
#include <unistd.h>
#include <unordered_map>
#include <vector>

#include "qfx_plan.h"

namespace qfx {

namespace {

std::string hex64(uint64_t h) {
  char b[17];
  std::snprintf(b, sizeof(b), "%016llx", (unsigned long long)h);
  return b;
}

uint64_t fnv1a(const std::string& s) {
  uint64_t h = 1469598103934665603ull;
  for (unsigned char c : s) {
    h ^= c;
    h *= 1099511628211ull;
  }
  return h;
}

bool is_diag_kind(int k) {
  return k == K_RZ || k == K_P || k == K_Z || k == K_S || k == K_SDG || k == K_T || k == K_TDG;
}

const char* kind_name(int k) {
  static const char* names[] = {"K_RX", "K_RY", "K_RZ", "K_P", "K_H", "K_X", "K_Y", "K_Z", "K_S", "K_SDG",
                                "K_T", "K_TDG", "K_SX", "K_CX", "K_CZ", "K_SWAP"};
  if (k == K_PAULI) return "K_PAULI";
  return (k >= 0 && k <= 15) ? names[k] : "K_RX";
}

}  // namespace

struct JitSpec {
  std::string source;
  size_t lds = 0;
  int tiles_pb = 1;
  int k = 0, n = 0;
};

// Generate the kernel source for pass `p` of `blob`.
JitSpec codegen_pass(const std::vector<int>& blob, int p, bool adjoint, bool bf16) {
  const int n = blob[HF_N], R = blob[HF_R], G = blob[HF_NGATES], n_theta = blob[HF_NTHETA];
  int RB = 0;
  while ((1 << RB) < R) ++RB;
  const int* pd = blob.data() + blob[HF_PASSES + p];
  const int* gt = blob.data() + blob[HF_GATES];
  const int k = pd[PF_K], tb = pd[PF_TB], T = 1 << tb, TPB = 256 >> tb, ltps = n - k;
  const int init = pd[PF_INIT], fin = pd[PF_FINAL], nops = pd[PF_NOPS], C = pd[PF_NREAD];
  const int* ops = blob.data() + pd[PF_OPS];
  const bool use_tab = T >= 64;
  auto gkind = [&](int g) { return gt[g * GATE_WORDS]; };
  auto gslot = [&](int g) { return gt[g * GATE_WORDS + 3]; };
  auto is_grad = [&](int g) { return adjoint && gslot(g) >= 0 && gslot(g) < n_theta && gkind(g) <= K_P; };
  // adjoint: is the gate's inverse needed by a live gate earlier in the circuit (processed later)?
  // (same liveness as the planner, which already dropped the dead gates)
  std::vector<char> need_inv(G, 1);
  if (adjoint) {
    std::vector<char> has_live(n, 0);
    for (int g = 0; g < G; ++g) {
      const int kd = gkind(g), q0 = gt[g * GATE_WORDS + 1], q1 = gt[g * GATE_WORDS + 2];
      const bool two = kd == K_CX || kd == K_CZ;
      const bool nd = has_live[q0] || (two && has_live[q1]);
      need_inv[g] = nd;
      if (is_grad(g) || nd) {
        has_live[q0] = 1;
        if (two) has_live[q1] = 1;
      }
    }
  }

  // gates referenced by this pass (coefficient table entries)
  std::vector<int> used, slot_of(G, -1);
  auto use = [&](int g) {
    if (slot_of[g] < 0) {
      slot_of[g] = (int)used.size();
      used.push_back(g);
    }
  };
  std::vector<int> grad_gates;
  for (int i = 0; i < nops; ++i) {
    const int* o = ops + i * OP_WORDS;
    if (o[0] == OP_G1) {
      for (int j = 0; j < o[2]; ++j) {
        use(blob[o[3] + j]);
        if (is_grad(blob[o[3] + j])) grad_gates.push_back(blob[o[3] + j]);
      }
    } else if (o[0] == OP_D1T) {
      use(o[3]);
      if (is_grad(o[3]) && (gkind(o[3]) == K_RZ || gkind(o[3]) == K_P)) grad_gates.push_back(o[3]);
    }
  }
  const int NG = std::max<int>(1, (int)used.size());
  const int NGR = (int)grad_gates.size();
  // forward fused 1-qubit groups: with one tile per wave or more (T >= 64) their 2x2 products are
  // tile-uniform, so they are built once per tile in LDS (gtab) instead of by every lane
  std::vector<std::vector<int>> fgroups;
  if (!adjoint)
    for (int i = 0; i < nops; ++i) {
      const int* o = ops + i * OP_WORDS;
      if (o[0] == OP_G1) fgroups.emplace_back(blob.begin() + o[3], blob.begin() + o[3] + o[2]);
    }
  const int NG1 = (int)fgroups.size();
  const bool use_gtab = use_tab && NG1 > 0;

  auto pbit_expr = [&](int phys, const std::string& r) -> std::string {
    if (phys < RB) return "((" + r + " >> " + std::to_string(phys) + ") & 1)";
    if (phys < PHYS_NONTILE) return "((tl >> " + std::to_string(phys - RB) + ") & 1)";
    return "((gbase >> " + std::to_string(phys - PHYS_NONTILE) + ") & 1u)";
  };
  auto xor_expr = [&](const int* tab, int cnt) {
    std::ostringstream e;
    e << "0u";
    for (int j = 0; j < cnt; ++j) e << " ^ (((tl >> " << j << ") & 1) ? " << (uint32_t)tab[j] << "u : 0u)";
    return e.str();
  };
  auto cs = [&](int g) {
    std::ostringstream e;
    if (use_tab) e << "ctab[tib * " << NG << " + " << slot_of[g] << "]";
    else e << "gate_cs(gt, " << g << ", prow, xrow, " << n_theta << ")";
    return e.str();
  };

  // state loads / stores: complex64, or packed bf16x2 (state_dtype=bf16)
  auto ld = [&](const std::string& arr, const std::string& idx) -> std::string {
    if (bf16) return "unpack_bf16x2(reinterpret_cast<const uint32_t*>(A." + arr + ")[" + idx + "])";
    return "A." + arr + "[" + idx + "]";
  };
  auto st = [&](const std::string& arr, const std::string& idx, const std::string& v) -> std::string {
    if (bf16) return "reinterpret_cast<uint32_t*>(A." + arr + ")[" + idx + "] = pack_bf16x2(" + v + ")";
    return "A." + arr + "[" + idx + "] = " + v;
  };

  std::ostringstream s;
  s << "// generated by qfedx_amd/csrc/jit.cpp - pass " << p << (adjoint ? " (adjoint)" : " (forward)")
    << (bf16 ? " bf16 state" : "") << "\n";
  s << "#include \"qfx_device.h\"\n";
  // occupancy target (waves per SIMD) for the register allocator: QFEDX_JIT_WAVES[_ADJ|_FWD] (0 = compiler
  // default).  Part of the generated source, hence of the code-object cache key.
  int waves = 0;
  if (const char* e = std::getenv(adjoint ? "QFEDX_JIT_WAVES_ADJ" : "QFEDX_JIT_WAVES_FWD")) waves = std::atoi(e);
  else if (const char* e2 = std::getenv("QFEDX_JIT_WAVES")) waves = std::atoi(e2);
  s << "extern \"C\" __global__ void __launch_bounds__(256)";
  if (waves > 0) s << " __attribute__((amdgpu_waves_per_eu(" << waves << ", " << waves << ")))";
  s << " qfx_jit_pass(qfx::PassArgs A) {\n";
  s << "  using namespace qfx;\n";
  s << "  constexpr int R = " << R << ", T = " << T << ", TPB = " << TPB << ", G = " << G << ";\n";
  s << "  extern __shared__ __attribute__((aligned(16))) char smem[];\n";
  s << "  const int tid = threadIdx.x, tib = tid >> " << tb << ", tl = tid & " << (T - 1) << ";\n";
  s << "  const long tile = (long)blockIdx.x * TPB + tib;\n";
  s << "  const long sample = tile >> " << ltps << ";\n";
  s << "  const uint32_t tau = (uint32_t)(tile & " << ((1L << ltps) - 1) << "L);\n";
  s << "  const bool valid = sample < A.n_samples;\n";
  s << "  const long s_eff = valid ? sample : 0;\n";
  s << "  const size_t sbase = (size_t)s_eff << " << n << ";\n";
  s << "  const float* prow = A.params + (size_t)(s_eff / A.spc) * A.p_stride;\n";
  s << "  const float* xrow = A.xang + (size_t)s_eff * A.x_stride;\n";
  s << "  const int wave = tid >> 6, lane = tid & 63;\n";
  s << "  (void)wave; (void)lane; (void)prow; (void)xrow;\n";
  s << "  cint_p gt = (cint_p)(A.blob) + " << blob[HF_GATES] << ";\n";
  s << "  (void)gt;\n";
  {
    s << "  const uint32_t gbase = 0u";
    const int nn = pd[PF_NNONTILE];
    for (int j = 0; j < nn; ++j) s << " | (((tau >> " << j << ") & 1u) << " << pd[PF_NONTILE + j] << ")";
    s << ";\n  (void)gbase;\n";
  }
  const int gacc_words = std::max(NGR, 1) * 16;
  s << "  v2f* xb = reinterpret_cast<v2f*>(smem) + (size_t)tib * " << (1u << k) << ";\n";
  s << "  float* red = reinterpret_cast<float*>(smem + " << (256 * R * 8) << ");\n";
  s << "  float* gacc = red + 128;\n";
  s << "  v2f* ctab = reinterpret_cast<v2f*>(gacc + " << gacc_words << ");\n";
  s << "  float4* vtab = reinterpret_cast<float4*>(ctab + " << ((TPB * NG + 1) & ~1) << ");\n";
  s << "  M2* gtab = reinterpret_cast<M2*>(vtab + " << TPB * n << ");\n";
  s << "  (void)xb; (void)red; (void)gacc; (void)ctab; (void)vtab; (void)gtab;\n";
  if (use_tab) {
    s << "  {\n    const long tile0 = (long)blockIdx.x * TPB;\n";
    s << "    static constexpr int USED[" << NG << "] = {";
    for (int i = 0; i < NG; ++i) s << (i ? "," : "") << (i < (int)used.size() ? used[i] : 0);
    s << "};\n";
    s << "    for (int e = tid; e < TPB * " << NG << "; e += 256) {\n";
    s << "      const int tb_ = e / " << NG << ", i = e - tb_ * " << NG << ";\n";
    s << "      long sm = (tile0 + tb_) >> " << ltps << "; if (sm >= A.n_samples) sm = 0;\n";
    s << "      ctab[e] = gate_cs(gt, USED[i], A.params + (size_t)(sm / A.spc) * A.p_stride, A.xang + (size_t)sm * A.x_stride, "
      << n_theta << ");\n    }\n";
    if (init == INIT_PRODUCT) {
      s << "    for (int e = tid; e < TPB * " << n << "; e += 256) {\n";
      s << "      const int tb_ = e / " << n << ", q = e - tb_ * " << n << ";\n";
      s << "      long sm = (tile0 + tb_) >> " << ltps << "; if (sm >= A.n_samples) sm = 0;\n";
      s << "      vtab[e] = prefix_vec((cint_p)(A.blob), q, A.params + (size_t)(sm / A.spc) * A.p_stride, A.xang + (size_t)sm * A.x_stride, "
        << n_theta << ");\n    }\n";
    }
    s << "    __syncthreads();\n";
    if (use_gtab) {
      s << "    for (int e = tid; e < TPB * " << NG1 << "; e += 256) {\n";
      s << "      const int tb_ = e / " << NG1 << ", i = e - tb_ * " << NG1 << ";\n";
      s << "      M2 m;\n      switch (i) {\n";
      for (int gi = 0; gi < NG1; ++gi) {
        const auto& gl = fgroups[gi];
        auto csx = [&](int g) { return "ctab[tb_ * " + std::to_string(NG) + " + " + std::to_string(slot_of[g]) + "]"; };
        s << "        case " << gi << ": m = gate_m2(" << kind_name(gkind(gl[0])) << ", " << csx(gl[0]) << ", false);";
        for (size_t j = 1; j < gl.size(); ++j)
          s << " m = m2mul(gate_m2(" << kind_name(gkind(gl[j])) << ", " << csx(gl[j]) << ", false), m);";
        s << " break;\n";
      }
      s << "        default: m = gate_m2(K_X, mk(0.f, 0.f), false); break;\n      }\n";
      s << "      gtab[e] = m;\n    }\n    __syncthreads();\n";
    }
    s << "  }\n";
  }
  s << "  v2f a[R];\n  v2f l[R];\n";
  s << "#pragma unroll\n  for (int r = 0; r < R; ++r) { a[r] = mk(0.f, 0.f); l[r] = mk(0.f, 0.f); }\n";

  // ---------------------------------------------------------------- init
  if (init == INIT_PRODUCT) {
    auto vq = [&](int q) {
      std::ostringstream e;
      if (use_tab) e << "vtab[tib * " << n << " + " << q << "]";
      else e << "prefix_vec((cint_p)(A.blob), " << q << ", prow, xrow, " << n_theta << ")";
      return e.str();
    };
    s << "  {\n    v2f base = mk(1.f, 0.f);\n";
    const int nn = pd[PF_NNONTILE];
    for (int j = 0; j < nn; ++j) {
      int q = pd[PF_NONTILE + j];
      s << "    { const float4 v = " << vq(q) << "; base = cmul(base, ((gbase >> " << q
        << ") & 1u) ? mk(v.z, v.w) : mk(v.x, v.y)); }\n";
    }
    for (int pp = RB; pp < k; ++pp) {
      int q = pd[PF_Q0 + pp];
      s << "    { const float4 v = " << vq(q) << "; base = cmul(base, ((tl >> " << (pp - RB)
        << ") & 1) ? mk(v.z, v.w) : mk(v.x, v.y)); }\n";
    }
    s << "    a[0] = base;\n";
    for (int pp = 0; pp < RB; ++pp) {
      int q = pd[PF_Q0 + pp];
      s << "    { const float4 v = " << vq(q) << ";\n";
      for (int r = 0; r < (1 << pp); ++r)
        s << "      a[" << (r | (1 << pp)) << "] = cmul(mk(v.z, v.w), a[" << r << "]); a[" << r << "] = cmul(mk(v.x, v.y), a["
          << r << "]);\n";
      s << "    }\n";
    }
    s << "  }\n";
  } else {
    s << "  {\n    const uint32_t gthr = " << xor_expr(pd + PF_GTHR0, tb) << ";\n";
    s << "    if (valid) {\n";
    for (int r = 0; r < R; ++r) {
      s << "      a[" << r << "] = " << ld("psi", "sbase + gbase + (gthr | " + std::to_string((uint32_t)pd[PF_GREG0 + r]) + "u)") << ";\n";
      if (adjoint && init == INIT_LOAD_BOTH)
        s << "      l[" << r << "] = " << ld("lam", "sbase + gbase + (gthr | " + std::to_string((uint32_t)pd[PF_GREG0 + r]) + "u)") << ";\n";
    }
    s << "    }\n  }\n";
    if (adjoint && init == INIT_PSI_LAMBDA) {
      s << "  {\n";
      for (int c = 0; c < C; ++c)
        s << "    const float w" << c << " = valid ? A.w_read[(size_t)s_eff * " << C << " + " << c << "] : 0.f;\n";
      for (int r = 0; r < R; ++r) {
        s << "    { const float sc = 0.f";
        for (int c = 0; c < C; ++c)
          s << " + (" << pbit_expr(pd[PF_LAM_PHYS + c], std::to_string(r)) << " ? -w" << c << " : w" << c << ")";
        s << "; l[" << r << "] = mk(a[" << r << "].x * sc, a[" << r << "].y * sc); }\n";
      }
      s << "  }\n";
    }
  }

  // ---------------------------------------------------------------- ops
  int gi_local = 0;
  int g1_idx = 0;
  auto emit_grad = [&](int g, const std::string& part) {
    // row-local DPP sum; tiles wider than a 16-lane row park one partial per row in LDS and
    // are summed once at the end of the kernel
    s << "    { float pg = row_sum<" << std::min(T, 16) << ">(" << part << ");\n";
    if (T <= 16) s << "      if (tl == 0 && valid) A.gslab[(size_t)tile * G + " << g << "] = pg; }\n";
    else s << "      if ((lane & 15) == 0) gacc[" << gi_local << " * 16 + (tid >> 4)] = pg; }\n";
    ++gi_local;
  };
  for (int i = 0; i < nops; ++i) {
    const int* o = ops + i * OP_WORDS;
    const int code = o[0], oa = o[1], ob = o[2], oc = o[3];
    if (code == OP_G1) {
      std::vector<int> gl(blob.begin() + oc, blob.begin() + oc + ob);
      if (!adjoint && use_gtab) {
        s << "  { const M2 m = gtab[tib * " << NG1 << " + " << g1_idx++ << "]; m2_apply<R, " << oa << ">(a, m); }\n";
      } else if (!adjoint) {
        s << "  { M2 m = gate_m2(" << kind_name(gkind(gl[0])) << ", " << cs(gl[0]) << ", false);\n";
        for (size_t j = 1; j < gl.size(); ++j)
          s << "    m = m2mul(gate_m2(" << kind_name(gkind(gl[j])) << ", " << cs(gl[j]) << ", false), m);\n";
        s << "    m2_apply<R, " << oa << ">(a, m); }\n";
      } else {
        for (int g : gl) {
          const int kd = gkind(g);
          const char* cls = is_grad(g) ? (kd == K_RX ? "CLS_RX" : kd == K_RY ? "CLS_RY" : "CLS_RZ")
                                       : (is_diag_kind(kd) ? "CLS_DIAG" : kd == K_RX ? "CLS_RX"
                                                                        : kd == K_RY ? "CLS_RY" : "CLS_GEN");
          if (is_grad(g) && !need_inv[g]) {   // gradient only: nothing processed later needs the inverse
            s << "  { const float part = adj_grad_only<R, " << oa << ", " << cls << ">(a, l);\n";
            emit_grad(g, "part");
            s << "  }\n";
            continue;
          }
          s << "  { const M2 mi = gate_m2(" << kind_name(kd) << ", " << cs(g) << ", true);\n";
          s << "    const float part = adj_step<R, " << oa << ", " << cls << ">(a, l, mi); (void)part;\n";
          if (is_grad(g)) emit_grad(g, "part");
          s << "  }\n";
        }
      }
    } else if (code == OP_D1T) {
      const int kd = gkind(oc);
      s << "  { const M2 m = gate_m2(" << kind_name(kd) << ", " << cs(oc) << ", " << (adjoint ? "true" : "false") << ");\n";
      s << "    const int bit = " << pbit_expr(oa, "0") << ";\n";
      s << "    const v2f ph = bit ? m.d : m.a;\n";
      if (adjoint && is_grad(oc) && (kd == K_RZ || kd == K_P)) {
        s << "    float part = 0.f;\n";
        s << "#pragma unroll\n    for (int r = 0; r < R; ++r) part += imcl(l[r], a[r]);\n";
        s << "    part = bit ? -part : part;\n";
        emit_grad(oc, "part");
      }
      if (adjoint && !need_inv[oc]) s << "  }\n";   // phase not needed by anything processed later
      else
        s << "#pragma unroll\n    for (int r = 0; r < R; ++r) { a[r] = cmul(ph, a[r]);"
          << (adjoint ? " l[r] = cmul(ph, l[r]);" : "") << " }\n  }\n";
    } else if (code == OP_REMAP) {
      const int* tab = blob.data() + oa;
      const int* wr = tab;
      const int* wt = tab + R;
      const int* rr = tab + R + tb;
      const int* rt = tab + 2 * R + tb;
      s << "  { const uint32_t wthr = " << xor_expr(wt, tb) << ";\n";
      s << "    const uint32_t rthr = " << xor_expr(rt, tb) << ";\n";
      // slot(r) = C_r ^ thr where thr only has bits in M = OR of the thread contributions: bits of C_r
      // outside M are ADDED (disjoint), so they become ds immediate offsets; one XOR per distinct
      // (C_r & M) pattern builds a base pointer instead of one XOR + shift-add per access
      auto bases = [&](const int* tc, const int* tt, const char* thr, const char* pre) {
        uint32_t M = 0;
        for (int j = 0; j < tb; ++j) M |= (uint32_t)tt[j];
        std::vector<std::pair<uint32_t, std::string>> ref(R);
        std::vector<uint32_t> seen;
        for (int r = 0; r < R; ++r) {
          const uint32_t lo = (uint32_t)tc[r] & M, hi = (uint32_t)tc[r] & ~M;
          size_t id = std::find(seen.begin(), seen.end(), lo) - seen.begin();
          if (id == seen.size()) {
            seen.push_back(lo);
            s << "    v2f* " << pre << id << " = xb + (" << lo << "u ^ " << thr << ");\n";
          }
          ref[r] = {hi, std::string(pre) + std::to_string(id)};
        }
        return ref;
      };
      const auto wref = bases(wr, wt, "wthr", "wb");
      const auto rref = bases(rr, rt, "rthr", "rb");
      const char* arrs[2] = {"a", "l"};
      for (int st = 0; st < (adjoint ? 2 : 1); ++st) {
        s << "    __syncthreads();\n";
        for (int r = 0; r < R; ++r)
          s << "    " << wref[r].second << "[" << wref[r].first << "u] = " << arrs[st] << "[" << r << "];\n";
        s << "    __syncthreads();\n";
        for (int r = 0; r < R; ++r)
          s << "    " << arrs[st] << "[" << r << "] = " << rref[r].second << "[" << rref[r].first << "u];\n";
      }
      s << "  }\n";
    } else if (code == OP_CX) {
      s << "  cx_apply<R, " << RB << ", " << ob << ", " << (adjoint ? "true" : "false") << ">(a, l, " << oa
        << ", tl, gbase);\n";
    } else if (code == OP_CZ) {
      s << "#pragma unroll\n  for (int r = 0; r < R; ++r) if (" << pbit_expr(oa, "r") << " & " << pbit_expr(ob, "r")
        << ") { a[r] = mk(-a[r].x, -a[r].y);" << (adjoint ? " l[r] = mk(-l[r].x, -l[r].y);" : "") << " }\n";
    }
  }

  // ---------------------------------------------------------------- finalize
  if (adjoint && T > 16 && NGR > 0) {
    s << "  __syncthreads();\n";
    s << "  {\n    static constexpr int GG[" << NGR << "] = {";
    for (int i = 0; i < NGR; ++i) s << (i ? "," : "") << grad_gates[i];
    s << "};\n";
    // tile tb_ owns rows [tb_ * RPT, (tb_ + 1) * RPT) of the block's 16 rows of 16 lanes
    const int RPT = T / 16;
    s << "    for (int e = tid; e < " << TPB * NGR << "; e += 256) {\n";
    s << "      const int tb_ = e / " << NGR << ", g = e - tb_ * " << NGR << ";\n";
    s << "      float sum = 0.f;\n";
    s << "#pragma unroll\n      for (int w = 0; w < " << RPT << "; ++w) sum += gacc[g * 16 + tb_ * " << RPT << " + w];\n";
    s << "      const long tile_ = (long)blockIdx.x * TPB + tb_;\n";
    s << "      if ((tile_ >> " << ltps << ") < A.n_samples) A.gslab[(size_t)tile_ * G + GG[g]] = sum;\n    }\n";
    s << "  }\n";
  }
  if (fin & FIN_READOUT) {
    for (int c = 0; c < C; ++c) {
      const int ph = pd[PF_READ_PHYS + c];
      s << "  { float acc = 0.f;\n";
      s << "#pragma unroll\n    for (int r = 0; r < R; ++r) { const float pr = fmaf(a[r].x, a[r].x, a[r].y * a[r].y); acc += "
        << pbit_expr(ph, "r") << " ? -pr : pr; }\n";
      s << "    acc = row_sum<" << std::min(T, 16) << ">(acc);\n";
      if (T <= 16) s << "    if (tl == 0 && valid) A.out_read[(size_t)tile * " << C << " + " << c << "] = acc; }\n";
      else s << "    if ((lane & 15) == 0) red[" << c << " * 16 + (tid >> 4)] = acc; }\n";
    }
    if (T > 16) {
      s << "  __syncthreads();\n";
      const int RPT = T / 16;
      s << "  for (int e = tid; e < " << TPB * C << "; e += 256) {\n";
      s << "    const int tb_ = e / " << C << ", c = e - tb_ * " << C << ";\n";
      s << "    float sum = 0.f;\n";
      s << "#pragma unroll\n    for (int w = 0; w < " << RPT << "; ++w) sum += red[c * 16 + tb_ * " << RPT << " + w];\n";
      s << "    const long tile_ = (long)blockIdx.x * TPB + tb_;\n";
      s << "    if ((tile_ >> " << ltps << ") < A.n_samples) A.out_read[(size_t)tile_ * " << C << " + c] = sum;\n  }\n";
    }
  }
  if (fin & FIN_STORE) {
    s << "  {\n    const uint32_t gthr = " << xor_expr(pd + PF_GTHRF, tb) << ";\n    if (valid) {\n";
    for (int r = 0; r < R; ++r) {
      const std::string idx = "sbase + gbase + (gthr | " + std::to_string((uint32_t)pd[PF_GREGF + r]) + "u)";
      s << "      " << st("psi", idx, "a[" + std::to_string(r) + "]") << ";\n";
      if (adjoint) s << "      " << st("lam", idx, "l[" + std::to_string(r) + "]") << ";\n";
    }
    s << "    }\n  }\n";
  }
  s << "}\n";

  JitSpec spec;
  spec.source = s.str();
  spec.tiles_pb = TPB;
  spec.k = k;
  spec.n = n;
  spec.lds = 256 * (size_t)R * 8 + 128 * 4 + (size_t)gacc_words * 4 +
             (use_tab ? (size_t)((TPB * NG + 1) & ~1) * 8 + (size_t)TPB * n * 16 : 0) +
             (use_gtab ? (size_t)TPB * NG1 * 32 : 0);
  return spec;
}

// ------------------------------------------------------------------------------ compile + cache
std::vector<char> hiprtc_compile(const std::string& src, const std::string& include_dir, const std::string& arch) {
  hiprtcProgram prog;
  if (hiprtcCreateProgram(&prog, src.c_str(), "qfx_jit.hip", 0, nullptr, nullptr) != HIPRTC_SUCCESS)
    throw std::runtime_error("hiprtcCreateProgram failed");
  std::string a = "--offload-arch=" + arch, inc = "-I" + include_dir;
  const char* opts[] = {a.c_str(), inc.c_str(), "-O3", "-std=c++17"};
  hiprtcResult rc = hiprtcCompileProgram(prog, 4, opts);
  if (rc != HIPRTC_SUCCESS) {
    size_t ls = 0;
    hiprtcGetProgramLogSize(prog, &ls);
    std::string log(ls, '\0');
    hiprtcGetProgramLog(prog, &log[0]);
    hiprtcDestroyProgram(&prog);
    throw std::runtime_error("hiprtc compile failed:\n" + log.substr(0, 4000));
  }
  size_t cs = 0;
  hiprtcGetCodeSize(prog, &cs);
  std::vector<char> code(cs);
  hiprtcGetCode(prog, code.data());
  hiprtcDestroyProgram(&prog);
  return code;
}

struct JitEntry {
  std::vector<char> code;
  hipModule_t mod = nullptr;
  hipFunction_t fn = nullptr;
  size_t lds = 0;
  int tiles_pb = 1, k = 0, n = 0;
  bool bf16 = false;
  std::string key;
};

static std::mutex g_mu;
static std::vector<std::unique_ptr<JitEntry>> g_entries;
static std::unordered_map<std::string, int> g_by_key;

static bool file_exists(const std::string& p) {
  struct stat st;
  return stat(p.c_str(), &st) == 0;
}

// Generate + compile (or load from the disk cache) pass p; returns a handle.  No GPU needed.
int jit_prepare(const std::vector<int>& blob, int p, bool adjoint, const std::string& cache_dir,
                const std::string& include_dir, const std::string& arch, std::string* key_out, bool bf16) {
  JitSpec spec = codegen_pass(blob, p, adjoint, bf16);
  std::string header;
  {
    std::ifstream f(include_dir + "/qfx_device.h");
    std::stringstream ss;
    ss << f.rdbuf();
    header = ss.str();
    std::ifstream f2(include_dir + "/qfx_plan.h");
    std::stringstream ss2;
    ss2 << f2.rdbuf();
    header += ss2.str();
  }
  const std::string key = hex64(fnv1a(spec.source + header + arch));
  if (key_out) *key_out = key;
  std::lock_guard<std::mutex> lk(g_mu);
  auto it = g_by_key.find(key);
  if (it != g_by_key.end()) return it->second;
  auto e = std::make_unique<JitEntry>();
  e->lds = spec.lds;
  e->tiles_pb = spec.tiles_pb;
  e->k = spec.k;
  e->n = spec.n;
  e->bf16 = bf16;
  e->key = key;
  const std::string path = cache_dir + "/" + key + ".co";
  if (!cache_dir.empty() && file_exists(path)) {
    std::ifstream f(path, std::ios::binary);
    e->code.assign(std::istreambuf_iterator<char>(f), std::istreambuf_iterator<char>());
  }
  if (e->code.empty()) {
    e->code = hiprtc_compile(spec.source, include_dir, arch);
    if (!cache_dir.empty()) {
      mkdir(cache_dir.c_str(), 0755);
      // one temp file per process: the ranks of a node share the cache and may compile the same key at once;
      // each renames a complete file of its own over the entry, so a reader never sees a partial code object
      const std::string tag = "." + std::to_string((long)getpid()) + ".tmp";
      std::string tmp = path + tag;
      bool ok;
      {
        std::ofstream f(tmp, std::ios::binary);
        f.write(e->code.data(), (std::streamsize)e->code.size());
        ok = (bool)f;
      }
      if (ok) std::rename(tmp.c_str(), path.c_str());
      else std::remove(tmp.c_str());
      const std::string src = cache_dir + "/" + key + ".hip";
      {
        std::ofstream fs(src + tag);
        fs << spec.source;
      }
      std::rename((src + tag).c_str(), src.c_str());
    }
  }
  g_entries.push_back(std::move(e));
  int h = (int)g_entries.size() - 1;
  g_by_key[key] = h;
  return h;
}

std::string jit_source(const std::vector<int>& blob, int p, bool adjoint, bool bf16) {
  return codegen_pass(blob, p, adjoint, bf16).source;
}

struct PassArgsHost {   // must match qfx::PassArgs in qfx_device.h
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

// bytes of one sample's statevector in the kernel's storage format (-1: bad handle)
long jit_state_bytes(int handle, bool* bf16) {
  std::lock_guard<std::mutex> lk(g_mu);
  if (handle < 0 || handle >= (int)g_entries.size()) return -1;
  const JitEntry* e = g_entries[handle].get();
  if (bf16) *bf16 = e->bf16;
  return (1L << e->n) * (e->bf16 ? 4L : 8L);
}

int jit_launch(int handle, const PassArgsHost& args, hipStream_t stream) {
  JitEntry* e;
  {
    std::lock_guard<std::mutex> lk(g_mu);
    if (handle < 0 || handle >= (int)g_entries.size()) return -10;
    e = g_entries[handle].get();
    if (!e->fn) {
      if (hipModuleLoadData(&e->mod, e->code.data()) != hipSuccess) return -11;
      if (hipModuleGetFunction(&e->fn, e->mod, "qfx_jit_pass") != hipSuccess) return -12;
    }
  }
  const long tiles_total = (long)args.n_samples << (e->n - e->k);
  const long blocks = (tiles_total + e->tiles_pb - 1) / e->tiles_pb;
  if (blocks <= 0) return 0;
  PassArgsHost a = args;
  void* params[] = {&a};
  hipError_t rc = hipModuleLaunchKernel(e->fn, (unsigned)blocks, 1, 1, 256, 1, 1, (unsigned)e->lds, stream, params, nullptr);
  return (int)rc;
}

}  // namespace qfx
