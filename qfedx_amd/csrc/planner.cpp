// Host-side pass planner: lowered circuit -> fused LDS-tile passes for the gfx950 kernels.
//
// Native equivalent of a circuit "graph builder / scheduler": the reference has none (its only
// quantum execution is Qiskit's Statevector, src/QFed/qAmplitude.py:44-46); the ROADMAP's VQC
// (ROADMAP.md:20-23,125-135) needs one to run 16-24 qubit circuits at HBM speed.  Strategy
// (SURVEY §2.3 K12b, §7.3 items 1-2):
//   * greedy DAG-frontier fusion: a pass keeps adding gates while the set of tile qubits needed in
//     registers stays <= k; diagonal gates and CZ need no tile membership (their bits can be
//     uniform per tile); CX controls may be outside the tile;
//   * the feature map + first rotation layer (all single-qubit gates before a qubit's first
//     two-qubit gate) collapse into a closed-form product-state initialisation (K11): no load;
//   * register allocation: Belady-style look-ahead over the register-bit demand sequence;
//   * CNOT chains with both qubits in the tile fold into a GF(2)-linear index map that is applied
//     for free inside the next LDS remap;
//   * the first and last layouts put qubits 0..3 on thread bits 0..3 so every 16-lane group moves
//     a contiguous 128-byte line (coalesced HBM access).
#include "qfx_plan.h"

#include <cstdint>

#include <algorithm>
#include <cstring>
#include <stdexcept>
#include <string>
#include <vector>

namespace qfx {

struct PGate {
  int kind, q0, q1, slot;
  float scale, offset;
};

static inline bool is_diag(int k) {
  return k == K_RZ || k == K_P || k == K_Z || k == K_S || k == K_SDG || k == K_T || k == K_TDG ||
         k == K_CZ;
}
static inline bool is_1q(int k) { return k <= K_SX || k == K_PAULI; }

static int f2i(float f) {
  int i;
  std::memcpy(&i, &f, 4);
  return i;
}

struct PassBuild {
  std::vector<int> tileq;            // tile bit -> qubit (ascending)
  std::vector<int> sched;            // gate indices in execution order
};

class Planner {
 public:
  Planner(int n, int R, int kmax, const std::vector<PGate>& gates, const std::vector<int>& readout,
          int n_theta)
      : n_(n), R_(R), gates_(gates), readout_(readout), n_theta_(n_theta) {
    if (R > 32 || R < 2) throw std::invalid_argument("R must be in [2, 32]");
    if (n > 30) throw std::invalid_argument("at most 30 qubits per state");
    rb_ = 0;
    while ((1 << rb_) < R) ++rb_;
    if ((1 << rb_) != R) throw std::invalid_argument("R must be a power of two");
    k_ = std::min(n, kmax);
    if (k_ < rb_) throw std::invalid_argument("n_qubits too small for R");
    tb_ = k_ - rb_;
    coal_ = std::min(4, std::min(tb_, k_));
    if ((int)readout_.size() > 8) throw std::invalid_argument("at most 8 readout qubits");
    for (auto& g : gates_) {
      if (g.q0 < 0 || g.q0 >= n) throw std::invalid_argument("gate qubit out of range");
      if (!is_1q(g.kind) && (g.q1 < 0 || g.q1 >= n)) throw std::invalid_argument("bad 2q gate");
      if (g.kind == K_SWAP) throw std::invalid_argument("SWAP must be lowered to CX");
    }
  }

  // mode: 0 = forward (product-state prefix), 1 = forward from a loaded state, 2 = adjoint
  std::vector<int> build(int mode, int final_flags) {
    std::vector<int> order(gates_.size());
    for (size_t i = 0; i < order.size(); ++i) order[i] = (int)i;
    std::vector<std::vector<int>> prefix(n_);
    std::vector<int> body;
    if (mode == 2) {
      // adjoint sweep = reverse circuit order.  A gate's inverse is only needed if some gate EARLIER in
      // the circuit (processed later) on one of its qubits is live (a gradient gate, or a gate whose
      // inverse is needed): gates that are neither are dead work (e.g. the feature map) and dropped.
      const std::vector<char> live = adjoint_liveness(nullptr);
      std::reverse(order.begin(), order.end());
      for (int gi : order)
        if (live[gi]) body.push_back(gi);
    } else if (mode == 0) {
      std::vector<char> ent(n_, 0);
      for (int gi : order) {
        const PGate& g = gates_[gi];
        if (is_1q(g.kind) && !ent[g.q0]) {
          prefix[g.q0].push_back(gi);
        } else {
          ent[g.q0] = 1;
          if (!is_1q(g.kind)) ent[g.q1] = 1;
          body.push_back(gi);
        }
      }
    } else {
      body = order;
    }

    // ---- pass formation ----------------------------------------------------------------
    std::vector<PassBuild> passes;
    std::vector<int> remaining = body;
    do {
      PassBuild pb;
      std::vector<char> inS(n_, 0), blocked(n_, 0);
      int sz = 0;
      if (n_ > k_)
        for (int q = 0; q < coal_; ++q) inS[q] = 1, ++sz;
      std::vector<int> rest;
      for (int gi : remaining) {
        const PGate& g = gates_[gi];
        bool two = !is_1q(g.kind);
        bool blk = blocked[g.q0] || (two && blocked[g.q1]);
        if (!blk) {
          int need = -1;
          if (is_1q(g.kind) && !is_diag(g.kind)) need = g.q0;
          else if (g.kind == K_CX) need = g.q1;
          if (need < 0 || inS[need] || sz < k_) {
            if (need >= 0 && !inS[need]) inS[need] = 1, ++sz;
            pb.sched.push_back(gi);
            continue;
          }
        }
        blocked[g.q0] = 1;
        if (two) blocked[g.q1] = 1;
        rest.push_back(gi);
      }
      for (int q = 0; q < n_ && sz < k_; ++q)
        if (!inS[q]) inS[q] = 1, ++sz;
      for (int q = 0; q < n_; ++q)
        if (inS[q]) pb.tileq.push_back(q);
      passes.push_back(pb);
      remaining.swap(rest);
    } while (!remaining.empty());

    // ---- emit blob -------------------------------------------------------------------
    std::vector<int> blob(HF_PASSES + passes.size(), 0);
    blob[HF_N] = n_;
    blob[HF_NPASS] = (int)passes.size();
    blob[HF_NGATES] = (int)gates_.size();
    blob[HF_R] = R_;
    blob[HF_NREAD] = (int)readout_.size();
    blob[HF_NTHETA] = n_theta_;
    // gate table
    blob[HF_GATES] = (int)blob.size();
    for (const PGate& g : gates_) {
      blob.push_back(g.kind);
      blob.push_back(g.q0);
      blob.push_back(g.q1);
      blob.push_back(g.slot);
      blob.push_back(f2i(g.scale));
      blob.push_back(f2i(g.offset));
    }
    // product-state prefix lists: per qubit [count, gates...]
    blob[HF_PREFIX] = (int)blob.size();
    std::vector<int> pref_off(n_);
    {
      size_t base = blob.size();
      blob.resize(base + n_, 0);
      for (int q = 0; q < n_; ++q) {
        blob[base + q] = (int)blob.size();
        blob.push_back((int)prefix[q].size());
        for (int gi : prefix[q]) blob.push_back(gi);
      }
    }
    for (size_t p = 0; p < passes.size(); ++p) {
      int init;
      if (mode == 2) init = (p == 0) ? INIT_PSI_LAMBDA : INIT_LOAD_BOTH;
      else if (mode == 0) init = (p == 0) ? INIT_PRODUCT : INIT_LOAD;
      else init = INIT_LOAD;
      int fin;
      bool last = p + 1 == passes.size();
      if (mode == 2) fin = last ? 0 : FIN_STORE;
      else fin = last ? final_flags : FIN_STORE;
      blob[HF_PASSES + p] = (int)blob.size();
      emit_pass(blob, passes[p], init, fin, mode == 2);
    }
    return blob;
  }

 private:
  // live[g] (grad gate or inverse needed) and, optionally, need_inverse[g], in circuit order
  std::vector<char> adjoint_liveness(std::vector<char>* need_inverse) const {
    const int G = (int)gates_.size();
    std::vector<char> live(G, 0), need(G, 0), has_live(n_, 0);
    for (int g = 0; g < G; ++g) {
      const PGate& x = gates_[g];
      const bool two = !is_1q(x.kind);
      const bool nd = has_live[x.q0] || (two && has_live[x.q1]);
      const bool grad = x.slot >= 0 && x.slot < n_theta_ && x.kind <= K_P;
      need[g] = nd;
      live[g] = grad || nd;
      if (live[g]) {
        has_live[x.q0] = 1;
        if (two) has_live[x.q1] = 1;
      }
    }
    if (need_inverse) *need_inverse = need;
    return live;
  }

  int n_, R_, rb_, k_, tb_, coal_, n_theta_;
  std::vector<PGate> gates_;
  std::vector<int> readout_;

  // demand: tile bit that must be in registers for op (or -1)
  int reg_demand(const PGate& g, const std::vector<int>& q2t) const {
    if (is_1q(g.kind) && !is_diag(g.kind)) return q2t[g.q0];
    if (g.kind == K_CX && q2t[g.q0] < 0) return q2t[g.q1];
    return -1;
  }

  void emit_pass(std::vector<int>& blob, const PassBuild& pb, int init, int fin, bool adjoint) {
    const int k = k_, rb = rb_;
    std::vector<int> q2t(n_, -1);
    for (int j = 0; j < k; ++j) q2t[pb.tileq[j]] = j;

    size_t desc = blob.size();
    blob.resize(desc + PF_SIZE, 0);
    blob[desc + PF_K] = k;
    blob[desc + PF_TB] = tb_;
    blob[desc + PF_INIT] = init;
    blob[desc + PF_FINAL] = fin;
    for (int j = 0; j < k; ++j) blob[desc + PF_TILEQ + j] = pb.tileq[j];
    int nn = 0;
    for (int q = 0; q < n_; ++q)
      if (q2t[q] < 0) blob[desc + PF_NONTILE + nn++] = q;
    blob[desc + PF_NNONTILE] = nn;
    blob[desc + PF_NREAD] = (int)readout_.size();

    // demand sequence for look-ahead
    std::vector<int> demand;
    for (int gi : pb.sched) demand.push_back(reg_demand(gates_[gi], q2t));

    // initial layout: thread bits 0..coal-1 <- tile bits 0..coal-1 (coalesced), registers <- the
    // first rb distinct demanded tile bits not among those, remaining thread bits <- the rest
    std::vector<int> want;
    for (int d : demand)
      if (d >= coal_ && std::find(want.begin(), want.end(), d) == want.end() && (int)want.size() < rb)
        want.push_back(d);
    for (int j = k - 1; j >= coal_ && (int)want.size() < rb; --j)
      if (std::find(want.begin(), want.end(), j) == want.end()) want.push_back(j);
    std::vector<int> layout(k, -1);  // phys -> tile bit
    for (int r = 0; r < rb; ++r) layout[r] = want[r];
    {
      int p = rb;
      for (int j = 0; j < k; ++j)
        if (std::find(want.begin(), want.end(), j) == want.end()) layout[p++] = j;
    }
    std::vector<int> layouts_words;  // appended after ops
    std::vector<std::vector<int>> layout_list{layout};
    std::vector<std::vector<int>> map_list;

    // pending linear map rows over tile bits
    std::vector<uint32_t> M(k);
    for (int j = 0; j < k; ++j) M[j] = 1u << j;
    bool pending = false;
    auto touches = [&](int t) {
      if (t < 0 || !pending) return false;
      if (M[t] != (1u << t)) return true;
      for (int j = 0; j < k; ++j)
        if (j != t && (M[j] >> t) & 1u) return true;
      return false;
    };
    auto t2p = [&](const std::vector<int>& lay) {
      std::vector<int> inv(k, -1);
      for (int p = 0; p < k; ++p) inv[lay[p]] = p;
      return inv;
    };
    std::vector<int> inv = t2p(layout);
    auto phys_of_q = [&](int q) { return q2t[q] >= 0 ? inv[q2t[q]] : PHYS_NONTILE + q; };

    struct Op { int code, a, b, c; };
    std::vector<Op> ops;
    // remap to a layout whose registers hold `regs` (plus pending map flush)
    auto remap_to_regs = [&](std::vector<int> regs) {
      std::vector<int> cur(layout.begin(), layout.begin() + rb);
      std::vector<int> nl = layout;
      // keep registers that stay
      std::vector<int> incoming;
      for (int t : regs)
        if (std::find(cur.begin(), cur.end(), t) == cur.end()) incoming.push_back(t);
      std::vector<int> outgoing;
      for (int r = 0; r < rb; ++r)
        if (std::find(regs.begin(), regs.end(), cur[r]) == regs.end()) outgoing.push_back(r);
      for (size_t i = 0; i < incoming.size() && i < outgoing.size(); ++i) {
        int rpos = outgoing[i];
        int tpos = inv[incoming[i]];
        std::swap(nl[rpos], nl[tpos]);
        inv[nl[rpos]] = rpos;
        inv[nl[tpos]] = tpos;
      }
      int map_idx = -1;
      if (pending) {
        map_list.push_back(std::vector<int>(M.begin(), M.end()));
        map_idx = (int)map_list.size() - 1;
        for (int j = 0; j < k; ++j) M[j] = 1u << j;
        pending = false;
      }
      layout = nl;
      inv = t2p(layout);
      layout_list.push_back(layout);
      ops.push_back({OP_REMAP, (int)layout_list.size() - 1, map_idx, 0});
    };
    auto lookahead_regs = [&](size_t from, int must) {
      std::vector<int> regs;
      if (must >= 0) regs.push_back(must);
      for (size_t i = from; i < demand.size() && (int)regs.size() < rb; ++i)
        if (demand[i] >= 0 && std::find(regs.begin(), regs.end(), demand[i]) == regs.end())
          regs.push_back(demand[i]);
      for (int r = 0; r < rb && (int)regs.size() < rb; ++r)
        if (std::find(regs.begin(), regs.end(), layout[r]) == regs.end()) regs.push_back(layout[r]);
      return regs;
    };

    for (size_t i = 0; i < pb.sched.size(); ++i) {
      int gi = pb.sched[i];
      const PGate& g = gates_[gi];
      int t0 = q2t[g.q0];
      if (is_1q(g.kind) && !is_diag(g.kind)) {
        if (touches(t0) || inv[t0] >= rb) remap_to_regs(lookahead_regs(i, t0));
        ops.push_back({OP_U1, inv[t0], 0, gi});
      } else if (is_1q(g.kind)) {  // diagonal 1q
        if (touches(t0)) remap_to_regs(lookahead_regs(i, -1));
        ops.push_back({OP_D1, phys_of_q(g.q0), 0, gi});
      } else if (g.kind == K_CX) {
        int tc = t0, tt = q2t[g.q1];
        if (tc >= 0) {
          bool in_reg = inv[tt] < rb;
          if (in_reg && !touches(tt) && !touches(tc)) {
            ops.push_back({OP_CX, inv[tc], inv[tt], gi});
          } else {  // fold into the pending GF(2) map: new bit tt ^= bit tc
            M[tt] ^= M[tc];
            pending = true;
          }
        } else {
          if (touches(tt) || inv[tt] >= rb) remap_to_regs(lookahead_regs(i, tt));
          ops.push_back({OP_CX, PHYS_NONTILE + g.q0, inv[tt], gi});
        }
      } else if (g.kind == K_CZ) {
        int tb1 = q2t[g.q1];
        if (touches(t0) || touches(tb1)) remap_to_regs(lookahead_regs(i, -1));
        ops.push_back({OP_CZ, phys_of_q(g.q0), phys_of_q(g.q1), gi});
      } else {
        throw std::invalid_argument("unsupported gate kind in planner: " + std::to_string(g.kind));
      }
    }
    // end of pass: flush pending map; restore coalesced thread bits for the store
    bool need_coal = false;
    if (fin & FIN_STORE)
      for (int j = 0; j < coal_; ++j)
        if (layout[rb + j] != j) need_coal = true;
    if (pending || need_coal) {
      std::vector<int> regs;
      if (need_coal) {
        // registers: current registers that are not coalescing bits, then highest free tile bits
        for (int r = 0; r < rb; ++r)
          if (layout[r] >= coal_) regs.push_back(layout[r]);
        for (int j = k - 1; j >= coal_ && (int)regs.size() < rb; --j)
          if (std::find(regs.begin(), regs.end(), j) == regs.end()) regs.push_back(j);
      } else {
        regs.assign(layout.begin(), layout.begin() + rb);
      }
      remap_to_regs(regs);
      if (need_coal) {
        // put coalescing tile bits on thread bits 0..coal-1 (permute thread bits only)
        std::vector<int> nl = layout;
        std::vector<int> others;
        for (int p = rb; p < k; ++p)
          if (nl[p] >= coal_) others.push_back(nl[p]);
        for (int j = 0; j < coal_; ++j) nl[rb + j] = j;
        for (size_t i = 0; i < others.size(); ++i) nl[rb + coal_ + i] = others[i];
        layout_list.back() = nl;
        layout = nl;
        inv = t2p(layout);
      }
    }

    // ---- lower U1/D1 on register bits into fused G1 groups, D1 elsewhere into D1T ----
    std::vector<Op> out;
    std::vector<std::vector<int>> glists;
    std::vector<int> open(rb, -1);   // open group (index into out) per register bit
    auto close_bit = [&](int phys) {
      if (phys >= 0 && phys < rb) open[phys] = -1;
    };
    for (const Op& o : ops) {
      if (o.code == OP_U1 || (o.code == OP_D1 && o.a < rb)) {
        int p = o.a;
        if (open[p] >= 0 && (int)glists[out[open[p]].c].size() < MAX_GROUP) {
          glists[out[open[p]].c].push_back(o.c);
        } else {
          glists.push_back({o.c});
          out.push_back({OP_G1, p, 0, (int)glists.size() - 1});
          open[p] = (int)out.size() - 1;
        }
      } else if (o.code == OP_D1) {
        out.push_back({OP_D1T, o.a, 0, o.c});
      } else if (o.code == OP_CX) {
        close_bit(o.a);
        close_bit(o.b);
        out.push_back(o);
      } else if (o.code == OP_CZ) {
        close_bit(o.a);
        close_bit(o.b);
        out.push_back(o);
      } else {  // REMAP
        for (int p = 0; p < rb; ++p) open[p] = -1;
        out.push_back(o);
      }
    }

    // ---- serialise ops, group lists, remap tables, layouts ----
    const int R = R_;
    auto swz = [&](uint32_t s) -> uint32_t {   // must equal the kernel-side LDS slot swizzle
      return k >= 10 ? (s ^ ((s >> 5) & 31u)) : (k >= 6 ? (s ^ ((s >> 5) & 15u)) : s);
    };
    auto apply_map = [&](uint32_t x, const std::vector<int>& rows) {
      uint32_t y = 0;
      for (int j = 0; j < k; ++j) y |= (uint32_t)(__builtin_popcount(x & (uint32_t)rows[j]) & 1) << j;
      return y;
    };
    auto treg = [&](const std::vector<int>& lay, int r) {
      uint32_t t = 0;
      for (int p = 0; p < rb; ++p)
        if ((r >> p) & 1) t |= 1u << lay[p];
      return t;
    };
    blob[desc + PF_NOPS] = (int)out.size();
    blob[desc + PF_OPS] = (int)blob.size();
    size_t ops_at = blob.size();
    blob.resize(ops_at + out.size() * OP_WORDS, 0);
    std::vector<int> lay_off(layout_list.size());
    for (size_t l = 0; l < layout_list.size(); ++l) {
      lay_off[l] = (int)blob.size();
      for (int p = 0; p < k; ++p) blob.push_back(layout_list[l][p]);
    }
    std::vector<int> glist_off(glists.size());
    for (size_t g = 0; g < glists.size(); ++g) {
      glist_off[g] = (int)blob.size();
      for (int gi : glists[g]) blob.push_back(gi);
    }
    int cur = 0;   // current layout index while walking the ops
    for (size_t i = 0; i < out.size(); ++i) {
      Op o = out[i];
      if (o.code == OP_G1) {
        o.b = (int)glists[o.c].size();
        o.c = glist_off[o.c];
      } else if (o.code == OP_REMAP) {
        const std::vector<int>& ol = layout_list[cur];
        const std::vector<int>& nl = layout_list[o.a];
        std::vector<int> ident(k);
        for (int j = 0; j < k; ++j) ident[j] = 1 << j;
        const std::vector<int>& rows = o.b >= 0 ? map_list[o.b] : ident;
        int tab = (int)blob.size();
        for (int r = 0; r < R; ++r) blob.push_back((int)swz(apply_map(treg(ol, r), rows)));
        for (int j = 0; j < tb_; ++j) blob.push_back((int)swz(apply_map(1u << ol[rb + j], rows)));
        for (int r = 0; r < R; ++r) blob.push_back((int)swz(treg(nl, r)));
        for (int j = 0; j < tb_; ++j) blob.push_back((int)swz(1u << nl[rb + j]));
        cur = o.a;
        o.b = lay_off[o.a];
        o.a = tab;
      }
      blob[ops_at + i * OP_WORDS + 0] = o.code;
      blob[ops_at + i * OP_WORDS + 1] = o.a;
      blob[ops_at + i * OP_WORDS + 2] = o.b;
      blob[ops_at + i * OP_WORDS + 3] = o.c;
    }
    blob[desc + PF_LAYOUT0] = lay_off[0];
    blob[desc + PF_FINAL_LAYOUT] = lay_off.back();
    // global amplitude offsets of registers / thread bits for the load and store layouts
    auto gq = [&](const std::vector<int>& lay, int p) { return pb.tileq[lay[p]]; };
    const std::vector<int>& L0 = layout_list[0];
    const std::vector<int>& LF = layout_list.back();
    for (int p = 0; p < k; ++p) blob[desc + PF_Q0 + p] = gq(L0, p);
    for (int r = 0; r < R; ++r) {
      uint32_t g0 = 0, gf = 0;
      for (int p = 0; p < rb; ++p)
        if ((r >> p) & 1) g0 |= 1u << gq(L0, p), gf |= 1u << gq(LF, p);
      blob[desc + PF_GREG0 + r] = (int)g0;
      blob[desc + PF_GREGF + r] = (int)gf;
    }
    for (int j = 0; j < tb_; ++j) {
      blob[desc + PF_GTHR0 + j] = 1 << gq(L0, rb + j);
      blob[desc + PF_GTHRF + j] = 1 << gq(LF, rb + j);
    }
    // readout phys bits: final layout (forward readout) and initial layout (adjoint lambda)
    std::vector<int> inv0 = t2p(layout_list[0]);
    std::vector<int> invf = t2p(layout_list.back());
    for (size_t c = 0; c < readout_.size(); ++c) {
      int q = readout_[c];
      int t = q2t[q];
      blob[desc + PF_READ_PHYS + c] = t >= 0 ? invf[t] : PHYS_NONTILE + q;
      blob[desc + PF_LAM_PHYS + c] = t >= 0 ? inv0[t] : PHYS_NONTILE + q;
    }
    int ngrad = 0;
    if (adjoint)
      for (int gi : pb.sched)
        if (gates_[gi].slot >= 0 && gates_[gi].slot < n_theta_ &&
            (gates_[gi].kind <= K_P))
          ++ngrad;
    blob[desc + PF_NGRAD] = ngrad;
  }
};

std::vector<int> plan_circuit(int n, int R, int kmax, const std::vector<int>& ops_i,
                              const std::vector<float>& coef, const std::vector<int>& readout,
                              int n_theta, int mode, int final_flags) {
  size_t G = ops_i.size() / 4;
  std::vector<PGate> gates(G);
  for (size_t g = 0; g < G; ++g)
    gates[g] = {ops_i[4 * g], ops_i[4 * g + 1], ops_i[4 * g + 2], ops_i[4 * g + 3], coef[2 * g],
                coef[2 * g + 1]};
  Planner p(n, R, kmax, gates, readout, n_theta);
  return p.build(mode, final_flags);
}

}  // namespace qfx
