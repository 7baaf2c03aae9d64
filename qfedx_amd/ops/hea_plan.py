"""Pass planner for the MFMA statevector engine of the hardware-efficient VQC (``models/vqc.py``).

The flagship circuit (ROADMAP.md:20-23, 125-128) is

    RY(x_q) feature map -> L x [ RX(theta_lq) RZ(phi_lq) on every qubit ; CNOT chain q -> q+1 ] -> <Z_c>

and this module turns it into a short sequence of LDS-tile passes whose work is dense 16 x 16 complex
GEMMs (MFMA, ``csrc/hea_mfma.hip``) instead of per-gate VALU sweeps:

* **Frames instead of permutations.**  A CNOT chain maps basis index y -> P y with P the prefix-XOR
  matrix over GF(2).  Nothing is moved: after k chains memory index y holds logical index z = P^k y,
  so a rotation on logical qubit q pairs memory indices y and y ^ P^-k e_q (a 1..k+1-bit mask) and its
  logical bit is parity(y & row_q(P^k)).  The readout <Z_c> after the last chain is the diagonal sign
  (-1)^parity(y & row_c(P^L)).
* **Layer 1 is closed form.**  RZ RX RY(x)|0> on every qubit is a product state, generated directly
  into the tile (no gate pass); its gradients come from 2 x 2 cross matrices.
* **4-qubit groups.**  Rotations of one layer commute, so the qubits of a layer are grouped by four;
  each group is one 16 x 16 complex unitary (tensor product of RZ.RX) acting on a 4-dim GF(2)
  subspace of the tile: Y[m', col] = sum_m U[m', m] X[m, col] - an MFMA GEMM over columns = cosets.
* **Staircase passes.**  A pass loads 2^t amplitudes (t = 14: fp16 (re, im) = 64 KB LDS, two states
  for the adjoint = 128 KB) spanning memory bits [0, c) u [lo, hi) and applies every group whose
  memory support lies in the tile and whose earlier-layer dependencies are done.  16 qubits x 3 layers
  needs 2 passes.
* **Adjoint.**  The forward stores every pass output (fp16); the reverse of pass j loads pass j's output
  and lambda and walks back: gradient cross matrix N = sum_col psi lambda^H per group (MFMA), then U^H
  on lambda and psi (no forward recompute).
  A layer-1 qubit's 2 x 2 cross matrix is measured in the first pass whose tile holds its bit (every
  earlier pass avoids that bit, and unitaries on other bits preserve the partial inner product).

Everything here is host-side planning (runs once per circuit shape).  ``emulate`` executes a plan
tile by tile with exactly the kernel's addressing tables in float64 numpy: it is the oracle the CPU
tests hold against a dense simulation, and the HIP kernel is tested against both.
"""
from __future__ import annotations

import copy
import os
from dataclasses import dataclass, field

import numpy as np

GROUP = 4                  # qubits per fused group (16-dim complex unitary -> K = 32 real MFMA)
TILE_BITS = 14             # 2^14 fp16 complex amplitudes = 64 KB of LDS per state
MIN_CONTIG = 5             # contiguous low bits in a strided tile (32 amplitudes = 128 B)

# op codes (kept in sync with csrc/hea_mfma.hip)
OP_APPLY, OP_GRAD_L1, OP_OBS, OP_READOUT, OP_BACK = 1, 5, 6, 7, 8
# chained pairs of two commuting 4-qubit groups X, Y of one layer on the 256-amplitude cosets of span(X, Y): one LDS
# read and write of the coset per pair, one op barrier (see pair_table)
OP_APPLY2, OP_BACK2, OP_GRAD2 = 2, 3, 4
PAIR_CODES = (OP_APPLY2, OP_BACK2, OP_GRAD2)
OP_WORDS = 128
W_CODE, W_SLOT, W_NREAL, W_FLAGS, W_RFULL, W_RT, W_TH, W_PH, W_OFF, W_BL, W_BH = 0, 1, 2, 3, 4, 8, 12, 16, 20, 36, 68
# pair records: the second group's rows in the W_RT words, and
W_RFULL2, W_GIDX2, W_SLOT2, W_NREAL2, W_OFF2, W_TH2, W_PH2 = 8, 101, 102, 103, 104, 120, 124
F_BACK_PSI = 1             # OP_BACK also un-applies the group on psi (still needed further back), in the transposed
                           # form (group_back_t): its cross matrix is taken at the op INPUT
W_GIDX = 100               # gradient ops: global index of the op's partial-trace record in the slab
MAX_CLASSES = 8
BANK_BITS = 5              # ds_read_b32 / ds_write_b32: bank = dword address % 32 per 32-lane half


def parity(x: int) -> int:
    return bin(x).count("1") & 1


def frame_vec(q: int, k: int, n: int) -> int:
    """Memory mask P^-k e_q that a rotation on logical qubit q pairs after k CNOT chains."""
    v = 1 << q
    full = (1 << n) - 1
    for _ in range(k):
        v = (v ^ (v << 1)) & full
    return v


def frame_rows(k: int, n: int) -> list:
    """Row masks of P^k: logical bit q of memory index y is parity(y & R[q])."""
    R = [1 << q for q in range(n)]
    for _ in range(k):
        acc, new = 0, []
        for q in range(n):
            acc ^= R[q]
            new.append(acc)
        R = new
    return R


@dataclass
class Group:
    layer: int                 # 1 = closed-form layer (gradient only), >= 2 rotation layer
    qubits: list               # logical qubits (<= 4)
    frame: int                 # CNOT chains before this layer
    slot: int = -1             # unitary fragment slot (rotation groups)

    def vecs(self, n):
        return [frame_vec(q, self.frame, n) for q in self.qubits]

    def support(self, n):
        s = 0
        for v in self.vecs(n):
            s |= v
        return s


@dataclass
class Pass:
    c: int
    lo: int
    hi: int
    groups: list = field(default_factory=list)      # rotation groups, forward order
    l1: list = field(default_factory=list)          # layer-1 gradient groups (measured at the pass input)
    H: list = field(default_factory=lambda: [0] * BANK_BITS)   # LDS swizzle rows (see sigma)
    cols: dict = field(default_factory=dict)        # per group: the 4 non-pivot bits that feed MFMA columns

    @property
    def bits(self) -> list:
        return list(range(self.c)) + list(range(self.lo, self.hi))

    @property
    def t(self) -> int:
        return self.c + self.hi - self.lo

    def mask(self) -> int:
        m = 0
        for b in self.bits:
            m |= 1 << b
        return m

    def to_tile(self, mem_mask: int) -> int:
        out = 0
        for i, b in enumerate(self.bits):
            if (mem_mask >> b) & 1:
                out |= 1 << i
        return out

    def fixed(self, tile_id: int, n: int) -> int:
        """Memory bits that are constant over tile ``tile_id`` (bits outside the tile)."""
        w1 = self.lo - self.c
        f1 = tile_id & ((1 << w1) - 1)
        f2 = tile_id >> w1
        return (f1 << self.c) | (f2 << self.hi)

    def mem_index(self, tau: np.ndarray, tile_id: int, n: int) -> np.ndarray:
        lo_part = tau & ((1 << self.c) - 1)
        hi_part = tau >> self.c
        return lo_part | (hi_part << self.lo) | self.fixed(tile_id, n)


@dataclass
class HEAPlan:
    n: int
    L: int
    C: int
    readout: list
    chain: bool
    feature: str
    t: int
    passes: list
    n_slots: int                 # rotation groups (unitary fragments per client)

    @property
    def n_theta(self) -> int:
        return 2 * self.n * self.L

    def layer_frame(self, layer: int) -> int:
        return (layer - 1) if self.chain else 0

    @property
    def obs_masks(self) -> list:
        R = frame_rows(self.L if self.chain else 0, self.n)
        return [R[q] for q in self.readout]

    def theta_slot(self, layer: int, q: int) -> int:
        return 2 * ((layer - 1) * self.n + q)


def eligible(spec) -> bool:
    """Circuits this engine covers: angle feature map, RX/RZ layers, chain (or no) entangler, no noise."""
    return (not spec.amplitude and not spec.noisy and spec.entangler in ("chain", "none")
            and spec.feature_map.lower() in ("rx", "ry", "rz") and spec.n_qubits >= 8
            and spec.n_qubits <= 30 and spec.n_classes <= MAX_CLASSES)


_PLAN_CACHE: dict = {}


def build_plan(n: int, L: int, readout, chain: bool = True, feature: str = "ry",
               tile_bits: int = TILE_BITS, swizzle: bool = True, trim=None) -> HEAPlan:
    """Plan the passes.  ``trim=None`` builds both the greedy plan (every ready rotation joins the current
    pass) and the trimmed plan (a non-final pass defers each layer's ragged tail so its groups are full
    4-qubit unitaries) and keeps the one with fewer passes, then fewer group ops: for 16q x 3L the trimmed
    plan runs 8 group ops instead of 10 in the same two passes."""
    key = (n, L, tuple(readout), chain, feature, tile_bits, swizzle)
    if trim is None and key in _PLAN_CACHE:          # the candidate search runs once per circuit shape
        return copy.deepcopy(_PLAN_CACHE[key])
    if trim is None:
        # candidates: no trimming, trimming everywhere, and per-layer trimming of the first (product-state)
        # pass with the later passes greedy or trimmed; ties keep the earlier candidate
        opts = [False, True]
        for m in range(1, 1 << max(L - 1, 0)):
            opts += [(m << 2,), (m << 2, -1)]
        cands = []
        for tr in opts:
            try:
                cands.append(build_plan(n, L, readout, chain, feature, tile_bits, False, tr))
            except RuntimeError:
                continue
        best = min(cands, key=lambda pl: (len(pl.passes), sum(len(p.groups) for p in pl.passes)))
        if swizzle:
            for j, p in enumerate(best.passes):
                layout_pass(best, p, seed=j)
        _PLAN_CACHE[key] = copy.deepcopy(best)
        return best
    t = min(tile_bits, n)
    if t < GROUP + 4:
        raise ValueError("the MFMA engine needs at least 8 tile qubits (16 columns per MFMA block)")
    frame = (lambda layer: layer - 1) if chain else (lambda layer: 0)
    sup = {}
    for layer in range(2, L + 1):
        for q in range(n):
            sup[(layer, q)] = frame_vec(q, frame(layer), n)
    preds = {}
    for (layer, q), s in sup.items():
        preds[(layer, q)] = [(layer - 1, p) for p in range(n) if layer > 2 and (sup[(layer - 1, p)] & s)]
    remaining = sorted(sup, key=lambda o: (o[0], o[1]))
    done = set()
    passes = []
    while True:
        if not passes:
            p = Pass(t, t, t) if n > t else Pass(n, n, n)
        else:
            mc = min(MIN_CONTIG, max(2, t - 6))
            low = lambda o: min(b for b in range(n) if (sup[o] >> b) & 1)
            lo_all = min(low(o) for o in remaining)      # one pass for everything left, if it fits
            ready = [o for o in remaining if all(d in done for d in preds[o])]
            lo_min = lo_all if t - (n - lo_all) >= mc else min(low(o) for o in ready)
            w = n - lo_min
            if t - w >= mc:
                p = Pass(t - w, lo_min, n)
            else:
                base = max(lo_min, mc)
                p = Pass(mc, base, min(n, base + t - mc))
        tm = p.mask()
        taken = []
        for o in remaining:
            if (sup[o] & ~tm) == 0 and all(d in done or d in taken for d in preds[o]):
                taken.append(o)
        if isinstance(trim, tuple):         # per-pass layer masks (bit l = trim layer l; -1 = all layers)
            j = len(passes)
            layers = trim[j] if j < len(trim) else (-1 if trim[-1] == -1 else 0)
        else:
            layers = -1 if trim else 0
        if layers and len(taken) < len(remaining):
            taken = _trim_ragged(taken, preds, layers)
        if not taken and remaining:
            raise RuntimeError(f"pass planner stuck at {len(passes)} passes (n={n}, L={L}, t={t})")
        for o in taken:
            done.add(o)
        remaining = [o for o in remaining if o not in done]
        by_layer = {}
        for (layer, q) in taken:
            by_layer.setdefault(layer, []).append(q)
        for layer in sorted(by_layer):
            qs = sorted(by_layer[layer])
            for i in range(0, len(qs), GROUP):
                p.groups.append(Group(layer, qs[i:i + GROUP], frame(layer)))
        passes.append(p)
        if not remaining:
            break
        if len(passes) > 16:
            raise RuntimeError("pass planner did not converge")
    # every qubit's bit must sit in some tile (layer-1 gradients): add group-free passes for the rest
    covered = 0
    for p in passes:
        covered |= p.mask()
    while covered != (1 << n) - 1:
        top = (1 << n) - 1 & ~covered
        lo = max(top.bit_length() - (t - MIN_CONTIG), min(b for b in range(n) if (top >> b) & 1))
        lo = max(lo, MIN_CONTIG)
        p = Pass(t - (min(n, lo + t - MIN_CONTIG) - lo), lo, min(n, lo + t - MIN_CONTIG))
        passes.append(p)
        covered |= p.mask()
    # layer-1 gradient groups: first pass whose tile holds the qubit's bit
    owner = {}
    for q in range(n):
        for j, p in enumerate(passes):
            if (p.mask() >> q) & 1:
                owner[q] = j
                break
    for j, p in enumerate(passes):
        qs = [q for q in range(n) if owner[q] == j]
        for i in range(0, len(qs), GROUP):
            p.l1.append(Group(1, qs[i:i + GROUP], 0))
    slot = 0
    for p in passes:
        for g in p.groups:
            g.slot = slot
            slot += 1
    plan = HEAPlan(n, L, len(readout), list(readout), chain, feature, t, passes, slot)
    if swizzle:
        for j, p in enumerate(passes):
            layout_pass(plan, p, seed=j)
    return plan


def _trim_ragged(taken: list, preds: dict, layers: int = -1) -> list:
    """Drop the highest rotations of each layer in the bitmask ``layers`` until its count is a multiple of
    GROUP, together with every taken rotation that depends on a dropped one.  Falls back to ``taken`` if
    nothing would be left."""
    keep = list(taken)
    while True:
        by_layer = {}
        for o in keep:
            by_layer.setdefault(o[0], []).append(o)
        drop = set()
        for layer, os_ in by_layer.items():
            r = len(os_) % GROUP
            if r and (layers >> layer) & 1:
                drop.update(sorted(os_, key=lambda o: o[1])[-r:])
        if not drop:
            return keep if keep else list(taken)
        changed = True
        while changed:
            changed = False
            for o in keep:
                if o not in drop and any(d in drop for d in preds[o]):
                    drop.add(o)
                    changed = True
        keep = [o for o in keep if o not in drop]


# ---------------------------------------------------------------------------------------- op tables
def _neutral_pads(vt: list, rt: list, t: int, need: int) -> list:
    """``need`` tile vectors independent of ``vt`` whose logical parity against every ``rt`` mask is 0."""
    def sig(v):
        return tuple(parity(v & r) for r in rt)
    basis = []          # GF(2) elimination of vt + chosen pads

    def independent(v):
        x = v
        for b in basis:
            x = min(x, x ^ b)
        return x != 0

    def add(v):
        x = v
        for b in basis:
            x = min(x, x ^ b)
        basis.append(x)
        basis.sort(reverse=True)

    for v in vt:
        add(v)
    pads = []
    cands = [1 << i for i in range(t)]
    by_sig = {}
    for e in cands:
        by_sig.setdefault(sig(e), []).append(e)
    pool = list(by_sig.get(tuple(0 for _ in rt), []))
    for s, es in by_sig.items():
        if any(s):
            pool += [es[0] ^ e for e in es[1:]]
    for v in pool:
        if len(pads) == need:
            break
        if independent(v):
            add(v)
            pads.append(v)
    if len(pads) < need:
        raise RuntimeError("could not pad a group to 4 qubits inside the tile")
    return pads


def _pivots(vecs: list) -> list:
    """Distinct pivot bit per vector after GF(2) elimination (rows stay the original span)."""
    rows = []
    piv = []
    for v in vecs:
        x = v
        for pb, r in zip(piv, rows):
            if (x >> pb) & 1:
                x ^= r
        if x == 0:
            raise RuntimeError("dependent group vectors")
        pb = x.bit_length() - 1
        # keep earlier rows reduced w.r.t. the new pivot
        for i in range(len(rows)):
            if (rows[i] >> pb) & 1:
                rows[i] ^= x
        rows.append(x)
        piv.append(pb)
    return piv


# ---------------------------------------------------------------------------------------- LDS layout
# The tile lives in LDS at dword sigma(tau) = tau ^ h(tau >> 5), h linear (rows H), an involution that
# only rewrites the 5 bank bits.  It is linear over GF(2), so every XOR-composed table entry is stored
# already swizzled.  Per pass H and per group the 4 non-pivot bits that become the 16 MFMA columns of
# a block are searched so that the 32 lanes of each half-wave hit 32 distinct banks in all three
# access patterns of a group op: apply reads (columns x m-bit 2), apply writes (columns x m-bit 1) and
# cross-matrix reads (m bits 0..3 x column bit 2), and so that the adjoint's b64 pair stores (16-lane
# groups) hit distinct bank pairs.
def _hmul(H, x: int) -> int:
    r = 0
    for b, row in enumerate(H):
        r |= parity(row & x) << b
    return r


def sigma(H, tau: int) -> int:
    return tau ^ _hmul(H, tau >> BANK_BITS)


def _bank(H, v: int) -> int:
    return (v & ((1 << BANK_BITS) - 1)) ^ _hmul(H, v >> BANK_BITS)


def _rank(vals) -> int:
    basis = []
    for v in vals:
        x = v
        for b in basis:
            x = min(x, x ^ b)
        if x:
            basis.append(x)
            basis.sort(reverse=True)
    return len(basis)


def _group_geom(plan: HEAPlan, p: Pass, g: Group):
    """Tile-local group vectors (padded to 4), row masks, non-pivot bits and their column directions."""
    n, t = plan.n, p.t
    R = frame_rows(g.frame, n)
    vt = [p.to_tile(v) for v in g.vecs(n)]
    for v, vm in zip(vt, g.vecs(n)):
        if p.to_tile(vm) != v or (vm & ~p.mask()):
            raise RuntimeError("group support leaves the tile")
    rfull = [R[q] for q in g.qubits]
    rt = [p.to_tile(r) for r in rfull]
    allv = vt + _neutral_pads(vt, rt, t, GROUP - len(g.qubits))
    off = [0] * 16
    for m in range(16):
        for j in range(GROUP):
            if (m >> j) & 1:
                off[m] ^= allv[j]
    piv = set(_pivots(allv))
    nonpiv = [b for b in range(t) if b not in piv]

    def bits(y):
        b = 0
        for j in range(len(g.qubits)):
            b |= parity(y & rt[j]) << j
        return b

    dirs = {b: (1 << b) ^ off[bits(1 << b)] for b in nonpiv}
    return allv, rfull, rt, off, nonpiv, bits, dirs


FULL_SCORE = 4


def _best_cols(H, allv, dirs, stores: bool = True):
    """(score, (c0, c1, c2, c3)): column bits maximising conflict-free access patterns (FULL_SCORE = all):
    apply reads and writes (a lane writes the amplitudes it read: columns x m-bit 2 per 32-lane half),
    cross-matrix reads, the ds_write_b64 pair stores of the U-as-A form, whose lane groups are 16 contiguous
    lanes (one amplitude, 16 columns) with bank (byte / 4) mod 32, i.e. the 16 columns need distinct swizzled
    pair indices mod 16, and the transposed BACK's pair stores (16 amplitudes of one column: the group vectors'
    pair indices mod 16 independent; a property of H alone; ``stores=False`` for the layer-1 gradient groups, whose
    ops only read)."""
    bv = [_bank(H, v) for v in allv]
    bd = {b: _bank(H, d) for b, d in dirs.items()}
    best = (-1, None)
    import itertools
    st = int(_rank([x & 15 for x in bv]) == 4) if stores else 1
    for combo in itertools.combinations(sorted(dirs), 4):
        cb = [bd[b] for b in combo]
        sa = int(_rank(cb + [bv[2]]) == 5)
        sw = st
        s16 = int(_rank([x & 15 for x in cb]) == 4)
        for c2 in combo:
            sg = int(_rank(bv + [bd[c2]]) == 5)
            sc = sa + sw + sg + s16
            if sc > best[0]:
                rest = [b for b in combo if b != c2]
                best = (sc, (rest[0], rest[1], c2, rest[2]))
                if sc == FULL_SCORE:
                    return best
    return best


def _pair_score(H, vx: list, vy: list, rotation: bool) -> int:
    """Conflict-free access patterns of a chained pair op (X, Y) under swizzle H.  A 32-lane half reads / writes
    (x = 4 g4 + j, y = cl) or (x = cl, y = 4 g4 + j): 32 banks when X's bit-2 vector and Y's four vectors (or the
    reverse) are independent in the 5 bank bits.  The forward pair (X, Y) reads the first pattern and writes the
    second; the adjoint pair runs (Y, X) and reads and writes the second pattern, its ds_write2_b32 pairs in 16-lane
    groups (X's four vectors independent in bank bits mod 16); a cross-only pair reads both patterns."""
    bx, by = [_bank(H, v) for v in vx], [_bank(H, v) for v in vy]
    a = int(_rank([bx[2]] + by) == 5)
    b = int(_rank([by[2]] + bx) == 5)
    if not rotation:
        return a + b
    return a + b + int(_rank([v & 15 for v in bx]) == 4)


def single_op_groups(plan: HEAPlan, p: Pass, mask: int) -> set:
    """(layer, qubits) of the pass' groups that run as single ops in some program under pair mask ``mask``
    (pass_programs): unpaired groups, both groups of a rotation pair when the forward or the adjoint splits it (the
    adjoint's last pair when psi is no longer needed), and layer-1 groups outside a cross pair."""
    out = set()
    units = _pairs(plan, p, p.groups, bool(mask & 3))
    for i, u in enumerate(units):
        split = len(u) == 1 or not (mask & 1) or not (mask & 2) or (i == 0 and not p.l1)
        if split:
            out |= {(g.layer, tuple(g.qubits)) for g in u}
    for u in _pairs(plan, p, p.l1, bool(mask & 4), cross=True):
        if len(u) == 1:
            out.add((u[0].layer, tuple(u[0].qubits)))
    return out


def layout_pass(plan: HEAPlan, p: Pass, seed: int = 0, tries: int = 256) -> None:
    """Pick the pass' LDS swizzle rows H and every group's column bits (bank-conflict search), scoring the chained
    pair ops the planner will form (``_pairs``) as well."""
    groups = p.groups + p.l1
    geoms = [_group_geom(plan, p, g) for g in groups]
    vec = {(g.layer, tuple(g.qubits)): geo[0] for g, geo in zip(groups, geoms)}
    mask = _pair_default()
    pairs = [(u, True) for u in _pairs(plan, p, p.groups, bool(mask & 3)) if len(u) == 2]
    pairs += [(u, False) for u in _pairs(plan, p, p.l1, bool(mask & 4), cross=True) if len(u) == 2]
    solo = single_op_groups(plan, p, mask)
    single = [(g.layer, tuple(g.qubits)) in solo for g in groups]
    full = FULL_SCORE * sum(single) + sum(3 if rot else 2 for _, rot in pairs)
    hb = max(p.t - BANK_BITS, 0)
    rng = np.random.default_rng(1234 + seed)
    best = None
    for i in range(tries):
        H = [0] * BANK_BITS if i == 0 else [int(x) for x in rng.integers(0, 1 << hb, BANK_BITS)] if hb else [0] * 5
        cols, score = [], 0
        for gi, (allv, _, _, _, _, _, dirs) in enumerate(geoms):
            sc, c = _best_cols(H, allv, dirs, gi < len(p.groups))
            cols.append(c)
            score += sc if single[gi] else 0
        for (g, h), rot in pairs:
            score += _pair_score(H, vec[(g.layer, tuple(g.qubits))], vec[(h.layer, tuple(h.qubits))], rot)
        if best is None or score > best[0]:
            best = (score, H, cols)
        if score == full:
            break
    p.H = best[1]
    p.cols = {(g.layer, tuple(g.qubits)): c for g, c in zip(groups, best[2])}
    p.layout_score = (best[0], full)


def group_table(plan: HEAPlan, p: Pass, g: Group, code: int, flags: int = 0) -> np.ndarray:
    """One op record: frame row masks, XOR offsets OFF[m], column bases and parameter slots.

    Column c's coset representative with logical group bits 0 is y'(c) ^ OFF[bits(y'(c)) ^ fp], y' the
    deposit of c into the non-pivot tile bits, bits() its logical group bits from the tile-local row
    masks and fp those of the tile's fixed memory bits.  Everything but OFF[fp] is tile independent,
    and deposit and parity are linear, so the table stores per 5-bit half of c the pre-XORed base
    BL[c & 31] / BH[c >> 5] = d ^ OFF[bits(d)]:  addr(c, m) = BL ^ BH ^ OFF[fp] ^ OFF[m]  (all swizzled).
    The first four deposit bits are the pass layout's column bits for this group (bank-conflict free)."""
    n, t = plan.n, p.t
    w = np.zeros(OP_WORDS, dtype=np.int64)
    w[W_CODE] = code
    w[W_SLOT] = g.slot
    w[W_FLAGS] = flags
    nreal = len(g.qubits)
    w[W_NREAL] = nreal
    allv, rfull, rt, off, nonpiv, bits, _ = _group_geom(plan, p, g)
    first = list(p.cols.get((g.layer, tuple(g.qubits))) or nonpiv[:4])
    order = first + [b for b in nonpiv if b not in first]
    assert len(order) == t - GROUP
    for j in range(GROUP):
        w[W_RFULL + j] = rfull[j] if j < nreal else 0
        w[W_RT + j] = rt[j] if j < nreal else 0
        w[W_TH + j] = plan.theta_slot(g.layer, g.qubits[j]) if j < nreal else -1
        w[W_PH + j] = plan.theta_slot(g.layer, g.qubits[j]) + 1 if j < nreal else -1
    for m in range(16):
        w[W_OFF + m] = sigma(p.H, off[m])
    for i in range(32):
        lo = hi = 0
        for j in range(5):
            if (i >> j) & 1:
                if j < len(order):
                    lo |= 1 << order[j]
                if 5 + j < len(order):
                    hi |= 1 << order[5 + j]
        w[W_BL + i] = sigma(p.H, lo ^ off[bits(lo)])
        w[W_BH + i] = sigma(p.H, hi ^ off[bits(hi)])
    return w


def pairable(plan: HEAPlan, p: Pass, gx: Group, gy: Group, cross: bool = False) -> bool:
    """Two rotation groups can run as one chained pair op: one layer (so one CNOT frame: each group's row masks
    annihilate the other's vectors and their 8 vectors are independent), 4 real qubits each, and at least one
    256-amplitude coset per... tile of 2^t >= 2^11 (8 cosets: one per wave of a forward workgroup at least).
    ``cross`` (layer-1 gradient pairs, OP_GRAD2: cross matrices only, no unitary): a group may be short - its padding
    vectors (``_neutral_pads``) act as more column coordinates, and only its real qubits get partial traces."""
    sizes_ok = (1 <= len(gx.qubits) <= GROUP and 1 <= len(gy.qubits) <= GROUP) if cross else \
        (len(gx.qubits) == GROUP and len(gy.qubits) == GROUP)
    return (gx.layer == gy.layer and gx.layer >= 1 and sizes_ok and p.t >= 11 and not set(gx.qubits) & set(gy.qubits))


def pair_table(plan: HEAPlan, p: Pass, gx: Group, gy: Group, code: int, flags: int = 0) -> np.ndarray:
    """Record of a chained pair op: group X runs first, then Y (X, Y commute).  A block is one coset of span(X, Y)
    in the tile, 256 amplitudes at  addr(x, y) = base ^ OFF_X[x] ^ OFF_Y[y] ^ fo  with x, y the two groups' logical
    coordinates (the OFF tables are linear, so the tile's fixed-bit offset is one word fo = OFF_X[fpX] ^ OFF_Y[fpY]).
    Block bases BL[blk & 31] ^ BH[blk >> 5] = d ^ OFF_X[bits_X(d)] ^ OFF_Y[bits_Y(d)] for a deposit d of the block
    index into the tile bits outside both groups' pivots (logical coordinates 0 in both groups).  The kernel chains
    the two 16 x 16 products in registers: X in the transposed MFMA form leaves each lane holding its x-amplitude of 4
    y-columns, which is exactly the operand layout of Y's product over y (csrc/hea_mfma.hip, group_pair)."""
    if not pairable(plan, p, gx, gy, cross=code == OP_GRAD2):
        raise ValueError("groups cannot be paired")
    n, t = plan.n, p.t
    w = np.zeros(OP_WORDS, dtype=np.int64)
    w[W_CODE] = code
    w[W_FLAGS] = flags
    w[W_NREAL], w[W_NREAL2] = len(gx.qubits), len(gy.qubits)
    geo = []
    for g, (wr, wth, wph, woff, wsl) in ((gx, (W_RFULL, W_TH, W_PH, W_OFF, W_SLOT)),
                                          (gy, (W_RFULL2, W_TH2, W_PH2, W_OFF2, W_SLOT2))):
        allv, rfull, rt, off, _, bits, _ = _group_geom(plan, p, g)
        geo.append((allv, off, bits))
        w[wsl] = g.slot
        w[wth:wth + GROUP] = -1                # (a short group's padding: no slots, row masks 0 - parity 0 always)
        w[wph:wph + GROUP] = -1
        for j in range(len(g.qubits)):
            w[wr + j] = rfull[j]
            w[wth + j] = plan.theta_slot(g.layer, g.qubits[j])
            w[wph + j] = plan.theta_slot(g.layer, g.qubits[j]) + 1
        for m in range(16):
            w[woff + m] = sigma(p.H, off[m])
    piv = set(_pivots(geo[0][0] + geo[1][0]))
    order = [b for b in range(t) if b not in piv]
    assert len(order) == t - 2 * GROUP
    (_, offx, bitsx), (_, offy, bitsy) = geo

    def rep(d):
        return d ^ offx[bitsx(d)] ^ offy[bitsy(d)]
    for i in range(32):
        lo = hi = 0
        for j in range(5):
            if (i >> j) & 1:
                if j < len(order):
                    lo |= 1 << order[j]
                if 5 + j < len(order):
                    hi |= 1 << order[5 + j]
        w[W_BL + i] = sigma(p.H, rep(lo))
        w[W_BH + i] = sigma(p.H, rep(hi))
    return w


def _pair_default() -> int:
    """Chained pair ops: QFEDX_HEA_PAIR bit mask of the kinds planned as pairs (1 APPLY2, 2 BACK2, 4 GRAD2; default 7,
    0 plans every group op alone: A/B)."""
    return int(os.environ.get("QFEDX_HEA_PAIR", "7"))


def obs_table(plan: HEAPlan, p: Pass, code: int) -> np.ndarray:
    w = np.zeros(OP_WORDS, dtype=np.int64)
    w[W_CODE] = code
    w[W_NREAL] = plan.C
    for c, m in enumerate(plan.obs_masks):
        w[W_RFULL + 2 * c] = m                  # 8 words: full masks (two words per class slot)
        ot = p.to_tile(m)                       # parity(sigma(w) & ot) = parity(w & ot')
        ht = 0
        for b in range(BANK_BITS):
            if (ot >> b) & 1:
                ht ^= p.H[b]
        w[W_OFF + c] = ot ^ (ht << BANK_BITS)
    return w


def _pairs(plan: HEAPlan, p: Pass, groups: list, pair: bool, cross: bool = False) -> list:
    """Greedy left-to-right grouping of consecutive pairable groups: [(g,), (g, h), ...]."""
    out, i = [], 0
    while i < len(groups):
        if pair and i + 1 < len(groups) and pairable(plan, p, groups[i], groups[i + 1], cross):
            out.append((groups[i], groups[i + 1]))
            i += 2
        else:
            out.append((groups[i],))
            i += 1
    return out


def pass_programs(plan: HEAPlan, meta: list | None = None, pair: bool | None = None):
    """Forward and adjoint op lists per pass: list of (Pass, fwd_ops [k, OP_WORDS], adj_ops).  ``meta``
    (optional list) receives one row per gradient (group) op: [tiles of its pass, nreal | inside << 4, theta slots x4,
    phi slots x4].  BACK ops that un-apply psi too run transposed (``group_back_t``): their cross matrix is taken at
    the op input (``inside``, hea_grad_reduce applies the input-side generators); a pass's last BACK op, when psi is
    no longer needed, un-applies lambda only and takes the cross matrix at its output.  ``pair`` (default on,
    QFEDX_HEA_PAIR): consecutive groups of one layer run as chained pair ops (``pair_table``) - the forward pairs
    (g_i, g_i+1) of the pass order, the adjoint the same pairs in reverse, and the layer-1 gradient groups in pairs
    - with the gradient records in the order of the unpaired program."""
    if pair is None:
        pair = _pair_default()
    pair = 7 if pair is True else (0 if pair is False else int(pair))
    out = []
    gidx = [0]
    gmeta = meta if meta is not None else []
    J = len(plan.passes)

    def meta_row(w, x: str):
        th, ph, nr = (W_TH, W_PH, W_NREAL) if x == "x" else (W_TH2, W_PH2, W_NREAL2)
        inside = 16 if (int(w[W_CODE]) in (OP_BACK, OP_BACK2) and int(w[W_FLAGS]) & F_BACK_PSI) else 0
        gmeta.append([1 << (plan.n - p.t), int(w[nr]) | inside] + [int(v) for v in w[th:th + 4]] +
                     [int(v) for v in w[ph:ph + 4]])
    for j, p in enumerate(plan.passes):
        units = _pairs(plan, p, p.groups, bool(pair & 3))
        fwd = []
        for u in units:
            if len(u) == 2 and pair & 1:
                fwd.append(pair_table(plan, p, u[0], u[1], OP_APPLY2))
            else:
                fwd += [group_table(plan, p, g, OP_APPLY) for g in u]
        if j == J - 1:
            fwd.append(obs_table(plan, p, OP_READOUT))
        # the adjoint of pass j starts from pass j's stored OUTPUT and walks back; a forward pair (g, h) un-applies h
        # first, then g
        adj = [obs_table(plan, p, OP_OBS)] if j == J - 1 else []
        for i, u in enumerate(reversed(units)):
            # gradient cross matrix + U^H on lambda (and on psi while it is still needed further back)
            psi_needed = i < len(units) - 1 or bool(p.l1)
            if len(u) == 2 and psi_needed and pair & 2:
                adj.append(pair_table(plan, p, u[1], u[0], OP_BACK2, F_BACK_PSI))
            elif len(u) == 2:                   # unpaired, or the pass's last pair without psi: two single ops
                adj.append(group_table(plan, p, u[1], OP_BACK, F_BACK_PSI))
                adj.append(group_table(plan, p, u[0], OP_BACK, F_BACK_PSI if psi_needed else 0))
            else:
                adj.append(group_table(plan, p, u[0], OP_BACK, F_BACK_PSI if psi_needed else 0))
        for u in _pairs(plan, p, p.l1, bool(pair & 4), cross=True):
            adj.append(group_table(plan, p, u[0], OP_GRAD_L1) if len(u) == 1 else
                       pair_table(plan, p, u[0], u[1], OP_GRAD2))
        for w in adj:
            code = int(w[W_CODE])
            if code in (OP_BACK, OP_GRAD_L1):
                w[W_GIDX] = gidx[0]
                meta_row(w, "x")
                gidx[0] += 1
            elif code in (OP_BACK2, OP_GRAD2):
                w[W_GIDX], w[W_GIDX2] = gidx[0], gidx[0] + 1
                meta_row(w, "x")
                meta_row(w, "y")
                gidx[0] += 2
        out.append((p, np.stack(fwd) if fwd else np.zeros((0, OP_WORDS), np.int64),
                    np.stack(adj) if adj else np.zeros((0, OP_WORDS), np.int64)))
    return out


# ---------------------------------------------------------------------------------------- numerics
def rot_u(theta, phi):
    """RZ(phi) RX(theta) as [..., 2, 2] complex."""
    c, s = np.cos(theta / 2), np.sin(theta / 2)
    em, ep = np.exp(-0.5j * phi), np.exp(0.5j * phi)
    u = np.empty(np.shape(theta) + (2, 2), dtype=np.complex128)
    u[..., 0, 0] = em * c
    u[..., 0, 1] = -1j * em * s
    u[..., 1, 0] = -1j * ep * s
    u[..., 1, 1] = ep * c
    return u


def feature_vec(x, basis: str):
    """F(x)|0> for the feature rotation."""
    a = np.asarray(x, dtype=np.float64) / 2
    v = np.zeros(np.shape(a) + (2,), dtype=np.complex128)
    b = basis.lower()
    if b == "rx":
        v[..., 0], v[..., 1] = np.cos(a), -1j * np.sin(a)
    elif b == "rz":
        v[..., 0] = np.exp(-1j * a)
    else:
        v[..., 0], v[..., 1] = np.cos(a), np.sin(a)
    return v


def group_unitary(theta: np.ndarray, nreal: int, th_slots, ph_slots) -> np.ndarray:
    """16 x 16 unitary U[m', m] = prod_j u_j[m'_j, m_j] (pads: identity) for one client's params."""
    U = np.ones((16, 16), dtype=np.complex128)
    mp = np.arange(16)[:, None]
    mm = np.arange(16)[None, :]
    for j in range(GROUP):
        bj_p, bj = (mp >> j) & 1, (mm >> j) & 1
        if j < nreal:
            u = rot_u(theta[th_slots[j]], theta[ph_slots[j]])
            U = U * u[bj_p, bj]
        else:
            U = U * (bj_p == bj)
    return U


def tile_fixed(p: Pass, n: int) -> np.ndarray:
    """Memory bits outside the tile of every tile id of pass ``p`` (the kernels' tile_fixed): [2^(n - t)] uint32."""
    tid = np.arange(1 << (n - p.t), dtype=np.uint64)
    w1 = p.lo - p.c
    return (((tid & ((1 << w1) - 1)) << p.c) | ((tid >> w1) << p.hi)).astype(np.uint32)


def fo_table(ops: np.ndarray, p: Pass, n: int) -> np.ndarray:
    """Per (tile, op) OFF base of a pass program: the op's OFF entry for the parities of the tile's fixed bits with
    its frame row masks (pair records: both groups', XORed).  [n_tiles, nops] int32, read by every workgroup in its
    prologue (one load per op instead of a dependent chain of record loads on one wave: round-5 stall table)."""
    fixed = tile_fixed(p, n)
    out = np.zeros((len(fixed), len(ops)), dtype=np.uint32)

    def fp(rows, k):
        v = np.zeros(len(fixed), dtype=np.uint32)
        for j in range(k):
            v |= ((np.bitwise_count(fixed & np.uint32(int(rows[j]) & 0xFFFFFFFF)) & 1).astype(np.uint32) << j)
        return v

    for o, w in enumerate(ops):
        code = int(w[W_CODE])
        if code in (OP_OBS, OP_READOUT):
            continue
        off = np.asarray(w[W_OFF:W_OFF + 16]).astype(np.uint32)
        fo = off[fp(w[W_RFULL:W_RFULL + 4], int(w[W_NREAL]))]
        if code in PAIR_CODES:
            fo = fo ^ np.asarray(w[W_OFF2:W_OFF2 + 16]).astype(np.uint32)[fp(w[W_RFULL2:W_RFULL2 + 4], GROUP)]
        out[:, o] = fo
    return out.view(np.int32)


def _addr(w, t, fixed):
    """[ncol, 16] tile addresses of (column, group coordinate m), computed as the kernel does."""
    col = np.arange(1 << (t - GROUP))
    fp = 0
    for j in range(int(w[W_NREAL])):
        fp |= parity(fixed & int(w[W_RFULL + j])) << j
    off = w[W_OFF:W_OFF + 16]
    base = w[W_BL + (col & 31)] ^ w[W_BH + (col >> 5)] ^ off[fp]
    return base[:, None] ^ off[None, :]


def _pair_addr(w, t, fixed):
    """[blocks, 16 (x), 16 (y)] tile addresses of a pair record's cosets, computed as the kernel does."""
    fo = 0
    for off, rows in ((W_OFF, W_RFULL), (W_OFF2, W_RFULL2)):
        fp = 0
        for j in range(GROUP):
            fp |= parity(fixed & int(w[rows + j])) << j
        fo ^= int(w[off + fp])
    blk = np.arange(1 << (t - 2 * GROUP))
    base = w[W_BL + (blk & 31)] ^ w[W_BH + (blk >> 5)] ^ fo
    return base[:, None, None] ^ w[W_OFF:W_OFF + 16][None, :, None] ^ w[W_OFF2:W_OFF2 + 16][None, None, :]


def _pair_half(w, which: str):
    """A single-op view (W_NREAL, W_TH, W_PH, W_GIDX) of group X or Y of a pair record (emulator)."""
    v = np.array(w, copy=True)
    if which == "y":
        v[W_NREAL] = w[W_NREAL2]
        v[W_TH:W_TH + 4] = w[W_TH2:W_TH2 + 4]
        v[W_PH:W_PH + 4] = w[W_PH2:W_PH2 + 4]
        v[W_SLOT] = w[W_SLOT2]
    return v


def _grad(w, ps, lm, th, gk, gfac, inside: bool = False):
    """Cross matrix N[b][a] = sum_col psi[b] conj(lam[a]); per qubit 2 x 2 partial trace -> d/dtheta, d/dphi.
    ``inside``: psi and lambda are the op's INPUT states (transposed BACK ops): the generators are X for theta and
    RX^H Z RX = cos(theta) Z + sin(theta) Y for phi (hea_grad_reduce_kernel)."""
    N = ps.T @ lm.conj()
    for jq in range(int(w[W_NREAL])):
        nn = np.zeros((2, 2), dtype=np.complex128)
        for bb in range(16):
            for aa in range(16):
                if ((bb ^ aa) & ~(1 << jq)) == 0:
                    nn[(bb >> jq) & 1, (aa >> jq) & 1] += N[bb, aa]
        sth, sph = int(w[W_TH + jq]), int(w[W_PH + jq])
        if inside:
            t = th[sth]
            gk[sth] += (nn[0, 1] + nn[1, 0]).imag * gfac
            gk[sph] += (np.cos(t) * (nn[0, 0] - nn[1, 1]).imag + np.sin(t) * (nn[0, 1] - nn[1, 0]).real) * gfac
            continue
        ph = th[sph]
        gk[sth] += (np.exp(-1j * ph) * nn[1, 0] + np.exp(1j * ph) * nn[0, 1]).imag * gfac
        gk[sph] += (nn[0, 0] - nn[1, 1]).imag * gfac


def _signs(w, t, fixed, C):
    tau = np.arange(1 << t)
    out = []
    for c in range(C):
        m_t, m_f = int(w[W_OFF + c]), int(w[W_RFULL + 2 * c])
        par = np.array([parity(int(x) & m_t) for x in tau]) ^ parity(fixed & m_f)
        out.append(1.0 - 2.0 * par)
    return np.stack(out)     # [C, 2^t]


def _round16(z):
    return (z.real.astype(np.float16).astype(np.float64) + 1j * z.imag.astype(np.float16).astype(np.float64))


def _bf16(x):
    """float64 -> the bf16 value the kernel stores (fp32 first, then round-to-nearest-even to 8 significand bits,
    as v_cvt_pk_bf16_f32 does)."""
    u = np.asarray(x, dtype=np.float32).view(np.uint32).astype(np.uint64)
    u = ((u + 0x7FFF + ((u >> 16) & 1)) >> 16) << 16
    return u.astype(np.uint32).view(np.float32).astype(np.float64)


def _round_bf16(z):
    return _bf16(z.real) + 1j * _bf16(z.imag)


def emulate(plan: HEAPlan, xang: np.ndarray, params: np.ndarray, wread=None, fp16: bool = False,
            storage: str | None = None):
    """Tile-exact execution of ``plan`` with the kernel's tables.

    xang [K, B, n] encoded feature angles, params [K, P] (theta first), wread [K, B, C] = dL/d<Z_c>.
    Returns expz [K, B, C] and (if wread is given) theta gradients [K, n_theta] summed over samples.
    ``fp16`` rounds the stored amplitudes to half precision after every op (kernel storage format);
    ``storage="bf16"`` to bf16 instead (the bf16 build, csrc/hea_mfma_bf16.hip).
    """
    n, t = plan.n, plan.t
    K, B, _ = xang.shape
    progs = pass_programs(plan)
    if storage is None:
        storage = "fp16" if fp16 else "exact"
    rnd = {"fp16": _round16, "bf16": _round_bf16, "exact": lambda z: z}[storage]
    scale = float(1 << (n // 2))
    expz = np.zeros((K, B, plan.C))
    grads = np.zeros((K, plan.n_theta))
    for k in range(K):
        th = params[k].astype(np.float64)
        Us = {}
        for p in plan.passes:
            for g in p.groups:
                w = group_table(plan, p, g, OP_APPLY)
                Us[g.slot] = group_unitary(th, len(g.qubits), w[W_TH:W_TH + 4], w[W_PH:W_PH + 4])
        for b in range(B):
            wv = [rot_u(th[plan.theta_slot(1, q)], th[plan.theta_slot(1, q) + 1]) @ feature_vec(xang[k, b, q], plan.feature)
                  for q in range(n)]
            idx = np.arange(1 << n)
            psi0 = np.full(1 << n, scale, dtype=np.complex128)
            for q in range(n):
                psi0 = psi0 * np.array(wv[q])[(idx >> q) & 1]
            psi0 = rnd(psi0)
            stored = [psi0]
            # forward passes
            psi = psi0.copy()
            for j, (p, fwd, _) in enumerate(progs):
                out = psi.copy()
                sg_w = np.array([sigma(p.H, int(x)) for x in range(1 << p.t)])
                for tid in range(1 << (n - p.t)):
                    tau = np.arange(1 << p.t)
                    mem = p.mem_index(tau, tid, n)
                    fixed = p.fixed(tid, n)
                    tile = np.empty(1 << p.t, dtype=np.complex128)
                    tile[sg_w] = psi[mem]                     # LDS dword sigma(tau) holds amplitude tau
                    for w in fwd:
                        if w[W_CODE] == OP_APPLY:
                            a = _addr(w, p.t, fixed)
                            tile[a] = rnd((Us[int(w[W_SLOT])] @ tile[a].T).T)
                        elif w[W_CODE] == OP_APPLY2:         # X along x, rounded, then Y along y
                            a = _pair_addr(w, p.t, fixed)
                            v = np.einsum("ij,bjy->biy", Us[int(w[W_SLOT])], tile[a])
                            tile[a] = rnd(np.einsum("ij,bxj->bxi", Us[int(w[W_SLOT2])], rnd(v)))
                        elif w[W_CODE] == OP_READOUT:
                            sg = _signs(w, p.t, fixed, plan.C)
                            expz[k, b] += sg @ (np.abs(tile) ** 2) / scale ** 2
                    out[mem] = tile[sg_w]
                psi = out
                stored.append(psi.copy())
            if wread is None:
                continue
            r = wread[k, b].astype(np.float64)
            rho = np.max(np.abs(r)) if np.max(np.abs(r)) > 0 else 1.0
            rr = r / rho
            gfac = rho / scale ** 2
            lam = None
            for j in range(len(progs) - 1, -1, -1):
                p, _, adj = progs[j]
                psi_in = stored[j + 1]                        # output of forward pass j
                lam_out = np.zeros(1 << n, dtype=np.complex128)
                sg_w = np.array([sigma(p.H, int(x)) for x in range(1 << p.t)])
                for tid in range(1 << (n - p.t)):
                    tau = np.arange(1 << p.t)
                    mem = p.mem_index(tau, tid, n)
                    fixed = p.fixed(tid, n)
                    ps = np.empty(1 << p.t, dtype=np.complex128)
                    ps[sg_w] = psi_in[mem]
                    lm = np.zeros_like(ps)
                    if lam is not None:
                        lm[sg_w] = lam[mem]
                    for w in adj:
                        code = int(w[W_CODE])
                        if code == OP_OBS:
                            sg = _signs(w, p.t, fixed, plan.C)
                            lm = rnd((rr @ sg) * ps)
                            continue
                        if code == OP_BACK2:
                            # X then Y, each transposed: U^H on both states, cross matrix of the rounded results
                            a = _pair_addr(w, p.t, fixed)
                            P, Lm = ps[a], lm[a]
                            Uh = Us[int(w[W_SLOT])].conj().T
                            P, Lm = rnd(np.einsum("ij,bjy->biy", Uh, P)), rnd(np.einsum("ij,bjy->biy", Uh, Lm))
                            _grad(w, P.transpose(0, 2, 1).reshape(-1, 16), Lm.transpose(0, 2, 1).reshape(-1, 16),
                                  th, grads[k], gfac, inside=True)
                            Uh = Us[int(w[W_SLOT2])].conj().T
                            P, Lm = rnd(np.einsum("ij,bxj->bxi", Uh, P)), rnd(np.einsum("ij,bxj->bxi", Uh, Lm))
                            _grad(_pair_half(w, "y"), P.reshape(-1, 16), Lm.reshape(-1, 16), th, grads[k], gfac,
                                  inside=True)
                            ps[a], lm[a] = P, Lm
                            continue
                        if code == OP_GRAD2:
                            a = _pair_addr(w, p.t, fixed)
                            _grad(w, ps[a].transpose(0, 2, 1).reshape(-1, 16), lm[a].transpose(0, 2, 1).reshape(-1, 16),
                                  th, grads[k], gfac)
                            _grad(_pair_half(w, "y"), ps[a].reshape(-1, 16), lm[a].reshape(-1, 16), th, grads[k], gfac)
                            continue
                        a = _addr(w, p.t, fixed)
                        if code == OP_BACK and int(w[W_FLAGS]) & F_BACK_PSI:
                            # transposed BACK: U^H on both, cross matrix of the rounded input states
                            Uh = Us[int(w[W_SLOT])].conj().T
                            lm[a] = rnd((Uh @ lm[a].T).T)
                            ps[a] = rnd((Uh @ ps[a].T).T)
                            _grad(w, ps[a], lm[a], th, grads[k], gfac, inside=True)
                        elif code == OP_BACK:           # lambda only, cross matrix at the op output
                            _grad(w, ps[a], lm[a], th, grads[k], gfac)
                            lm[a] = rnd((Us[int(w[W_SLOT])].conj().T @ lm[a].T).T)
                        else:   # OP_GRAD_L1
                            _grad(w, ps[a], lm[a], th, grads[k], gfac)
                    lam_out[mem] = lm[sg_w]
                lam = lam_out
    return expz, grads
