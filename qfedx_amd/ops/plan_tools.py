"""Host-side helpers for the pass planner blob (``csrc/qfx_plan.h`` layout).

* ``parse_blob`` - decode header / per-pass descriptors into Python dicts.
* ``emulate_forward`` / ``emulate_adjoint`` - a float64 numpy interpreter of the plan with the
  SAME micro-op semantics as the gfx950 kernel (register/thread/non-tile physical bits, layouts,
  GF(2) remap maps, product-state prefix, lambda = O psi, Im<lambda|G|psi> gradients).  It runs on
  the CPU, so the planner's correctness is tested without a GPU; on the GPU box the kernels are
  then tested against it and against the statevector oracle.
"""
from __future__ import annotations

import math
import struct

import numpy as np

# qfx_plan.h constants
OP_U1, OP_D1, OP_CX, OP_CZ, OP_REMAP = 1, 2, 3, 4, 5
INIT_LOAD, INIT_PRODUCT, INIT_PSI_LAMBDA, INIT_LOAD_BOTH = 0, 1, 2, 3
FIN_STORE, FIN_READOUT = 1, 2
PHYS_NONTILE = 64
PF = dict(K=0, TB=1, INIT=2, FINAL=3, NOPS=4, OPS=5, LAYOUT0=6, NGRAD=7, NNONTILE=8, NREAD=9,
          FINAL_LAYOUT=10, TILEQ=16, NONTILE=40, READ_PHYS=72, LAM_PHYS=80)
HF = dict(N=0, NPASS=1, NGATES=2, GATES=3, PREFIX=4, R=5, NREAD=6, NTHETA=7, PASSES=8)
K_RX, K_RY, K_RZ, K_P, K_H, K_X, K_Y, K_Z, K_S, K_SDG, K_T, K_TDG, K_SX, K_CX, K_CZ = range(15)
DIAG = {K_RZ, K_P, K_Z, K_S, K_SDG, K_T, K_TDG}


def _f(i: int) -> float:
    return struct.unpack("<f", struct.pack("<i", int(i)))[0]


def parse_blob(blob) -> dict:
    b = [int(v) for v in (blob.tolist() if hasattr(blob, "tolist") else blob)]
    n, npass, G = b[HF["N"]], b[HF["NPASS"]], b[HF["NGATES"]]
    gt = b[HF["GATES"]]
    gates = []
    for g in range(G):
        e = b[gt + 6 * g: gt + 6 * g + 6]
        gates.append(dict(kind=e[0], q0=e[1], q1=e[2], slot=e[3], scale=_f(e[4]), offset=_f(e[5])))
    pref = b[HF["PREFIX"]]
    prefix = []
    for q in range(n):
        o = b[pref + q]
        prefix.append(b[o + 1: o + 1 + b[o]])
    passes = []
    for p in range(npass):
        off = b[HF["PASSES"] + p]
        d = {name: b[off + idx] for name, idx in PF.items() if idx < 16}
        k = d["K"]
        d["offset"] = off
        d["tileq"] = b[off + PF["TILEQ"]: off + PF["TILEQ"] + k]
        d["nontile"] = b[off + PF["NONTILE"]: off + PF["NONTILE"] + d["NNONTILE"]]
        d["read_phys"] = b[off + PF["READ_PHYS"]: off + PF["READ_PHYS"] + d["NREAD"]]
        d["lam_phys"] = b[off + PF["LAM_PHYS"]: off + PF["LAM_PHYS"] + d["NREAD"]]
        ops = []
        for i in range(d["NOPS"]):
            o = b[d["OPS"] + 4 * i: d["OPS"] + 4 * i + 4]
            ops.append(tuple(o))
        d["ops"] = ops
        passes.append(d)
    return dict(n=n, npass=npass, G=G, gates=gates, prefix=prefix, passes=passes, R=b[HF["R"]],
                n_read=b[HF["NREAD"]], n_theta=b[HF["NTHETA"]], raw=b)


def _m2(kind: int, ang: float, inv: bool) -> np.ndarray:
    c, s = math.cos(ang / 2), math.sin(ang / 2)
    if kind == K_RX:
        m = np.array([[c, -1j * s], [-1j * s, c]])
    elif kind == K_RY:
        m = np.array([[c, -s], [s, c]], dtype=complex)
    elif kind == K_H:
        m = np.array([[1, 1], [1, -1]], dtype=complex) / math.sqrt(2)
    elif kind == K_X:
        m = np.array([[0, 1], [1, 0]], dtype=complex)
    elif kind == K_Y:
        m = np.array([[0, -1j], [1j, 0]])
    elif kind == K_SX:
        m = 0.5 * np.array([[1 + 1j, 1 - 1j], [1 - 1j, 1 + 1j]])
    else:
        d0, d1 = _d2(kind, ang, False)
        m = np.diag([d0, d1])
    return m.conj().T if inv else m


def _d2(kind: int, ang: float, inv: bool):
    t = complex(math.cos(math.pi / 4), math.sin(math.pi / 4))
    d0, d1 = 1.0 + 0j, 1.0 + 0j
    if kind == K_RZ:
        d0, d1 = np.exp(-0.5j * ang), np.exp(0.5j * ang)
    elif kind == K_P:
        d1 = np.exp(1j * ang)
    elif kind == K_Z:
        d1 = -1
    elif kind == K_S:
        d1 = 1j
    elif kind == K_SDG:
        d1 = -1j
    elif kind == K_T:
        d1 = t
    elif kind == K_TDG:
        d1 = t.conjugate()
    if inv:
        d0, d1 = np.conj(d0), np.conj(d1)
    return d0, d1


class _Ctx:
    def __init__(self, info, p):
        self.info, self.p = info, p
        self.raw = info["raw"]
        self.k = p["K"]
        self.R = info["R"]
        self.rb = int(round(math.log2(self.R)))
        self.lay = p["LAYOUT0"]

    def layout(self, off=None):
        off = self.lay if off is None else off
        return self.raw[off: off + self.k]

    def phys_to_qubit(self, phys: int) -> int:
        if phys >= PHYS_NONTILE:
            return phys - PHYS_NONTILE
        return self.p["tileq"][self.layout()[phys]]


def _angle(g, prow, xrow, n_theta):
    s = g["slot"]
    v = 0.0 if s < 0 else (prow[s] if s < n_theta else xrow[s - n_theta])
    return g["scale"] * v + g["offset"]


def _apply_1q(st, q, m):
    n = int(round(math.log2(st.size)))
    v = st.reshape(1 << (n - q - 1), 2, 1 << q)
    a0, a1 = v[:, 0, :].copy(), v[:, 1, :].copy()
    v[:, 0, :] = m[0, 0] * a0 + m[0, 1] * a1
    v[:, 1, :] = m[1, 0] * a0 + m[1, 1] * a1


def _bits(n):
    return np.arange(1 << n)


def _remap_perm(ctx, n, map_off):
    """Global index permutation applied by a REMAP with a GF(2) map over the tile bits."""
    if map_off < 0:
        return None
    k = ctx.k
    rows = ctx.raw[map_off: map_off + k]
    tq = ctx.p["tileq"]
    idx = _bits(n)
    tidx = np.zeros_like(idx)
    for j, q in enumerate(tq):
        tidx |= ((idx >> q) & 1) << j
    new_t = np.zeros_like(idx)
    for j in range(k):
        par = np.zeros_like(idx)
        m = rows[j]
        for b in range(k):
            if (m >> b) & 1:
                par ^= (tidx >> b) & 1
        new_t |= par << j
    clear = idx.copy()
    for q in tq:
        clear &= ~(1 << q)
    dest = clear.copy()
    for j, q in enumerate(tq):
        dest |= ((new_t >> j) & 1) << q
    return dest   # new_state[dest[i]] = old_state[i]


def _bitvals(n, q):
    return (_bits(n) >> q) & 1


def emulate_pass(info, p, psi, lam, prow, xrow, w_read, adjoint, grads):
    n = info["n"]
    ctx = _Ctx(info, p)
    n_theta = info["n_theta"]
    gates = info["gates"]
    if p["INIT"] == INIT_PRODUCT:
        st = np.ones(1, dtype=complex)
        for q in range(n - 1, -1, -1):
            v = np.array([1.0 + 0j, 0.0])
            for gi in info["prefix"][q]:
                g = gates[gi]
                v = _m2(g["kind"], _angle(g, prow, xrow, n_theta), False) @ v
            st = np.kron(st, v)
        psi[:] = st
    if adjoint and p["INIT"] == INIT_PSI_LAMBDA:
        s = np.zeros(1 << n)
        for c, ph in enumerate(p["lam_phys"]):
            q = ctx.phys_to_qubit(ph)
            s += w_read[c] * (1 - 2 * _bitvals(n, q))
        lam[:] = psi * s
    for code, oa, ob, oc in p["ops"]:
        if code == OP_REMAP:
            perm = _remap_perm(ctx, n, ob)
            if perm is not None:
                for st in ([psi, lam] if adjoint else [psi]):
                    new = np.empty_like(st)
                    new[perm] = st
                    st[:] = new
            ctx.lay = oa
            continue
        g = gates[oc]
        kind = g["kind"]
        ang = _angle(g, prow, xrow, n_theta)
        is_grad = adjoint and 0 <= g["slot"] < n_theta and kind in (K_RX, K_RY, K_RZ, K_P)
        if code == OP_U1:
            q = ctx.phys_to_qubit(oa)
            if is_grad:
                G = {K_RX: np.array([[0, 1], [1, 0]]), K_RY: np.array([[0, -1j], [1j, 0]])}[kind]
                tmp = psi.copy()
                _apply_1q(tmp, q, G)
                grads[oc] = np.vdot(lam, tmp).imag
            m = _m2(kind, ang, adjoint)
            _apply_1q(psi, q, m)
            if adjoint:
                _apply_1q(lam, q, m)
        elif code == OP_D1:
            q = ctx.phys_to_qubit(oa)
            bv = _bitvals(n, q)
            if is_grad:
                grads[oc] = np.vdot(lam, psi * (1 - 2 * bv)).imag
            d0, d1 = _d2(kind, ang, adjoint)
            ph = np.where(bv == 1, d1, d0)
            psi *= ph
            if adjoint:
                lam *= ph
        elif code == OP_CX:
            c = ctx.phys_to_qubit(oa)
            t = ctx.phys_to_qubit(ob)
            idx = _bits(n)
            perm = np.where(((idx >> c) & 1) == 1, idx ^ (1 << t), idx)
            psi[:] = psi[perm]
            if adjoint:
                lam[:] = lam[perm]
        elif code == OP_CZ:
            a, b = ctx.phys_to_qubit(oa), ctx.phys_to_qubit(ob)
            sg = np.where((_bitvals(n, a) & _bitvals(n, b)) == 1, -1.0, 1.0)
            psi *= sg
            if adjoint:
                lam *= sg
    out = None
    if p["FINAL"] & FIN_READOUT:
        probs = np.abs(psi) ** 2
        out = np.array([np.sum(probs * (1 - 2 * _bitvals(n, ctx.phys_to_qubit(ph)))) for ph in p["read_phys"]])
    return out


def emulate_forward(info, prow, xrow):
    n = info["n"]
    psi = np.zeros(1 << n, dtype=complex)
    psi[0] = 1.0
    out = None
    for p in info["passes"]:
        out = emulate_pass(info, p, psi, None, prow, xrow, None, False, None)
    return psi, out


def emulate_adjoint(info, psi_final, prow, xrow, w_read):
    psi = psi_final.astype(complex).copy()
    lam = np.zeros_like(psi)
    grads = np.zeros(info["G"])
    for p in info["passes"]:
        emulate_pass(info, p, psi, lam, prow, xrow, w_read, True, grads)
    return grads
