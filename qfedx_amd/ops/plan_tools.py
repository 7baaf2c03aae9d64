"""Host-side helpers for the pass planner blob (``csrc/qfx_plan.h`` layout).

* ``parse_blob`` - decode header / per-pass descriptors into Python dicts.
* ``emulate_forward`` / ``emulate_adjoint`` - a float64 numpy interpreter that mirrors the gfx950
  pass kernel at REGISTER level: every tile is gathered into a [tiles, threads, R] array with the
  precomputed load offsets, micro-ops act on register/thread/non-tile physical bits exactly as the
  kernel does (G1 groups, D1T, CX, CZ), remaps go through an emulated LDS buffer using the
  precomputed XOR slot tables, and results are scattered with the precomputed store offsets.  It
  runs on the CPU, so the planner AND every table it emits are tested without a GPU; on the GPU box
  the kernels are then tested against the torch engine and the statevector oracle.
"""
from __future__ import annotations

import math
import struct

import numpy as np

# qfx_plan.h constants
OP_G1, OP_D1T, OP_CX, OP_CZ, OP_REMAP = 1, 2, 3, 4, 5
INIT_LOAD, INIT_PRODUCT, INIT_PSI_LAMBDA, INIT_LOAD_BOTH = 0, 1, 2, 3
FIN_STORE, FIN_READOUT = 1, 2
PHYS_NONTILE = 64
PF = dict(K=0, TB=1, INIT=2, FINAL=3, NOPS=4, OPS=5, LAYOUT0=6, NGRAD=7, NNONTILE=8, NREAD=9,
          FINAL_LAYOUT=10, TILEQ=16, NONTILE=40, READ_PHYS=72, LAM_PHYS=80, Q0=96, GREG0=120, GTHR0=152,
          GREGF=168, GTHRF=200)
HF = dict(N=0, NPASS=1, NGATES=2, GATES=3, PREFIX=4, R=5, NREAD=6, NTHETA=7, PASSES=8)
K_RX, K_RY, K_RZ, K_P, K_H, K_X, K_Y, K_Z, K_S, K_SDG, K_T, K_TDG, K_SX, K_CX, K_CZ = range(15)
K_PAULI = 18
DIAG = {K_RZ, K_P, K_Z, K_S, K_SDG, K_T, K_TDG}


def _f(i: int) -> float:
    return struct.unpack("<f", struct.pack("<i", int(i)))[0]


def parse_blob(blob) -> dict:
    b = [int(v) for v in (blob.tolist() if hasattr(blob, "tolist") else blob)]
    n, npass, G = b[HF["N"]], b[HF["NPASS"]], b[HF["NGATES"]]
    R = b[HF["R"]]
    rb = int(round(math.log2(R)))
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
        k, tb = d["K"], d["TB"]
        d["offset"] = off
        d["tileq"] = b[off + PF["TILEQ"]: off + PF["TILEQ"] + k]
        d["nontile"] = b[off + PF["NONTILE"]: off + PF["NONTILE"] + d["NNONTILE"]]
        d["read_phys"] = b[off + PF["READ_PHYS"]: off + PF["READ_PHYS"] + d["NREAD"]]
        d["lam_phys"] = b[off + PF["LAM_PHYS"]: off + PF["LAM_PHYS"] + d["NREAD"]]
        d["q0"] = b[off + PF["Q0"]: off + PF["Q0"] + k]
        d["greg0"] = b[off + PF["GREG0"]: off + PF["GREG0"] + R]
        d["gthr0"] = b[off + PF["GTHR0"]: off + PF["GTHR0"] + tb]
        d["gregF"] = b[off + PF["GREGF"]: off + PF["GREGF"] + R]
        d["gthrF"] = b[off + PF["GTHRF"]: off + PF["GTHRF"] + tb]
        ops = []
        for i in range(d["NOPS"]):
            code, a, bb, c = b[d["OPS"] + 4 * i: d["OPS"] + 4 * i + 4]
            op = dict(code=code, a=a, b=bb, c=c)
            if code == OP_G1:
                op["gates"] = b[c: c + bb]
            elif code == OP_REMAP:
                op["wr"] = b[a: a + R]
                op["wt"] = b[a + R: a + R + tb]
                op["rr"] = b[a + R + tb: a + 2 * R + tb]
                op["rt"] = b[a + 2 * R + tb: a + 2 * R + 2 * tb]
            ops.append(op)
        d["ops"] = ops
        passes.append(d)
    return dict(n=n, npass=npass, G=G, gates=gates, prefix=prefix, passes=passes, R=R, rb=rb,
                n_read=b[HF["NREAD"]], n_theta=b[HF["NTHETA"]], raw=b)


def _m2(kind: int, ang: float, inv: bool) -> np.ndarray:
    if kind == K_PAULI:
        m = [np.eye(2), np.array([[0, 1], [1, 0]]), np.array([[0, -1j], [1j, 0]]), np.diag([1, -1])][int(round(ang))]
        return np.asarray(m, dtype=complex)
    c, s = math.cos(ang / 2), math.sin(ang / 2)
    t = complex(math.cos(math.pi / 4), math.sin(math.pi / 4))
    table = {
        K_RX: [[c, -1j * s], [-1j * s, c]],
        K_RY: [[c, -s], [s, c]],
        K_RZ: [[np.exp(-0.5j * ang), 0], [0, np.exp(0.5j * ang)]],
        K_P: [[1, 0], [0, np.exp(1j * ang)]],
        K_H: [[1 / math.sqrt(2), 1 / math.sqrt(2)], [1 / math.sqrt(2), -1 / math.sqrt(2)]],
        K_X: [[0, 1], [1, 0]],
        K_Y: [[0, -1j], [1j, 0]],
        K_Z: [[1, 0], [0, -1]],
        K_S: [[1, 0], [0, 1j]],
        K_SDG: [[1, 0], [0, -1j]],
        K_T: [[1, 0], [0, t]],
        K_TDG: [[1, 0], [0, t.conjugate()]],
        K_SX: [[0.5 + 0.5j, 0.5 - 0.5j], [0.5 - 0.5j, 0.5 + 0.5j]],
    }
    m = np.array(table[kind], dtype=complex)
    return m.conj().T if inv else m


def _angle(g, prow, xrow, n_theta):
    s = g["slot"]
    v = 0.0 if s < 0 else (prow[s] if s < n_theta else xrow[s - n_theta])
    return g["scale"] * v + g["offset"]


def _xor_bits(tab, tl):
    v = np.zeros_like(tl)
    for j, t in enumerate(tab):
        v ^= np.where((tl >> j) & 1 == 1, t, 0)
    return v


class _Tile:
    """Register-level state of one pass over all tiles: arrays [ntiles, T, R]."""

    def __init__(self, info, p):
        self.n = info["n"]
        self.R, self.rb = info["R"], info["rb"]
        self.k, self.tb = p["K"], p["TB"]
        self.T = 1 << self.tb
        self.ntiles = 1 << (self.n - self.k)
        tau = np.arange(self.ntiles)
        self.gbase = np.zeros(self.ntiles, dtype=np.int64)
        for j, q in enumerate(p["nontile"]):
            self.gbase |= ((tau >> j) & 1) << q
        self.tl = np.arange(self.T)
        self.r = np.arange(self.R)

    def bit(self, phys):
        """bit value of phys for every (tile, thread, register) -> int array [ntiles, T, R]"""
        sh = (self.ntiles, self.T, self.R)
        if phys < self.rb:
            return np.broadcast_to(((self.r >> phys) & 1)[None, None, :], sh)
        if phys < PHYS_NONTILE:
            return np.broadcast_to(((self.tl >> (phys - self.rb)) & 1)[None, :, None], sh)
        return np.broadcast_to(((self.gbase >> (phys - PHYS_NONTILE)) & 1)[:, None, None], sh)

    def offsets(self, greg, gthr):
        thr = _xor_bits(gthr, self.tl)
        return self.gbase[:, None, None] + (thr[None, :, None] | np.asarray(greg)[None, None, :])


def _pair_apply(a, rbit, m):
    R = a.shape[-1]
    lo = [r for r in range(R) if not (r >> rbit) & 1]
    hi = [r | (1 << rbit) for r in lo]
    x, y = a[..., lo].copy(), a[..., hi].copy()
    a[..., lo] = m[0, 0] * x + m[0, 1] * y
    a[..., hi] = m[1, 0] * x + m[1, 1] * y


def _pair_grad(a, l, rbit, gen):
    R = a.shape[-1]
    lo = [r for r in range(R) if not (r >> rbit) & 1]
    hi = [r | (1 << rbit) for r in lo]
    p0, p1, l0, l1 = a[..., lo], a[..., hi], l[..., lo], l[..., hi]
    if gen == 1:
        v = (np.conj(l0) * p1 + np.conj(l1) * p0).imag
    elif gen == 2:
        v = (np.conj(l1) * p0).real - (np.conj(l0) * p1).real
    else:
        v = (np.conj(l0) * p0).imag - (np.conj(l1) * p1).imag
    return float(v.sum())


def emulate_pass(info, p, psi, lam, prow, xrow, w_read, adjoint, grads):
    t = _Tile(info, p)
    n_theta = info["n_theta"]
    gates = info["gates"]
    if p["INIT"] == INIT_PRODUCT:
        st = np.ones(1, dtype=complex)
        for q in range(t.n - 1, -1, -1):
            v = np.array([1.0 + 0j, 0.0])
            for gi in info["prefix"][q]:
                g = gates[gi]
                v = _m2(g["kind"], _angle(g, prow, xrow, n_theta), False) @ v
            st = np.kron(st, v)
        a = st[t.offsets(p["greg0"], p["gthr0"])]
        l = np.zeros_like(a)
    else:
        off0 = t.offsets(p["greg0"], p["gthr0"])
        a = psi[off0].copy()
        l = lam[off0].copy() if (adjoint and p["INIT"] == INIT_LOAD_BOTH) else np.zeros_like(a)
        if adjoint and p["INIT"] == INIT_PSI_LAMBDA:
            s = np.zeros(a.shape)
            for c, ph in enumerate(p["lam_phys"]):
                s += np.where(t.bit(ph) == 1, -w_read[c], w_read[c])
            l = a * s
    for op in p["ops"]:
        code = op["code"]
        if code == OP_G1:
            if not adjoint:
                m = np.eye(2, dtype=complex)
                for gi in op["gates"]:
                    g = gates[gi]
                    m = _m2(g["kind"], _angle(g, prow, xrow, n_theta), False) @ m
                _pair_apply(a, op["a"], m)
            else:
                for gi in op["gates"]:
                    g = gates[gi]
                    isg = 0 <= g["slot"] < n_theta and g["kind"] <= K_P
                    if isg:
                        gen = 1 if g["kind"] == K_RX else 2 if g["kind"] == K_RY else 3
                        grads[gi] += _pair_grad(a, l, op["a"], gen)
                    mi = _m2(g["kind"], _angle(g, prow, xrow, n_theta), True)
                    _pair_apply(a, op["a"], mi)
                    _pair_apply(l, op["a"], mi)
        elif code == OP_D1T:
            g = gates[op["c"]]
            m = _m2(g["kind"], _angle(g, prow, xrow, n_theta), adjoint)
            bit = t.bit(op["a"])
            if adjoint and 0 <= g["slot"] < n_theta and g["kind"] in (K_RZ, K_P):
                v = (np.conj(l) * a).imag
                grads[op["c"]] += float(np.where(bit == 1, -v, v).sum())
            ph = np.where(bit == 1, m[1, 1], m[0, 0])
            a = a * ph
            if adjoint:
                l = l * ph
        elif code == OP_REMAP:
            for arr in ([a, l] if adjoint else [a]):
                lds = np.zeros((t.ntiles, 1 << t.k), dtype=complex)
                ws = np.asarray(op["wr"])[None, :] ^ _xor_bits(op["wt"], t.tl)[:, None]   # [T, R]
                rs = np.asarray(op["rr"])[None, :] ^ _xor_bits(op["rt"], t.tl)[:, None]
                assert len(np.unique(ws)) == ws.size, "remap write slots collide"
                lds[:, ws] = arr
                arr[...] = lds[:, rs]
        elif code == OP_CX:
            ctl = t.bit(op["a"])
            R = t.R
            lo = [r for r in range(R) if not (r >> op["b"]) & 1]
            hi = [r | (1 << op["b"]) for r in lo]
            for arr in ([a, l] if adjoint else [a]):
                c = ctl[..., lo] == 1
                x, y = arr[..., lo].copy(), arr[..., hi].copy()
                arr[..., lo] = np.where(c, y, x)
                arr[..., hi] = np.where(c, x, y)
        elif code == OP_CZ:
            neg = (t.bit(op["a"]) & t.bit(op["b"])) == 1
            a = np.where(neg, -a, a)
            if adjoint:
                l = np.where(neg, -l, l)
    out = None
    if p["FINAL"] & FIN_READOUT:
        pr = np.abs(a) ** 2
        out = np.array([float(np.where(t.bit(ph) == 1, -pr, pr).sum()) for ph in p["read_phys"]])
    if p["FINAL"] & FIN_STORE:
        offF = t.offsets(p["gregF"], p["gthrF"])
        psi[offF] = a
        if adjoint:
            lam[offF] = l
    return out


def emulate_forward(info, prow, xrow):
    n = info["n"]
    psi = np.zeros(1 << n, dtype=complex)
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
