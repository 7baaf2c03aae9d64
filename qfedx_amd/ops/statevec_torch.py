"""Portable torch implementation of the batched statevector program.

This executes EXACTLY the lowered program (``Circuit.to_program``: ops int32 [G,4] =
kind,q0,q1,slot; coef float32 [G,2] = scale,offset) that the gfx950 pass kernels execute, on a
batch of complex64 states [B, 2^n] where every sample may carry its own parameter row
(``params[B, S]`` = [theta (per-client, expanded) | encoded features]).

Used (a) as the CPU backend (north-star config 1: 4 qubits on CPU, world_size=2 gloo) and
(b) as the numerics oracle for the HIP kernels on the GPU box (tests compare HIP vs this vs the
float64 numpy oracle of ``quantum/statevector.py``).

Gradients: ``adjoint_grads`` implements adjoint differentiation (ROADMAP.md:23,135):
walk the program backwards holding psi_g and lambda_g = U_{g+1}^dag..U_G^dag O psi, and for a
rotation exp(-i a P/2) accumulate dL/da = Im<lambda_g|P|psi_g>.
"""
from __future__ import annotations

import math
from typing import Optional

import torch

from ..quantum.circuit import KIND

RX, RY, RZ, P = KIND["rx"], KIND["ry"], KIND["rz"], KIND["p"]
H, X, Y, Z, S, SDG, T, TDG, SX = (KIND[k] for k in ("h", "x", "y", "z", "s", "sdg", "t", "tdg", "sx"))
CX, CZ = KIND["cx"], KIND["cz"]
PAULI = KIND["pauli"]

_R2 = 1.0 / math.sqrt(2.0)


def gate_angles(ops: torch.Tensor, coef: torch.Tensor, params: torch.Tensor) -> torch.Tensor:
    """Per-sample angle table [B, G] (0 for non-parametric gates)."""
    slot = ops[:, 3].long()
    has = slot >= 0
    vals = torch.zeros(params.shape[0], ops.shape[0], dtype=params.dtype, device=params.device)
    if bool(has.any()):
        vals[:, has] = params[:, slot[has]]
    return coef[:, 0].to(params) * vals + coef[:, 1].to(params)


def _u1(kind: int, ang: torch.Tensor, dtype) -> tuple:
    """2x2 matrix entries (u00,u01,u10,u11), each [B] complex, for a 1-qubit gate."""
    B = ang.shape[0]
    one = torch.ones(B, dtype=dtype, device=ang.device)
    zero = torch.zeros(B, dtype=dtype, device=ang.device)
    c = torch.cos(ang / 2).to(dtype)
    s = torch.sin(ang / 2).to(dtype)
    if kind == RX:
        return c, -1j * s, -1j * s, c
    if kind == RY:
        return c, -s, s, c
    if kind == RZ:
        return torch.exp(-0.5j * ang.to(dtype)), zero, zero, torch.exp(0.5j * ang.to(dtype))
    if kind == P:
        return one, zero, zero, torch.exp(1j * ang.to(dtype))
    if kind == H:
        return one * _R2, one * _R2, one * _R2, -one * _R2
    if kind == X:
        return zero, one, one, zero
    if kind == Y:
        return zero, -1j * one, 1j * one, zero
    if kind == Z:
        return one, zero, zero, -one
    if kind == S:
        return one, zero, zero, 1j * one
    if kind == SDG:
        return one, zero, zero, -1j * one
    if kind == T:
        return one, zero, zero, one * complex(math.cos(math.pi / 4), math.sin(math.pi / 4))
    if kind == TDG:
        return one, zero, zero, one * complex(math.cos(math.pi / 4), -math.sin(math.pi / 4))
    if kind == SX:
        return one * (0.5 + 0.5j), one * (0.5 - 0.5j), one * (0.5 - 0.5j), one * (0.5 + 0.5j)
    if kind == PAULI:   # per-sample trajectory Pauli, value 0/1/2/3 = I/X/Y/Z
        ch = torch.round(ang).long()
        i_, x_, y_, z_ = ((ch == v).to(dtype) for v in range(4))
        return i_ + z_, x_ - 1j * y_, x_ + 1j * y_, i_ - z_
    raise ValueError(f"not a 1-qubit kind: {kind}")


def _apply_1q(state: torch.Tensor, q: int, u) -> torch.Tensor:
    B, N = state.shape
    s = state.view(B, N >> (q + 1), 2, 1 << q)
    a0, a1 = s[:, :, 0, :], s[:, :, 1, :]
    u00, u01, u10, u11 = (t.view(B, 1, 1) for t in u)
    return torch.stack([u00 * a0 + u01 * a1, u10 * a0 + u11 * a1], 2).reshape(B, N)


def _cx_perm(n: int, c: int, t: int, device) -> torch.Tensor:
    idx = torch.arange(1 << n, device=device)
    return torch.where(((idx >> c) & 1) == 1, idx ^ (1 << t), idx)


def _cz_sign(n: int, a: int, b: int, device, dtype) -> torch.Tensor:
    idx = torch.arange(1 << n, device=device)
    both = (((idx >> a) & 1) & ((idx >> b) & 1)) == 1
    return torch.where(both, -1.0, 1.0).to(dtype)


def z_signs(n: int, qubits, device, dtype=torch.float32) -> torch.Tensor:
    """[C, 2^n] table of (1 - 2*bit_q(i)) for readout qubits."""
    idx = torch.arange(1 << n, device=device)
    return torch.stack([(1 - 2 * ((idx >> q) & 1)).to(dtype) for q in qubits])


class TorchProgram:
    """A lowered circuit bound to a device; caches permutation/sign tables."""

    def __init__(self, ops, coef, n_qubits: int, device="cpu", dtype=torch.complex64):
        self.ops = torch.as_tensor(ops, dtype=torch.int32).cpu()
        self.coef = torch.as_tensor(coef, dtype=torch.float32).cpu()
        self.n = n_qubits
        self.device = torch.device(device)
        self.dtype = dtype
        self.rdtype = torch.float64 if dtype == torch.complex128 else torch.float32
        self._perm = {}
        self._sign = {}
        self.ops_list = [tuple(int(v) for v in r) for r in self.ops.tolist()]

    def perm(self, c, t):
        key = (c, t)
        if key not in self._perm:
            self._perm[key] = _cx_perm(self.n, c, t, self.device)
        return self._perm[key]

    def sign(self, a, b):
        key = (min(a, b), max(a, b))
        if key not in self._sign:
            self._sign[key] = _cz_sign(self.n, a, b, self.device, self.dtype)
        return self._sign[key]

    def initial_state(self, B: int) -> torch.Tensor:
        st = torch.zeros(B, 1 << self.n, dtype=self.dtype, device=self.device)
        st[:, 0] = 1.0
        return st

    def angles(self, params: torch.Tensor) -> torch.Tensor:
        return gate_angles(self.ops.to(params.device), self.coef.to(params.device), params.to(self.rdtype))

    def run(self, params: torch.Tensor, state: Optional[torch.Tensor] = None, inverse: bool = False,
            gate_range: Optional[tuple] = None) -> torch.Tensor:
        ang = self.angles(params)
        B = params.shape[0]
        st = self.initial_state(B) if state is None else state
        g0, g1 = gate_range if gate_range is not None else (0, len(self.ops_list))
        order = range(g1 - 1, g0 - 1, -1) if inverse else range(g0, g1)
        for g in order:
            st = self.apply_gate(st, g, ang[:, g], inverse)
        return st

    def apply_gate(self, st: torch.Tensor, g: int, ang: torch.Tensor, inverse: bool = False) -> torch.Tensor:
        kind, q0, q1, _ = self.ops_list[g]
        if kind == CX:
            return st[:, self.perm(q0, q1)]
        if kind == CZ:
            return st * self.sign(q0, q1)
        u = _u1(kind, ang, self.dtype)
        if inverse:
            u = (u[0].conj(), u[2].conj(), u[1].conj(), u[3].conj())
        return _apply_1q(st, q0, u)

    # ------------------------------------------------------------------ readout
    def expz(self, state: torch.Tensor, readout) -> torch.Tensor:
        probs = (state.real ** 2 + state.imag ** 2).to(self.rdtype)
        return probs @ z_signs(self.n, readout, state.device, self.rdtype).T

    # ------------------------------------------------------------------ adjoint
    def adjoint_grads(self, params: torch.Tensor, psi: torch.Tensor, w: torch.Tensor, readout) -> torch.Tensor:
        """dL/d(angle_g) for every gate, given final psi [B,N] and dL/d<Z_c> = w [B,C].

        Returns [B, G] (zero for non-parametric gates).  O = sum_c w_c Z_c.
        """
        ang = self.angles(params)
        zs = z_signs(self.n, readout, psi.device, self.rdtype)       # [C, N]
        lam = psi * (w.to(self.rdtype) @ zs).to(self.dtype)          # O psi
        G = len(self.ops_list)
        grads = torch.zeros(psi.shape[0], G, dtype=self.rdtype, device=psi.device)
        for g in range(G - 1, -1, -1):
            kind, q0, _, slot = self.ops_list[g]
            if slot >= 0 and kind in (RX, RY, RZ, P):
                grads[:, g] = self._grad_term(kind, q0, psi, lam)
            psi = self.apply_gate(psi, g, ang[:, g], inverse=True)
            lam = self.apply_gate(lam, g, ang[:, g], inverse=True)
        return grads

    def _grad_term(self, kind: int, q: int, psi: torch.Tensor, lam: torch.Tensor) -> torch.Tensor:
        B, N = psi.shape
        p = psi.view(B, N >> (q + 1), 2, 1 << q)
        l = lam.view(B, N >> (q + 1), 2, 1 << q)
        p0, p1 = p[:, :, 0, :], p[:, :, 1, :]
        l0, l1 = l[:, :, 0, :].conj(), l[:, :, 1, :].conj()
        if kind == RX:      # <l|X|p>
            v = l0 * p1 + l1 * p0
        elif kind == RY:    # <l|Y|p>
            v = -1j * l0 * p1 + 1j * l1 * p0
        else:               # RZ / P: <l|Z|p>
            v = l0 * p0 - l1 * p1
        return v.sum(dim=(1, 2)).imag.to(self.rdtype)


def slot_grads(grads_gate: torch.Tensor, ops: torch.Tensor, coef: torch.Tensor, n_slots: int) -> torch.Tensor:
    """Map per-gate angle grads [B,G] to per-slot grads [B,S] (chain rule through scale)."""
    slot = ops[:, 3].long().to(grads_gate.device)
    scale = coef[:, 0].to(grads_gate)
    out = torch.zeros(grads_gate.shape[0], n_slots, dtype=grads_gate.dtype, device=grads_gate.device)
    m = slot >= 0
    out.index_add_(1, slot[m], grads_gate[:, m] * scale[m])
    return out
