"""Exact density-matrix simulator for small noisy VQCs (ROADMAP.md:64-73).

The statevector engines realise gate noise as Pauli-channel trajectories, which is exact for depolarizing noise
but only the Pauli twirl of amplitude damping.  ``model.simulator=density`` (auto-selected for
``noise.kind=amplitude``) runs every sample's circuit as a density matrix instead, with the gate-noise channel as
its exact Kraus operators after every gate:

  * HIP: ``csrc/density.hip`` - one workgroup per circuit instance, rho in LDS up to 6 qubits, an L2-resident
    global slab up to 10; a one-qubit gate and its channel are ONE 4 x 4 superoperator pass
  * torch: the same superoperator passes on a [S, 2^n, 2^n] complex128 tensor (CPU path and test oracle)

Readout confusion and shots apply to the exact <Z> as on the other engines.  Gradients: parameter shift (valid
for the exp(-i theta P / 2) rotations with parameter-independent channels in between) or SPSA; the adjoint method
is statevector-only.
"""
from __future__ import annotations

import math

import numpy as np
import torch

from ..quantum.circuit import KIND, gate_matrix

MAX_QUBITS = 10
_INV = {v: k for k, v in KIND.items()}
_PARAM = {"rx", "ry", "rz", "p"}
_TWO = {"cx", "cz", "swap"}

_I = np.eye(2, dtype=complex)
_X = np.array([[0, 1], [1, 0]], complex)
_Y = np.array([[0, -1j], [1j, 0]])
_Z = np.diag([1.0, -1.0]).astype(complex)


def kraus_ops(kind: str, p: float = 0.0, gamma: float = 0.0) -> list[np.ndarray]:
    """Kraus operators of the per-gate channel: ``depolarizing`` (p: X, Y, Z with p / 3 each), ``amplitude``
    (exact amplitude damping: K0 = diag(1, sqrt(1 - gamma)), K1 = sqrt(gamma) |0><1|), ``amplitude_twirl`` (its
    Pauli twirl, what the statevector trajectories realise)."""
    kind = (kind or "none").lower()
    if kind in ("none", "ideal", ""):
        return [_I]
    if kind in ("depolarizing", "depolarising", "dep"):
        return [math.sqrt(1 - p) * _I, math.sqrt(p / 3) * _X, math.sqrt(p / 3) * _Y, math.sqrt(p / 3) * _Z]
    if kind in ("amplitude", "amplitude_damping", "amp"):
        return [np.diag([1.0, math.sqrt(max(0.0, 1.0 - gamma))]).astype(complex),
                np.array([[0.0, math.sqrt(gamma)], [0.0, 0.0]], complex)]
    if kind in ("amplitude_twirl", "amp_twirl"):
        from ..quantum.noise import pauli_probs
        px, py, pz = pauli_probs(kind, p, gamma)
        return [math.sqrt(max(0.0, 1 - px - py - pz)) * _I, math.sqrt(px) * _X, math.sqrt(py) * _Y,
                math.sqrt(pz) * _Z]
    raise ValueError(f"unknown noise kind '{kind}'")


def superop(kraus: list[np.ndarray]) -> np.ndarray:
    """4 x 4 S[(a, b)][(a', b')] = sum_i K_i[a][a'] conj(K_i[b][b']) over quad index a + 2 b (a: row bit,
    b: column bit of the qubit)."""
    S = np.zeros((4, 4), complex)
    for K in kraus:
        for r in range(4):
            for c in range(4):
                S[r, c] += K[r & 1, c & 1] * np.conj(K[r >> 1, c >> 1])
    return S


def lower(ops: np.ndarray, coef: np.ndarray) -> np.ndarray:
    """Program (ops [G, 4] kind/q0/q1/slot, coef [G, 2] scale/offset) -> the kernel's gate records as int32 words
    [G, 14]: kind, q0, q1, slot, scale, off (float bits), fixed 2 x 2 matrix (re, im) x 4 (float bits)."""
    rec = np.zeros((len(ops), 14), dtype=np.int32)
    fl = rec.view(np.float32)
    for g, ((kind, q0, q1, slot), (sc, off)) in enumerate(zip(np.asarray(ops).tolist(), np.asarray(coef).tolist())):
        name = _INV[int(kind)]
        if name in ("pauli", "unitary", "initialize"):
            raise ValueError(f"the density-matrix simulator does not run '{name}' ops")
        rec[g, :4] = (int(kind), int(q0), int(q1), int(slot))
        fl[g, 4], fl[g, 5] = float(sc), float(off)
        if name not in _PARAM and name not in _TWO:
            m = gate_matrix(name)
            fl[g, 6:14] = np.stack([m.real, m.imag], -1).reshape(-1).astype(np.float32)
    return rec


class DensityProgram:
    """Batched exact density-matrix evaluation of one lowered program: ``expz(rows)`` -> <Z_c> [S, C]."""

    def __init__(self, ops, coef, n_qubits: int, readout, device, kraus: list[np.ndarray] | None = None):
        if n_qubits > MAX_QUBITS:
            raise ValueError(f"density-matrix simulation is for <= {MAX_QUBITS} qubits (got {n_qubits}); use the "
                             "statevector engine with noise.kind=amplitude_twirl / depolarizing trajectories")
        self.n = n_qubits
        self.ops = np.asarray(ops)
        self.coef = np.asarray(coef)
        self.readout = [int(c) for c in readout]
        self.device = torch.device(device)
        self.S = superop(kraus) if kraus is not None and len(kraus) > 1 else None
        self.chi_max = 1
        if self.device.type == "cuda":
            from ._ext import ext
            E = ext()
            if E.dm_gate_bytes() != 56:
                raise RuntimeError("density gate record layout mismatch")
            self._gates = torch.from_numpy(lower(self.ops, self.coef).reshape(-1)).to(self.device)
            self._ro = torch.tensor(self.readout, dtype=torch.int32, device=self.device)
            self._sup = (torch.from_numpy(np.stack([self.S.real, self.S.imag], -1).reshape(-1).astype(np.float32))
                         .to(self.device) if self.S is not None else torch.zeros(0, device=self.device))
            self._lds = E.dm_lds_qubits()

    def state_bytes(self) -> int:
        return (1 << (2 * self.n)) * 8

    @torch.no_grad()
    def expz(self, rows: torch.Tensor) -> torch.Tensor:
        rows = rows.float().contiguous()
        S = rows.shape[0]
        C = len(self.readout)
        if S == 0:
            return torch.zeros(0, C, device=rows.device)
        if self.device.type == "cuda":
            from ._ext import ext
            out = torch.empty(S, C, dtype=torch.float32, device=self.device)
            scratch = (torch.empty(S << (2 * self.n), dtype=torch.complex64, device=self.device)
                       if self.n > self._lds else torch.zeros(0, dtype=torch.complex64, device=self.device))
            ext().dm_run(self._gates, len(self.ops), self.n, rows, self._ro, self._sup, scratch, out)
            return out
        return self._expz_torch(rows.double()).float()

    # ------------------------------------------------------------------ torch path (CPU / oracle)
    def _apply_quad(self, rho: torch.Tensor, q: int, T: torch.Tensor) -> torch.Tensor:
        """rho [S, 2^n (rows), 2^n (cols)]; T [S or 1, 4, 4] on (row bit q, col bit q)."""
        S, D = rho.shape[0], 1 << self.n
        hi = D >> (q + 1)
        lo = 1 << q
        r = rho.reshape(S, hi, 2, lo, hi, 2, lo)                     # [S, rh, a, rl, ch, b, cl]
        v = r.permute(0, 1, 3, 4, 6, 5, 2).reshape(S, -1, 4)        # quad index a + 2 b -> (b, a) order
        v = torch.einsum("sij,smj->smi", T.expand(S, 4, 4), v)
        v = v.reshape(S, hi, lo, hi, lo, 2, 2).permute(0, 1, 6, 2, 3, 5, 4)
        return v.reshape(S, D, D)

    def _expz_torch(self, rows: torch.Tensor) -> torch.Tensor:
        S, D = rows.shape[0], 1 << self.n
        rho = torch.zeros(S, D, D, dtype=torch.complex128, device=rows.device)
        rho[:, 0, 0] = 1.0
        Sn = torch.from_numpy(self.S) if self.S is not None else None
        idx = torch.arange(D, device=rows.device)
        for (kind, q0, q1, slot), (sc, off) in zip(self.ops.tolist(), self.coef.tolist()):
            name = _INV[int(kind)]
            if name in _TWO:
                if name == "cz":
                    z = 1 - 2 * (((idx >> q0) & (idx >> q1)) & 1)
                    zz = (z[:, None] * z[None, :]).to(rho.dtype)
                    rho = rho * zz
                else:
                    if name == "cx":
                        perm = torch.where(((idx >> q0) & 1).bool(), idx ^ (1 << q1), idx)
                    else:
                        b0, b1 = (idx >> q0) & 1, (idx >> q1) & 1
                        perm = torch.where(b0 != b1, idx ^ ((1 << q0) | (1 << q1)), idx)
                    rho = rho[:, perm][:, :, perm]
                if Sn is not None:
                    rho = self._apply_quad(rho, q0, Sn[None])
                    rho = self._apply_quad(rho, q1, Sn[None])
                continue
            if name in _PARAM:
                ang = (sc * (rows[:, slot] if slot >= 0 else torch.zeros_like(rows[:, 0])) + off).cpu().numpy()
                U = torch.from_numpy(np.stack([gate_matrix(name, float(a)) for a in ang]))
            else:
                U = torch.from_numpy(gate_matrix(name))[None].expand(S, 2, 2)
            UU = torch.einsum("sac,sbd->sabcd", U, U.conj())        # [(a, b), (a', b')] with a + 2 b order below
            T = UU.permute(0, 2, 1, 4, 3).reshape(S, 4, 4)          # row index b * 2 + a, col b' * 2 + a'
            if Sn is not None:
                T = torch.einsum("ij,sjk->sik", Sn, T)
            rho = self._apply_quad(rho, q0, T.to(rho.device))
        diag = torch.diagonal(rho, dim1=1, dim2=2).real
        return torch.stack([(diag * (1 - 2 * ((idx >> c) & 1))).sum(-1) for c in self.readout], -1)
