"""Quantum noise model (ROADMAP.md:64-73): ``NoiseConfig`` -> gate noise as stochastic
Pauli trajectories, readout confusion and finite-shot sampling of the <Z> readout.

Gate noise.  After every gate, each qubit it acts on passes through a single-qubit channel:
    * ``depolarizing``(p):         Pauli channel px = py = pz = p / 3
    * ``amplitude``(gamma):        EXACT amplitude damping, K0 = diag(1, sqrt(1 - gamma)), K1 = sqrt(gamma) |0><1|.
                                   Its jumps are norm-dependent, so it runs on the density-matrix simulator
                                   (ops/density.py, csrc/density.hip; <= 10 qubits, auto-selected)
    * ``amplitude_twirl``(gamma):  the Pauli twirl of amplitude damping, px = py = gamma / 4,
                                   pz = (1 - gamma / 2 - sqrt(1 - gamma)) / 2 - a unitary-trajectory
                                   approximation for the statevector engines past density-matrix sizes
Pauli channels run on the statevector engines as stochastic trajectories (exact in expectation); the density
simulator applies any of the three as exact Kraus maps.
A trajectory is realised by ``pauli`` ops (``Circuit.pauli``) whose per-sample selector 0/1/2/3 =
I/X/Y/Z is an extra x-slot column drawn from Philox keyed by (seed, round, client, local step,
sample, op): the statevector kernels execute it like any other 1-qubit gate, averaging over samples
(and ``trajectories`` replicas) estimates the noisy channel.

Readout.  <Z>' = (1 - p01 - p10) <Z> + p10 - p01 on each readout marginal (exact for the confusion
channel), then with ``shots`` > 0 the estimate 1 - 2 k / shots, k ~ Binomial(shots, (1 - <Z>') / 2)
(drawn as a count of keyed uniforms, identical on CPU and in the HIP kernels).  Training uses the
straight-through gradient d<Z>_noisy/d<Z> = 1 - p01 - p10.
"""
from __future__ import annotations

import math
from dataclasses import dataclass
from typing import Optional

import numpy as np
import torch

from ..utils.seeding import philox_keys, philox_uniform_rows


EXACT_ONLY = ("amplitude", "amplitude_damping", "amp")     # channels with no Pauli-trajectory realisation


def pauli_probs(kind: str, p: float = 0.0, gamma: float = 0.0) -> tuple[float, float, float]:
    """Pauli-channel probabilities of a noise kind the statevector trajectories realise exactly in expectation."""
    kind = (kind or "none").lower()
    if kind in ("none", "ideal", ""):
        return 0.0, 0.0, 0.0
    if kind in ("depolarizing", "depolarising", "dep"):
        return p / 3.0, p / 3.0, p / 3.0
    if kind in ("amplitude_twirl", "amp_twirl"):
        pz = (1.0 - gamma / 2.0 - math.sqrt(max(0.0, 1.0 - gamma))) / 2.0
        return gamma / 4.0, gamma / 4.0, pz
    if kind in EXACT_ONLY:
        raise ValueError("exact amplitude damping is not a Pauli channel: it runs on the density-matrix simulator "
                         "(model.simulator=density, <= 10 qubits); noise.kind=amplitude_twirl is its Pauli-twirl "
                         "approximation for statevector trajectories")
    raise ValueError(f"unknown noise kind '{kind}' (none | depolarizing | amplitude | amplitude_twirl)")


@dataclass
class NoiseModel:
    px: float = 0.0
    py: float = 0.0
    pz: float = 0.0
    p01: float = 0.0
    p10: float = 0.0
    shots: int = 0
    trajectories: int = 1
    seed: int = 0
    kind: str = "none"
    p: float = 0.0
    gamma: float = 0.0

    @classmethod
    def from_config(cls, nc, seed: int = 0) -> Optional["NoiseModel"]:
        if nc is None:
            return None
        kind = (nc.kind or "none").lower()
        px, py, pz = (0.0, 0.0, 0.0) if kind in EXACT_ONLY else pauli_probs(kind, nc.p, nc.gamma)
        m = cls(px, py, pz, float(nc.readout_p01), float(nc.readout_p10), int(nc.shots),
                max(1, int(nc.trajectories)), seed, kind, float(nc.p), float(nc.gamma))
        return m if (m.gate_noise or m.readout_noise) else None

    @property
    def exact_only(self) -> bool:
        """The gate channel has no Pauli-trajectory realisation (exact amplitude damping): density simulator."""
        return self.kind in EXACT_ONLY and self.gamma > 0

    @property
    def gate_noise(self) -> bool:
        return self.px + self.py + self.pz > 0 or self.exact_only

    @property
    def pauli_noise(self) -> bool:
        """Gate noise realised as Pauli trajectories on the statevector engines."""
        return self.px + self.py + self.pz > 0

    def kraus(self):
        """Kraus operators of the per-gate channel (ops/density.py)."""
        from ..ops.density import kraus_ops
        return kraus_ops(self.kind, self.p, self.gamma)

    @property
    def readout_noise(self) -> bool:
        return self.p01 > 0 or self.p10 > 0 or self.shots > 0

    def client_keys(self, purpose: str, round_num: int, client_ids, device) -> torch.Tensor:
        """int64 [K, 2] Philox key words per client for this round (rank-count invariant)."""
        return torch.tensor(philox_keys(self.seed, (purpose, round_num), [int(c) for c in client_ids]),
                            dtype=torch.int64).to(device)

    # ---------------------------------------------------------------- gate noise
    def pauli_columns(self, keys: torch.Tensor, B: int, n_ops: int, step: int) -> torch.Tensor:
        """[K, B, n_ops] float Pauli selectors (0 I, 1 X, 2 Y, 3 Z) for local step ``step``."""
        K = keys.shape[0]
        u = uniforms(keys, B * n_ops, step).reshape(K, B, n_ops)
        t1, t2, t3 = self.px, self.px + self.py, self.px + self.py + self.pz
        sel = (u <= t1).float() + ((u > t1) & (u <= t2)).float() * 2 + ((u > t2) & (u <= t3)).float() * 3
        return sel

    # ---------------------------------------------------------------- readout
    def apply_readout(self, expz: torch.Tensor, keys: Optional[torch.Tensor], step: int) -> torch.Tensor:
        """Confusion + shots on exact expectations [K, B, C] (torch path; the HIP path fuses the
        identical computation into the readout kernels)."""
        z = (1.0 - self.p01 - self.p10) * expz + (self.p10 - self.p01)
        if self.shots <= 0:
            return z
        K, B, C = z.shape
        p1 = ((1.0 - z) * 0.5).clamp(0.0, 1.0)
        u = uniforms(keys, B * C * self.shots, step).reshape(K, B, C, self.shots)
        k = (u <= p1.float()[..., None]).sum(-1).to(z.dtype)
        return 1.0 - 2.0 * k / self.shots


def uniforms(keys: torch.Tensor, n: int, stream: int) -> torch.Tensor:
    """[K, n] Philox uniforms (0,1]; the HIP kernel on GPU, the bit-identical torch oracle on CPU."""
    if keys.is_cuda:
        from ..ops._ext import ext
        out = torch.empty(keys.shape[0], n, dtype=torch.float32, device=keys.device)
        ext().philox_uniform(keys.contiguous(), n, int(stream), out)
        return out
    return philox_uniform_rows(keys, n, stream)


# ------------------------------------------------------------------------------------------------
# float64 density-matrix oracle (tests): exact channel evolution of small circuits
# ------------------------------------------------------------------------------------------------
_PAULI = [np.eye(2, dtype=complex), np.array([[0, 1], [1, 0]], complex), np.array([[0, -1j], [1j, 0]]),
          np.diag([1.0, -1.0]).astype(complex)]


def _op_on(n: int, q: int, m: np.ndarray) -> np.ndarray:
    # little-endian: qubit q is bit q of the index -> kron order (q_{n-1} ... q_0)
    out = np.eye(1, dtype=complex)
    for k in range(n - 1, -1, -1):
        out = np.kron(out, m if k == q else np.eye(2))
    return out


def density_expz(ops: np.ndarray, coef: np.ndarray, n: int, slots: np.ndarray, readout, probs,
                 kraus=None) -> np.ndarray:
    """Exact <Z_c> of the lowered program with a channel after every gate on each qubit it touches: the Pauli
    channel ``probs`` = (px, py, pz), or the Kraus operators ``kraus`` (list of 2 x 2) when given.

    ``ops``/``coef`` = the NOISELESS program (no ``pauli`` ops); ``slots`` = parameter row.
    """
    from .circuit import KIND, gate_matrix
    inv = {v: k for k, v in KIND.items()}
    dim = 1 << n
    rho = np.zeros((dim, dim), complex)
    rho[0, 0] = 1.0
    px, py, pz = probs
    if kraus is None:
        kraus = [math.sqrt(max(0.0, 1 - px - py - pz)) * _PAULI[0], math.sqrt(px) * _PAULI[1],
                 math.sqrt(py) * _PAULI[2], math.sqrt(pz) * _PAULI[3]]
    for (kind, q0, q1, slot), (sc, off) in zip(ops, coef):
        name = inv[int(kind)]
        ang = sc * (slots[slot] if slot >= 0 else 0.0) + off
        if name == "cx":
            U = np.zeros((dim, dim))
            for i in range(dim):
                j = i ^ (1 << q1) if (i >> q0) & 1 else i
                U[j, i] = 1.0
            qs = (q0, q1)
        elif name == "cz":
            U = np.diag([-1.0 if ((i >> q0) & 1) and ((i >> q1) & 1) else 1.0 for i in range(dim)])
            qs = (q0, q1)
        else:
            U = _op_on(n, q0, gate_matrix(name, ang))
            qs = (q0,)
        rho = U @ rho @ U.conj().T
        for q in qs:
            acc = np.zeros_like(rho)
            for K in kraus:
                Kq = _op_on(n, q, K)
                acc = acc + Kq @ rho @ Kq.conj().T
            rho = acc
    diag = np.real(np.diag(rho))
    idx = np.arange(dim)
    return np.array([np.sum(diag * (1 - 2 * ((idx >> c) & 1))) for c in readout])
