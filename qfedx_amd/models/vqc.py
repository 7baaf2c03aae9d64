"""Variational quantum classifier (ROADMAP.md:20-23, 125-135).

Architecture (hardware-efficient ansatz):
  feature map   RY(alpha * x_i) on qubit i            (ROADMAP:126; basis rx/ry/rz selectable,
                                                        reference angle basis ``qAngle.py:44-50``)
  L layers of   RX(theta_{l,q,0}) RZ(theta_{l,q,1}) on every qubit, then a CNOT entangler
                (chain q->q+1, or ring adds n-1 -> 0)    (ROADMAP:21,127)
  readout       <Z_c> on qubits c = 0..C-1; logit_c = a_c <Z_c> + b_c; cross-entropy (ROADMAP:22,128)

Parameters per client: ``theta`` [2nL] (angles, wrapped on aggregation) followed by the classical
readout ``a`` [C] and ``b`` [C]; the flat vector layout is ``[theta | a | b]``.

Gradients: adjoint (default), parameter-shift (ROADMAP:130-133), SPSA (ROADMAP:38) and torch
autograd (CPU cross-check only) - see ``qfedx_amd/ops/engine.py``.
"""
from __future__ import annotations

import math
from dataclasses import dataclass, field
from typing import Optional

import torch

from ..quantum.circuit import Circuit, ParameterVector
from ..utils.seeding import generator


@dataclass
class VQCSpec:
    n_qubits: int = 4
    n_layers: int = 2
    n_classes: int = 3
    feature_map: str = "ry"
    feature_scale: str = "scale"      # 'scale' (alpha*x) | 'minmax' (reference per-sample pi*minmax)
    alpha: float = math.pi
    entangler: str = "chain"          # chain | ring | none
    readout: Optional[list] = None    # readout qubits, default first n_classes
    readout_scale: float = 1.0
    init_std: float = 0.1
    noisy: bool = False               # insert noise-trajectory Pauli ops after every gate (NoiseConfig)

    def __post_init__(self):
        if self.readout is None:
            self.readout = list(range(self.n_classes))
        if len(self.readout) != self.n_classes or max(self.readout) >= self.n_qubits:
            raise ValueError("need one readout qubit per class and n_classes <= n_qubits")
        if self.n_classes < 2:
            raise ValueError("n_classes must be >= 2")

    @property
    def n_theta(self) -> int:
        return 2 * self.n_qubits * self.n_layers

    @property
    def n_params(self) -> int:
        return self.n_theta + 2 * self.n_classes

    @property
    def amplitude(self) -> bool:
        """feature_map='amplitude': the 2^n features ARE the (normalised) initial state (reference
        ``amplitude_encode``, qAmplitude.py:25-41) instead of an RY(alpha x) angle map."""
        return self.feature_map.lower() == "amplitude"

    @property
    def n_features(self) -> int:
        return (1 << self.n_qubits) if self.amplitude else self.n_qubits

    @property
    def n_x_slots(self) -> int:
        return 0 if self.amplitude else self.n_qubits

    @property
    def n_noise_ops(self) -> int:
        """Pauli trajectory ops: one per qubit touched by each gate (feature map, rotations, CNOTs)."""
        if not self.noisy:
            return 0
        n = self.n_qubits
        ent = (n - 1) + (1 if self.entangler == "ring" and n > 2 else 0) if self.entangler in ("chain", "ring") else 0
        return (0 if self.amplitude else n) + self.n_layers * (2 * n + 2 * ent)

    @property
    def x_width(self) -> int:
        """Per-sample x-slot row: encoded angles, then the Pauli selectors of the trajectory (at least one
        column: an amplitude-encoded model without noise carries a dummy)."""
        return max(1, self.n_x_slots + self.n_noise_ops)

    def circuit(self) -> Circuit:
        n = self.n_qubits
        x = ParameterVector("x", n)
        th = ParameterVector("theta", self.n_theta)
        nz = ParameterVector("noise", max(self.n_noise_ops, 1))
        qc = Circuit(n, name=f"VQC_{n}q_{self.n_layers}L")
        j = [0]

        def noise(*qs):
            if self.noisy:
                for q in qs:
                    qc.pauli(nz[j[0]], q)
                    j[0] += 1

        fm = self.feature_map.lower()
        if not self.amplitude:
            for q in range(n):
                getattr(qc, fm if fm in ("rx", "ry", "rz") else "ry")(x[q], q)
                noise(q)
        k = 0
        for _ in range(self.n_layers):
            for q in range(n):
                qc.rx(th[k], q)
                noise(q)
                qc.rz(th[k + 1], q)
                noise(q)
                k += 2
            if self.entangler in ("chain", "ring"):
                for q in range(n - 1):
                    qc.cx(q, q + 1)
                    noise(q, q + 1)
                if self.entangler == "ring" and n > 2:
                    qc.cx(n - 1, 0)
                    noise(n - 1, 0)
        assert j[0] == self.n_noise_ops
        return qc

    def program(self):
        """(ops, coef) with slots [theta (n_theta) | x (n) | noise selectors (n_noise_ops)]."""
        return self.circuit().to_program({"theta": 0, "x": self.n_theta, "noise": self.n_theta + self.n_x_slots})

    def encode_features(self, x: torch.Tensor) -> torch.Tensor:
        """Raw features [.., n] -> encoding angles fed to the x slots (gate scale is 1).  Amplitude
        encoding has no x slots: a dummy column (or nothing, when noise selectors follow)."""
        if self.amplitude:
            return x.new_zeros(*x.shape[:-1], 0 if self.noisy else 1)
        from ..data.features import angle_scale
        return angle_scale(x, self.feature_scale, self.alpha)

    def initial_states(self, x: torch.Tensor) -> Optional[torch.Tensor]:
        """Amplitude encoding: features [.., <= 2^n] -> normalised complex64 states [.., 2^n] (zero vector ->
        uniform state, reference normalize_for_amplitude); None for angle encodings."""
        if not self.amplitude:
            return None
        from ..quantum.encoders import amplitude_states
        N = 1 << self.n_qubits
        if x.shape[-1] < N:
            x = torch.cat([x, x.new_zeros(*x.shape[:-1], N - x.shape[-1])], -1)
        return amplitude_states(x[..., :N]).to(torch.complex64)

    def init_params(self, seed: int = 0) -> torch.Tensor:
        g = generator(seed, "init", 0)
        theta = torch.randn(self.n_theta, generator=g, dtype=torch.float64) * self.init_std
        a = torch.full((self.n_classes,), float(self.readout_scale), dtype=torch.float64)
        b = torch.zeros(self.n_classes, dtype=torch.float64)
        return torch.cat([theta, a, b]).float()

    def split(self, params: torch.Tensor):
        P = self.n_theta
        C = self.n_classes
        return params[..., :P], params[..., P:P + C], params[..., P + C:P + 2 * C]

    def angle_mask(self) -> torch.Tensor:
        """1 for angle parameters (wrapped on aggregation, ROADMAP:37), 0 for readout a/b."""
        m = torch.zeros(self.n_params)
        m[: self.n_theta] = 1.0
        return m

    def state_dict(self, params: torch.Tensor) -> dict:
        th, a, b = self.split(params)
        return {"theta": th.detach().clone(), "readout.a": a.detach().clone(), "readout.b": b.detach().clone()}

    def from_state_dict(self, sd: dict) -> torch.Tensor:
        return torch.cat([sd["theta"].reshape(-1), sd["readout.a"].reshape(-1), sd["readout.b"].reshape(-1)]).float()


def logits_from_expz(expz: torch.Tensor, a: torch.Tensor, b: torch.Tensor) -> torch.Tensor:
    """logit_c = a_c <Z_c> + b_c, broadcasting a/b over leading sample dims."""
    return expz * a.unsqueeze(-2) + b.unsqueeze(-2)
