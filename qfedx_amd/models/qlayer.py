"""Quantum layers for hybrid PyTorch models, backed by the native statevector engine.

``QuantumExpectation`` is a ``torch.autograd.Function``: forward = <Z_c> of a parametrised circuit per row
of slot values (HIP circuit-specialised kernels on a GPU, the torch executor on CPU); backward = the
adjoint vector-Jacobian product of the incoming gradient, for *every* slot (trainable weights and encoded
inputs alike), so gradients flow into classical layers placed before the circuit.

``VQCLayer`` wraps the VQC ansatz of ``models/vqc.py`` (angle or amplitude feature map, RX/RZ layers,
CNOT chain/ring) as an ``nn.Module``:

    model = nn.Sequential(nn.Linear(8, 4), nn.Tanh(), VQCLayer(4, 2, readout=[0, 1]), nn.Linear(2, 2))

This is the hybrid-model entry point ROADMAP.md:16,20-23 plans through PennyLane's TorchLayer; here it
runs on the same kernels as federated training.
"""
from __future__ import annotations

import math
from typing import Optional

import torch
from torch import nn

from .vqc import VQCSpec


class QuantumExpectation(torch.autograd.Function):
    @staticmethod
    def forward(ctx, values: torch.Tensor, sim, init: Optional[torch.Tensor] = None):
        z = sim.expectation_z(values.detach(), init)
        ctx.sim, ctx.init = sim, init
        ctx.save_for_backward(values)
        return z.to(values.dtype)

    @staticmethod
    def backward(ctx, gz: torch.Tensor):
        (values,) = ctx.saved_tensors
        _, g = ctx.sim.vjp(values.detach(), gz.detach().float(), ctx.init)
        return g[:, : values.shape[1]].to(values.dtype), None, None


class VQCLayer(nn.Module):
    """<Z_c> of the VQC ansatz for inputs x [N, n_features] -> [N, len(readout)].

    Angle feature maps are differentiable in x; with ``feature_map='amplitude'`` x [N, <= 2^n] is the
    (normalised) initial state and receives no gradient."""

    def __init__(self, n_qubits: int, n_layers: int, readout: Optional[list] = None, feature_map: str = "ry",
                 feature_scale: str = "scale", alpha: float = math.pi, entangler: str = "chain",
                 init_std: float = 0.1, seed: int = 0, backend: str = "auto"):
        super().__init__()
        if n_qubits < 2:
            raise ValueError("VQCLayer needs >= 2 qubits")
        self.spec = VQCSpec(n_qubits, n_layers, 2, feature_map, feature_scale, alpha, entangler, init_std=init_std)
        self.readout = list(range(n_qubits)) if readout is None else list(readout)
        if not self.readout or max(self.readout) >= n_qubits:
            raise ValueError("readout qubits out of range")
        g = torch.Generator().manual_seed(seed)
        self.theta = nn.Parameter(torch.randn(self.spec.n_theta, generator=g) * init_std)
        self.backend = backend
        self._sims: dict = {}

    @property
    def n_features(self) -> int:
        return self.spec.n_features

    def _sim(self, device: torch.device):
        key = (device.type, device.index)
        sim = self._sims.get(key)
        if sim is None:
            from ..quantum.simulator import Simulator
            sim = Simulator(self.spec.circuit(), self.readout, device, self.backend,
                            slots=["theta"] if self.spec.amplitude else ["theta", "x"])
            self._sims[key] = sim
        return sim

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        N = x.shape[0]
        th = self.theta[None, :].expand(N, -1)
        if self.spec.amplitude:
            init = self.spec.initial_states(x.detach()).to(x.device)
            return QuantumExpectation.apply(th.float(), self._sim(x.device), init)
        if x.shape[-1] != self.spec.n_features:
            raise ValueError(f"VQCLayer expects {self.spec.n_features} features, got {x.shape[-1]}")
        ang = self.spec.encode_features(x)
        vals = torch.cat([th.to(ang.dtype), ang], 1)
        return QuantumExpectation.apply(vals.float(), self._sim(x.device), None)

    def extra_repr(self) -> str:
        s = self.spec
        return (f"n_qubits={s.n_qubits}, n_layers={s.n_layers}, readout={self.readout}, "
                f"feature_map={s.feature_map}, entangler={s.entangler}")
