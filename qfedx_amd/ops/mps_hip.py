"""HIP fast path of the MPS backend for the CNOT-chain VQC (csrc/mps_chain.hip; math: quantum/mps_chain.py).

``VQCEngine(backend="mps")`` routes <Z> and adjoint gradients here on a GPU when ``mps_chain.eligible(spec)`` (the
angle-encoded RX/RZ + CNOT-chain ansatz with <= 3 layers: exact bond 2^L <= 8, any qubit count); the generic
einsum-network MPS (``quantum/mps.py``) stays the path for every other circuit and on the CPU."""
from __future__ import annotations

import torch

from ..quantum.mps_chain import _FEATURES, eligible
from ._ext import ext

_EMPTY = torch.zeros(0)


class MpsChainProgram:
    def __init__(self, spec, device):
        if not eligible(spec):
            raise ValueError("the MPS chain kernel covers angle-encoded RX/RZ + CNOT-chain VQCs with 1..3 layers")
        self.spec = spec
        self.n, self.L, self.C = spec.n_qubits, spec.n_layers, spec.n_classes
        self.n_theta = spec.n_theta
        self.readout = [int(q) for q in spec.readout]
        self.feature = _FEATURES[spec.feature_map.lower()]
        self.device = torch.device(device)
        self._ws = {}

    def _buf(self, name, numel):
        t = self._ws.get(name)
        if t is None or t.numel() < numel:
            t = torch.empty(numel, dtype=torch.float32, device=self.device)
            self._ws[name] = t
        return t[:numel]

    def _run(self, xang, theta, w=None):
        K, B, F = xang.shape
        S = K * B
        x = xang.reshape(S, F).float().contiguous()
        th = theta.float().contiguous()
        z = torch.empty(S, self.C, dtype=torch.float32, device=self.device)
        rp = self._buf("rp", S * self.n * 128)
        if w is None:
            ext().mps_chain(x, th, B, self.n, self.L, self.feature, self.readout, _EMPTY, z, _EMPTY, rp, _EMPTY)
            return z.view(K, B, self.C), None
        g = torch.empty(S, 2 * self.n * self.L, dtype=torch.float32, device=self.device)
        ro = self._buf("ro", S * (max(self.readout) + 1) * 128)
        ext().mps_chain(x, th, B, self.n, self.L, self.feature, self.readout, w.reshape(S, self.C).float().contiguous(),
                        z, g, rp, ro)
        return z.view(K, B, self.C), g.view(K, B, -1)

    @torch.no_grad()
    def expz(self, xang: torch.Tensor, theta: torch.Tensor) -> torch.Tensor:
        """<Z_c> [K, B, C] for encoded features [K, B, n] and per-client theta [K, >= n_theta]."""
        return self._run(xang, theta)[0]

    @torch.no_grad()
    def grads(self, xang: torch.Tensor, theta: torch.Tensor, w: torch.Tensor) -> torch.Tensor:
        """d/dtheta of sum_{b, c} w[k, b, c] <Z_c>_{k, b}: [K, n_theta] (per-sample gradients summed over each
        client's samples in order)."""
        return self._run(xang, theta, w)[1].sum(1)
