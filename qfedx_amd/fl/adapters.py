"""Model adapters: bind a model family to the generic federated runner.

An adapter exposes ``n_params``, ``init_params(seed)``, ``angle_mask()``, ``trainer`` (client-batched
local training), ``evaluate(params, X, y)`` and ``state_dict`` / ``from_state_dict`` for the
checkpoint layout (VQC: ``theta``, ``readout.a``, ``readout.b``; TinyCNN: the reference keys
``conv1.weight`` ... ``fc2.bias``, ``Classical_FL.py:21-38``).
"""
from __future__ import annotations

import torch

from ..models.vqc import VQCSpec
from ..ops.engine import VQCEngine, ce_readout
from .trainer import VQCClientTrainer


class VQCAdapter:
    def __init__(self, cfg, device, backend: str):
        m = cfg.model
        self.spec = VQCSpec(m.n_qubits, m.n_layers, m.n_classes, m.feature_map, m.feature_scale,
                            m.alpha, m.entangler, None, m.readout_scale, m.init_std)
        self.device = torch.device(device)
        self.engine = VQCEngine(self.spec, device, backend, m.state_dtype)
        self.trainer = VQCClientTrainer(self.spec, self.engine, cfg.train, device, backend)
        self.trainer.graphs = bool(getattr(cfg.runtime, "use_graphs", True))
        self.n_params = self.spec.n_params
        self.eval_batch = 4096

    def init_params(self, seed: int) -> torch.Tensor:
        return self.spec.init_params(seed)

    def angle_mask(self) -> torch.Tensor:
        return self.spec.angle_mask()

    def state_dict(self, params: torch.Tensor) -> dict:
        return self.spec.state_dict(params.cpu())

    def from_state_dict(self, sd: dict) -> torch.Tensor:
        return self.spec.from_state_dict(sd)

    @torch.no_grad()
    def evaluate(self, params: torch.Tensor, X: torch.Tensor, y: torch.Tensor):
        if X.shape[0] == 0:
            return 0.0, 0.0, 0.0
        th, a, b = self.spec.split(params[None, :])
        loss_sum = 0.0
        correct = 0.0
        for s in range(0, X.shape[0], self.eval_batch):
            xb = X[s: s + self.eval_batch][None]
            yb = y[s: s + self.eval_batch][None]
            z = self.engine.expz(self.spec.encode_features(xb), th)
            loss, _, _, _, corr = ce_readout(z, yb, torch.ones_like(yb, dtype=z.dtype), a, b)
            loss_sum += float(loss.sum())
            correct += float(corr.sum())
        return loss_sum, correct, float(X.shape[0])


    @torch.no_grad()
    def logits(self, params: torch.Tensor, X: torch.Tensor) -> torch.Tensor:
        """Test-set logits [N, C] (AUC / calibration metrics)."""
        out = []
        for s in range(0, X.shape[0], self.eval_batch):
            xb = self.spec.encode_features(X[s: s + self.eval_batch][None])
            out.append(self.engine.predict(xb, params[None, :])[0])
        return torch.cat(out) if out else torch.zeros(0, self.spec.n_classes, device=X.device)


def make_adapter(cfg, device, backend: str):
    if cfg.model.kind == "vqc":
        return VQCAdapter(cfg, device, backend)
    if cfg.model.kind == "tinycnn":
        from .cnn_adapter import TinyCNNAdapter
        return TinyCNNAdapter(cfg, device, backend)
    raise ValueError(f"unknown model kind '{cfg.model.kind}'")
