"""Model adapters: bind a model family to the generic federated runner.

An adapter exposes ``n_params``, ``init_params(seed)``, ``angle_mask()``, ``trainer`` (client-batched
local training), ``evaluate(params, X, y)`` and ``state_dict`` / ``from_state_dict`` for the
checkpoint layout (VQC: ``theta``, ``readout.a``, ``readout.b``; TinyCNN: the reference keys
``conv1.weight`` ... ``fc2.bias``, ``Classical_FL.py:21-38``).
"""
from __future__ import annotations

import torch

from ..models.vqc import VQCSpec
from ..quantum.noise import NoiseModel
from ..ops.engine import VQCEngine
from .trainer import VQCClientTrainer


def resolve_state_dtype(state_dtype: str, spec, backend: str, noise) -> str:
    """``auto``: the fp16 MFMA engine (ops/hea_mfma.py) on the HIP backend for the specs it covers (CNOT-chain
    or no entangler, angle features, >= 8 qubits, no gate noise; readout confusion and shots are applied by its
    readout kernels), the fp32 VALU pass engine otherwise.  ``bf16``: the bf16 MFMA engine (``mfma_bf16``) where the
    MFMA engine applies, else bf16 storage on the VALU pass engine; ``bf16_valu`` forces the latter."""
    if state_dtype == "bf16_valu":
        return "bf16"
    if state_dtype == "bf16":
        if backend == "hip" and (noise is None or not noise.gate_noise):
            from ..ops.hea_plan import eligible
            if eligible(spec):
                return "mfma_bf16"
        return "bf16"
    if state_dtype != "auto":
        return state_dtype
    if backend == "hip" and (noise is None or not noise.gate_noise):
        from ..ops.hea_plan import eligible
        if eligible(spec):
            return "mfma"
    return "fp32"


class VQCAdapter:
    def __init__(self, cfg, device, backend: str):
        m = cfg.model
        self.noise = NoiseModel.from_config(getattr(cfg, "noise", None), cfg.train.seed)
        sim = getattr(m, "simulator", "statevector")
        if sim not in ("statevector", "mps", "density"):
            raise ValueError(f"model.simulator must be statevector, mps or density, got '{sim}'")
        if self.noise is not None and self.noise.exact_only and sim != "density":
            if sim == "mps" or m.n_qubits > 10:
                raise ValueError("noise.kind=amplitude (exact amplitude damping) runs on the density-matrix simulator "
                                 "(<= 10 qubits); use noise.kind=amplitude_twirl (Pauli-twirl trajectories) beyond")
            sim = "density"                   # exact Kraus channel: the only simulator that realises it
        self.simulator = sim
        # statevector / MPS engines realise Pauli channels as trajectories; the density simulator applies the
        # channel itself (no trajectory ops in the circuit)
        self.spec = VQCSpec(m.n_qubits, m.n_layers, m.n_classes, m.feature_map, m.feature_scale,
                            m.alpha, m.entangler, None, m.readout_scale, m.init_std,
                            noisy=self.noise is not None and self.noise.pauli_noise and sim != "density")
        self.device = torch.device(device)
        # the circuit engine follows model.simulator; optimizer / aggregation kernels follow the runtime backend
        self.state_dtype = resolve_state_dtype(m.state_dtype, self.spec, backend, self.noise)
        self.engine = VQCEngine(self.spec, device, sim if sim in ("mps", "density") else backend, self.state_dtype,
                                noise=self.noise, mps_chi=int(getattr(m, "mps_chi", 64)))
        self.trainer = VQCClientTrainer(self.spec, self.engine, cfg.train, device, backend)
        # QR/SVD recompression is data dependent: the MPS round runs eagerly, not as a captured graph
        self.trainer.graphs = bool(getattr(cfg.runtime, "use_graphs", True)) and sim not in ("mps", "density")
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

    def _eval_logits(self, params: torch.Tensor, X: torch.Tensor, chunk: int) -> torch.Tensor:
        xang = self.spec.encode_features(X[None])
        ro_keys = None
        if self.noise is not None:     # noisy device: one keyed trajectory per test sample, noisy readout
            xang = self.engine.augment(xang, self.noise.client_keys("noise_eval", chunk, [0], X.device), 0)
            ro_keys = self.noise.client_keys("shots_eval", chunk, [0], X.device)
        return self.engine.predict(xang, params[None, :], ro_keys, 0, X[None] if self.spec.amplitude else None)[0]

    @torch.no_grad()
    def evaluate(self, params: torch.Tensor, X: torch.Tensor, y: torch.Tensor):
        if X.shape[0] == 0:
            return 0.0, 0.0, 0.0
        loss_sum = torch.zeros((), dtype=torch.float64, device=X.device)
        correct = torch.zeros((), dtype=torch.float64, device=X.device)
        for i, s in enumerate(range(0, X.shape[0], self.eval_batch)):
            lg = self._eval_logits(params, X[s: s + self.eval_batch], i)
            yb = y[s: s + self.eval_batch]
            loss_sum += torch.nn.functional.cross_entropy(lg.float(), yb, reduction="sum").double()
            correct += (lg.argmax(-1) == yb).sum().double()
        return float(loss_sum), float(correct), float(X.shape[0])

    @torch.no_grad()
    def logits(self, params: torch.Tensor, X: torch.Tensor) -> torch.Tensor:
        """Test-set logits [N, C] (AUC / calibration metrics)."""
        out = [self._eval_logits(params, X[s: s + self.eval_batch], i)
               for i, s in enumerate(range(0, X.shape[0], self.eval_batch))]
        return torch.cat(out) if out else torch.zeros(0, self.spec.n_classes, device=X.device)


def make_adapter(cfg, device, backend: str):
    if cfg.model.kind == "vqc":
        return VQCAdapter(cfg, device, backend)
    if cfg.model.kind == "tinycnn":
        from .cnn_adapter import TinyCNNAdapter
        return TinyCNNAdapter(cfg, device, backend)
    raise ValueError(f"unknown model kind '{cfg.model.kind}'")
