"""Typed experiment configuration: dataclasses + YAML files + Hydra-like ``key=value`` overrides.

Reference: configuration is hard-coded dicts (``src/CFed/Classical_FL.py:161-173``,
``src/QFed/testEncoder.py:64-72``) and function defaults (``src/CFed/Preprocess.py:137-138``,
``Classical_FL.py:41,104-110``); ROADMAP plans Hydra (``ROADMAP.md:16,70``).  Hydra is not
installed, so this module gives the same ergonomics (YAML + dotted CLI overrides) with
dataclasses.  The reference key names are kept verbatim: ``raw_folder, processed_folder,
digits, val_split, num_clients, partition_type, alpha, num_rounds, local_epochs,
learning_rate, batch_size``.
"""
from __future__ import annotations

import dataclasses
import json
from dataclasses import dataclass, field, asdict
from typing import Any, Optional

import yaml


@dataclass
class DataConfig:
    dataset: str = "synthetic"          # mnist | synthetic | synthetic_digits (MNIST-like images) | iris
    raw_folder: str = "./dataset/raw"
    processed_folder: str = "./dataset/processed"
    digits: tuple = (0, 1, 2)
    val_split: float = 0.1
    num_clients: int = 4
    partition_type: str = "iid"         # iid | non_iid (Dirichlet)
    alpha: float = 0.5                  # Dirichlet concentration
    features: str = "pool"              # pool | pca | downsample | raw
    n_features: int = 0                 # 0 = one per qubit (angle map) / 2^n_qubits (amplitude encoding)
    samples_per_client: int = 256       # synthetic data size per client
    test_samples: int = 512


@dataclass
class ModelConfig:
    kind: str = "vqc"                   # vqc | tinycnn
    n_qubits: int = 4
    n_layers: int = 2
    n_classes: int = 3
    feature_map: str = "ry"             # ry | rx | rz (angle encoding basis) | amplitude (2^n features = state)
    feature_scale: str = "scale"        # scale (RY(alpha*x), ROADMAP:126) | minmax (qAngle.py:36-41)
    alpha: float = 3.141592653589793
    entangler: str = "chain"            # chain | ring | none
    readout_scale: float = 1.0          # initial a in logit = a<Z> + b
    init_std: float = 0.1
    state_dtype: str = "auto"           # auto (mfma when eligible on HIP, else fp32) | fp32 | mfma (fp16 MFMA engine,
                                        # hardware-efficient ansatz) | bf16 (bf16 MFMA engine when eligible, else
                                        # bf16 storage on the VALU pass engine) | bf16_valu
    simulator: str = "statevector"      # statevector | mps (tensor network past statevector memory) | density
                                        # (exact Kraus channels, <= 10 qubits; auto for noise.kind=amplitude)
    mps_chi: int = 64                   # MPS bond-dimension cap (exact while the circuit's bound fits)


@dataclass
class TrainConfig:
    num_rounds: int = 30
    mode: str = "federated"             # federated | centralized (all shards pooled into one client: the
                                        # ROADMAP.md:109 centralized-VQC baseline)
    local_epochs: int = 1
    local_steps: int = 0                # if >0, overrides local_epochs with a fixed step count
    learning_rate: float = 0.05
    batch_size: int = 32
    optimizer: str = "adam"             # adam | sgd | spsa
    momentum: float = 0.9
    grad_method: str = "adjoint"        # adjoint | param_shift | spsa | autograd
    client_fraction: float = 1.0        # ROADMAP:35,106 client sampling
    sampling: str = "auto"              # auto (poisson under DP, else fixed) | fixed (m = round(q N)) | poisson
    dropout_prob: float = 0.0           # simulated client dropouts (ROADMAP:91)
    aggregate: str = "delta"            # delta (ROADMAP:36) | weights (Classical_FL.py:66-81)
    wrap_angles: bool = True            # wrap angle deltas to [-pi, pi] (ROADMAP:37)
    weighting: str = "samples"          # samples | uniform
    server_optimizer: str = "fedavg"    # fedavg | momentum (FedAvgM) | adam (FedAdam); state sharded over ranks
    server_lr: float = 1.0
    server_momentum: float = 0.9
    eval_every: int = 1
    fuse_optimizer: bool = True         # HIP CFed: SGD-momentum step fused into the gradient kernels (csrc/cnn_args.h)
    seed: int = 42


@dataclass
class PrivacyConfig:
    dp: bool = False
    clip_norm: float = 1.0              # C (ROADMAP:50)
    noise_multiplier: float = 1.0       # sigma (ROADMAP:51)
    delta: float = 1e-5
    secure_agg: bool = False
    secagg_bits: int = 48               # fixed-point ring Z_{2^bits} for exact mask cancellation
    secagg_scale: float = 2.0 ** 24
    secagg_graph: str = "full"          # full (every pair) | sparse (SecAgg+: 2 ceil(log2 K) neighbours, O(K log K))
    # a round is aborted (no update aggregated) if a surviving participant has fewer live mask neighbours than this;
    # 0 = auto: half its graph degree (sparse, SecAgg+), 1 (full graph)
    secagg_min_live: int = 0
    # local: every client adds N(0, sigma^2 C^2) (ROADMAP.md:50-51; the sum carries sqrt(m) sigma C);
    # distributed: every client adds N(0, sigma^2 C^2 / m) for the round's m live participants, so the SecAgg sum
    # carries exactly the sigma C the accountant charges (distributed DP: needs secure_agg to hide each share)
    noise_mode: str = "local"
    # testing/debug only: key DP noise and DP client sampling by the PUBLIC train.seed (reproducible
    # across runs and rank counts) instead of a per-run secret - voids the DP guarantee
    deterministic_noise: bool = False


@dataclass
class NoiseConfig:
    """Quantum noise model (ROADMAP.md:64-73)."""
    kind: str = "none"                  # none | depolarizing | amplitude (exact, density simulator) | amplitude_twirl
    p: float = 0.0                      # depolarizing probability per gate
    gamma: float = 0.0                  # amplitude damping per gate
    readout_p01: float = 0.0            # P(read 1 | 0)
    readout_p10: float = 0.0            # P(read 0 | 1)
    shots: int = 0                      # 0 = exact expectation
    trajectories: int = 1


@dataclass
class RuntimeConfig:
    device: str = "auto"                # auto | cpu | cuda
    backend: str = "auto"               # auto | hip | torch
    dist_backend: str = "auto"          # auto | nccl (RCCL) | gloo
    checkpoint_dir: str = ""
    checkpoint_every: int = 0
    resume: bool = False
    metrics_path: str = ""
    tracking_dir: str = ""              # MLflow file-store root (e.g. ./mlruns); "" = off
    experiment: str = ""                # tracking experiment name ("" = config name)
    log_every: int = 5
    overlap_comm: bool = True
    use_graphs: bool = True            # hipGraph capture of the local round (HIP backend)
    graph_comm: bool = True            # capture the round's all-reduce + apply into that graph (RCCL / no group)
    # CC4: with more than one rank, round r + 1's theta-independent inputs (setup, minibatch plan, tables, gather +
    # encode) are built while round r's collective is in flight (gloo: async all-reduce).  overlap_comm_device: the
    # graphed HIP round's upload + gather on a side stream against the previous round's graph + collective - bitwise
    # the same, but the cross-queue join costs +12-15 us per round at one RCCL rank against a ~5 us gather
    # (profiles/r6_cc4_overlap.txt), so it is opt-in.  QFEDX_CC4=0 / 1 overrides both (1 also at one rank, for tests)
    overlap_comm: bool = True
    overlap_comm_device: bool = False
    timer_every: int = 0               # time the GPU phases every N-th round (0: 16 on GPU, every round on CPU)
    log_client_norms: bool = False     # NON-PRIVATE debug diagnostic (DP rounds): every client's raw pre-clip update
                                       # norm reaches every rank in the round all-reduce (CC6) and clip fraction +
                                       # norm quantiles are logged; they are not noised nor charged to the
                                       # accountant (never under SecAgg)


@dataclass
class ExperimentConfig:
    name: str = "qfedx"
    data: DataConfig = field(default_factory=DataConfig)
    model: ModelConfig = field(default_factory=ModelConfig)
    train: TrainConfig = field(default_factory=TrainConfig)
    privacy: PrivacyConfig = field(default_factory=PrivacyConfig)
    noise: NoiseConfig = field(default_factory=NoiseConfig)
    runtime: RuntimeConfig = field(default_factory=RuntimeConfig)

    def to_dict(self) -> dict:
        return asdict(self)

    def to_json(self) -> str:
        return json.dumps(self.to_dict(), sort_keys=True)


def _coerce(value: str, target: Any):
    if isinstance(target, bool):
        return value.lower() in ("1", "true", "yes", "on")
    if isinstance(target, int) and not isinstance(target, bool):
        return int(float(value))
    if isinstance(target, float):
        return float(value)
    if isinstance(target, tuple):
        v = yaml.safe_load(value)
        return tuple(v) if isinstance(v, (list, tuple)) else (v,)
    if target is None:
        return yaml.safe_load(value)
    return value


def _merge(dc, updates: dict):
    for k, v in updates.items():
        if not hasattr(dc, k):
            raise KeyError(f"unknown config key '{k}' in {type(dc).__name__}")
        cur = getattr(dc, k)
        if dataclasses.is_dataclass(cur):
            _merge(cur, v)
        else:
            if isinstance(cur, tuple) and isinstance(v, list):
                v = tuple(v)
            setattr(dc, k, v)
    return dc


def apply_overrides(cfg: ExperimentConfig, overrides: list[str]) -> ExperimentConfig:
    """Apply ``section.key=value`` overrides (Hydra style). Reference flat keys resolve too."""
    flat_alias = _flat_aliases()
    for ov in overrides:
        if "=" not in ov:
            raise ValueError(f"override '{ov}' is not key=value")
        key, value = ov.split("=", 1)
        key = key.strip().lstrip("+")
        if "." not in key and key in flat_alias:
            key = flat_alias[key]
        obj = cfg
        parts = key.split(".")
        for p in parts[:-1]:
            obj = getattr(obj, p)
        if not hasattr(obj, parts[-1]):
            raise KeyError(f"unknown config key '{key}'")
        setattr(obj, parts[-1], _coerce(value, getattr(obj, parts[-1])))
    return cfg


def _flat_aliases() -> dict:
    out = {}
    for sec in ("data", "model", "train", "privacy", "noise", "runtime"):
        dc = getattr(ExperimentConfig(), sec)
        for f in dataclasses.fields(dc):
            out.setdefault(f.name, f"{sec}.{f.name}")
    return out


def load_config(path: Optional[str] = None, overrides: Optional[list[str]] = None) -> ExperimentConfig:
    cfg = ExperimentConfig()
    if path:
        with open(path) as f:
            raw = yaml.safe_load(f) or {}
        # accept flat reference-style dicts too
        nested: dict = {}
        aliases = _flat_aliases()
        for k, v in raw.items():
            if isinstance(v, dict) and k in ("data", "model", "train", "privacy", "noise", "runtime"):
                nested.setdefault(k, {}).update(v)
            elif k == "name":
                nested["name"] = v
            elif k in aliases:
                sec, key = aliases[k].split(".")
                nested.setdefault(sec, {})[key] = v
            else:
                raise KeyError(f"unknown config key '{k}' in {path}")
        name = nested.pop("name", None)
        _merge(cfg, nested)
        if name:
            cfg.name = name
    if overrides:
        apply_overrides(cfg, overrides)
    return cfg


def save_config(cfg: ExperimentConfig, path: str) -> None:
    with open(path, "w") as f:
        yaml.safe_dump(json.loads(cfg.to_json()), f, sort_keys=True)
