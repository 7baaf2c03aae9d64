"""High-level entry: ``run_experiment(cfg)`` = device/world setup -> this rank's client shards ->
model adapter -> federated runner.  Works single-process, under ``torchrun`` (one process per GPU,
RCCL), and on CPU with gloo (north-star config 1).
"""
from __future__ import annotations

import torch

from .config import ExperimentConfig
from .data.datasets import build_federated_data
from .fl.adapters import make_adapter
from .fl.server import FederatedRunner
from .parallel.dist import init_distributed, shard_clients
from .utils.device import resolve_backend, resolve_device
from .utils.seeding import set_seeds


def setup(cfg: ExperimentConfig):
    device = resolve_device(cfg.runtime.device)
    backend = resolve_backend(cfg.runtime.backend, device)
    world = init_distributed(device, cfg.runtime.dist_backend)
    return device, backend, world


def run_experiment(cfg: ExperimentConfig, world=None, device=None, backend=None) -> dict:
    set_seeds(cfg.train.seed)
    if world is None:
        device, backend, world = setup(cfg)
    n_clients = 1 if getattr(cfg.train, "mode", "federated") == "centralized" else cfg.data.num_clients
    my_clients = shard_clients(n_clients, world.world_size, world.rank)
    data = build_federated_data(cfg, clients=my_clients)
    adapter = make_adapter(cfg, device, backend)
    runner = FederatedRunner(cfg, adapter, data, world, device, backend)
    out = runner.run()
    out["world_size"] = world.world_size
    out["backend"] = backend
    out["device"] = str(device)
    out["simulator"] = getattr(adapter, "simulator", None)     # statevector | mps | density (VQC adapters)
    return out
