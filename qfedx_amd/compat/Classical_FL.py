"""``src/CFed/Classical_FL.py`` API (reference ``Classical_FL.py:12-218``) on the client-batched engine.

Same names, signatures and return shapes as the reference: ``set_seeds``, ``device``, ``TinyCNN``,
``client_update -> (state_dict, n)``, ``federated_averaging``, ``evaluate_model -> float``,
``federated_learning -> {'model', 'accuracies'}``, ``main``.  Differences (all reference bugs, SURVEY
§2.1): client shards may be numpy or torch (C16 crash), the class count is read from the weights
instead of hard-coded 3 (C12), evaluation does not sync per batch (C14), and clients of a round
train as one batched job instead of a sequential loop (C15).  Unlike the reference, ``set_seeds`` is
not called at import time (C9) - entry points seed explicitly.
"""
from __future__ import annotations

import numpy as np
import torch

from ..config import ExperimentConfig
from ..data.datasets import FederatedData
from ..fl.aggregator import federated_averaging  # noqa: F401  (C13, Classical_FL.py:66-81)
from ..fl.cnn_adapter import CNNClientTrainer, TinyCNNAdapter
from ..fl.server import FederatedRunner
from ..fl.trainer import ShardStore
from ..models import tinycnn as tc
from ..models.tinycnn import TinyCNN  # noqa: F401  (C11, Classical_FL.py:21-38)
from ..parallel.dist import World
from ..utils.device import resolve_backend, resolve_device
from ..utils.seeding import set_seeds  # noqa: F401  (C9, Classical_FL.py:12-18)


def __getattr__(name):
    # reference's module-global ``device`` (C10, :19), resolved lazily so importing does not touch the GPU
    if name == "device":
        return resolve_device("auto")
    raise AttributeError(name)


def _as_tensors(data):
    X, y = data
    X = torch.as_tensor(np.asarray(X) if not torch.is_tensor(X) else X, dtype=torch.float32)
    y = torch.as_tensor(np.asarray(y) if not torch.is_tensor(y) else y).long()
    if X.dim() == 3:
        X = X[:, None]
    return X, y


def _train_cfg(epochs, lr, batch_size, seed=42):
    cfg = ExperimentConfig()
    cfg.model.kind = "tinycnn"
    cfg.train.optimizer = "sgd"          # fresh SGD(lr, momentum=0.9) per round (:53)
    cfg.train.momentum = 0.9
    cfg.train.learning_rate = lr
    cfg.train.local_epochs = epochs
    cfg.train.batch_size = batch_size
    cfg.train.aggregate = "weights"       # FedAvg of weights (:66-81)
    cfg.train.wrap_angles = False
    cfg.train.seed = seed
    return cfg


def client_update(model_params: dict, client_data, epochs: int = 5, lr: float = 0.01, batch_size: int = 32,
                  round_num: int = 0, seed: int = 42):
    """C12 (``Classical_FL.py:40-64``): train one client from ``model_params``; returns (state_dict, n)."""
    dev = resolve_device("auto")
    backend = resolve_backend("auto", dev)
    C = int(model_params["fc2.bias"].shape[0])
    X, y = _as_tensors(client_data)
    cfg = _train_cfg(epochs, lr, batch_size, seed)
    trainer = CNNClientTrainer(C, cfg.train, dev, backend)
    store = ShardStore([(X, y)], [0], dev)
    flat = tc.state_dict_to_flat({k: v.detach().cpu() for k, v in model_params.items()}, C).to(dev)
    res = trainer.run_round(store, [0], flat, round_num)
    return tc.flat_to_state_dict(res["params"][0].detach().cpu(), C), int(y.shape[0])


@torch.no_grad()
def evaluate_model(model: torch.nn.Module, test_data, batch_size: int = 256) -> float:
    """C14 (``Classical_FL.py:83-102``): argmax accuracy; correct counts stay on device until the end."""
    X, y = _as_tensors(test_data)
    dev = next(model.parameters()).device
    model.eval()
    correct = torch.zeros((), dtype=torch.int64, device=dev)
    for s in range(0, X.shape[0], batch_size):
        xb = X[s: s + batch_size].to(dev)
        yb = y[s: s + batch_size].to(dev)
        correct += (model(xb).argmax(-1) == yb).sum()
    return float(correct) / max(int(X.shape[0]), 1)


def federated_learning(client_data, test_data, num_rounds: int = 30, local_epochs: int = 5,
                       learning_rate: float = 0.01, batch_size: int = 32, num_classes: int = 3,
                       seed: int = 42, log_every: int = 5) -> dict:
    """C15 (``Classical_FL.py:104-157``): round-0 eval, then ``num_rounds`` of (all clients train ->
    FedAvg -> test eval); returns ``{'model': TinyCNN, 'accuracies': [round0, ..., roundR]}``."""
    dev = resolve_device("auto")
    backend = resolve_backend("auto", dev)
    cfg = _train_cfg(local_epochs, learning_rate, batch_size, seed)
    cfg.train.num_rounds = num_rounds
    cfg.model.n_classes = num_classes
    cfg.data.num_clients = len(client_data)
    cfg.runtime.log_every = log_every
    shards = [_as_tensors(c) for c in client_data]
    data = FederatedData(shards, list(range(len(shards))), _as_tensors(test_data), num_classes, 28 * 28,
                         len(shards))
    adapter = TinyCNNAdapter(cfg, dev, backend)
    runner = FederatedRunner(cfg, adapter, data, World(0, 1, 0, "none", dev), dev, backend)
    out = runner.run()
    model = TinyCNN(num_classes)
    model.load_state_dict(out["model"])
    return {"model": model.to(dev), "accuracies": out["accuracies"], "history": out["history"]}


def main(raw_folder: str = "./dataset/raw", processed_folder: str = "./dataset/processed", **overrides):
    """C16 (``Classical_FL.py:159-218``): the reference's config dict -> preprocess -> federated learning."""
    config = {"raw_folder": raw_folder, "processed_folder": processed_folder, "digits": (0, 1, 2),
              "val_split": 0.1, "num_clients": 4, "partition_type": "iid", "alpha": 0.5, "num_rounds": 30,
              "local_epochs": 5, "learning_rate": 0.01, "batch_size": 32}
    config.update(overrides)
    set_seeds(42)
    from ..data.mnist import preprocess_mnist
    out = preprocess_mnist(config["raw_folder"], config["processed_folder"], config["digits"],
                           config["val_split"], config["num_clients"], config["partition_type"], config["alpha"],
                           plots=False)
    if out is None:
        print("Preprocessing failed: MNIST IDX files not found.")
        return None
    train_data, val_data, test_data, client_data = out
    return federated_learning(client_data, test_data, config["num_rounds"], config["local_epochs"],
                              config["learning_rate"], config["batch_size"], len(config["digits"]))
