"""Dataset builders that return federated client shards + a held-out test set.

Sources (ROADMAP.md:17-24, 102-103): MNIST (IDX -> digit filter -> features), Iris (4 features,
4 qubits; sklearn ships it offline), and synthetic non-IID shards (benchmarks).
Every builder returns a ``FederatedData``: per-client (X, y) torch tensors in feature space plus
(X_test, y_test).  Shards are built per client id so a rank only materialises its own clients.
"""
from __future__ import annotations

import os
from dataclasses import dataclass
from typing import Optional

import numpy as np
import torch

from ..utils.seeding import np_rng
from .features import make_features
from .partition import partition
from .synthetic import (synthetic_client_shards, synthetic_images_shards, synthetic_test_set,
                        synthetic_digit_images)


@dataclass
class FederatedData:
    clients: list                # list[(X [n_k, ...] float32, y [n_k] int64)] for the requested ids
    client_ids: list
    test: tuple                  # (X_test, y_test)
    n_classes: int
    n_features: int
    num_clients: int
    transformer: Optional[object] = None

    def sizes(self) -> list[int]:
        return [int(c[1].shape[0]) for c in self.clients]


def load_iris_federated(num_clients: int, partition_type: str = "iid", alpha: float = 0.5,
                        seed: int = 42, test_fraction: float = 0.3,
                        clients: Optional[list[int]] = None) -> FederatedData:
    from sklearn.datasets import load_iris
    from sklearn.model_selection import train_test_split
    d = load_iris()
    X = d.data.astype(np.float32)
    y = d.target.astype(np.int64)
    X = (X - X.min(0)) / (X.max(0) - X.min(0))  # -> [0,1]
    Xtr, Xte, ytr, yte = train_test_split(X, y, test_size=test_fraction, stratify=y, random_state=seed)
    parts = partition(Xtr, ytr, num_clients, partition_type, alpha, np_rng(seed, "partition"))
    ids = list(range(num_clients)) if clients is None else clients
    shards = [(torch.from_numpy(parts[i][0]), torch.from_numpy(parts[i][1])) for i in ids]
    return FederatedData(shards, ids, (torch.from_numpy(Xte), torch.from_numpy(yte)), 3, 4, num_clients)


def load_mnist_federated(raw_folder: str, num_clients: int, digits=(0, 1, 2),
                         partition_type: str = "iid", alpha: float = 0.5, features: str = "pool",
                         n_features: int = 4, seed: int = 42, val_split: float = 0.1,
                         clients: Optional[list[int]] = None, keep_images: bool = False) -> FederatedData:
    from .idx import read_idx_images, read_idx_labels
    from .mnist import FILES, stratified_split
    Xtr = read_idx_images(os.path.join(raw_folder, FILES["train_images"]))
    ytr = read_idx_labels(os.path.join(raw_folder, FILES["train_labels"]))
    Xte = read_idx_images(os.path.join(raw_folder, FILES["test_images"]))
    yte = read_idx_labels(os.path.join(raw_folder, FILES["test_labels"]))
    mtr, mte = np.isin(ytr, digits), np.isin(yte, digits)
    Xtr = (Xtr[mtr].astype(np.float32) / 255.0)[:, None]
    Xte = (Xte[mte].astype(np.float32) / 255.0)[:, None]
    # labels re-indexed 0..C-1 in digit order
    remap = {d: i for i, d in enumerate(digits)}
    ytr = np.array([remap[int(v)] for v in ytr[mtr]], np.int64)
    yte = np.array([remap[int(v)] for v in yte[mte]], np.int64)
    Xtr, _, ytr, _ = stratified_split(Xtr, ytr, val_split, 42)
    parts = partition(Xtr, ytr, num_clients, partition_type, alpha, np_rng(seed, "partition"))
    ids = list(range(num_clients)) if clients is None else clients
    if keep_images:
        shards = [(torch.from_numpy(np.ascontiguousarray(parts[i][0])), torch.from_numpy(parts[i][1])) for i in ids]
        return FederatedData(shards, ids, (torch.from_numpy(Xte), torch.from_numpy(yte)),
                             len(digits), 28 * 28, num_clients)
    Ftr_all, tf = make_features(torch.from_numpy(Xtr), features, n_features)
    # features computed per client with the transformer fitted on the full training split
    shards = []
    for i in ids:
        f, _ = make_features(torch.from_numpy(np.ascontiguousarray(parts[i][0])), features, n_features, tf)
        shards.append((f, torch.from_numpy(parts[i][1])))
    fte, _ = make_features(torch.from_numpy(Xte), features, n_features, tf)
    return FederatedData(shards, ids, (fte, torch.from_numpy(yte)), len(digits), n_features,
                         num_clients, tf)


def load_synthetic_federated(num_clients: int, n_features: int, n_classes: int,
                             samples_per_client: int, test_samples: int, alpha: float = 0.5,
                             seed: int = 42, non_iid: bool = True,
                             clients: Optional[list[int]] = None) -> FederatedData:
    ids = list(range(num_clients)) if clients is None else clients
    shards = synthetic_client_shards(num_clients, n_features, n_classes, samples_per_client,
                                     alpha, seed, non_iid, clients=ids)
    test = synthetic_test_set(n_features, n_classes, test_samples, seed)
    return FederatedData(shards, ids, test, n_classes, n_features, num_clients)


def load_synthetic_images_federated(num_clients: int, n_classes: int, samples_per_client: int,
                                    test_samples: int, alpha: float = 0.5, seed: int = 42,
                                    clients: Optional[list[int]] = None) -> FederatedData:
    ids = list(range(num_clients)) if clients is None else clients
    shards = synthetic_images_shards(num_clients, n_classes, samples_per_client, alpha, seed, ids)
    rng = np_rng(seed, "synthetic", 77)
    yt = rng.integers(0, n_classes, size=test_samples).astype(np.int64)
    Xt = torch.from_numpy(synthetic_digit_images(yt, seed + 17).astype(np.float32) / 255.0)[:, None]
    return FederatedData(shards, ids, (Xt, torch.from_numpy(yt)), n_classes, 28 * 28, num_clients)


def load_synthetic_digits_federated(num_clients: int, n_classes: int, samples_per_client: int, test_samples: int,
                                    alpha: float, seed: int, features: str, n_features: int, images: bool,
                                    clients: Optional[list[int]] = None) -> FederatedData:
    """Synthetic MNIST-like digit images (the images of MNIST are absent offline), the SAME shards for the TinyCNN
    (images) and the VQC (``features``, e.g. PCA to n_qubits, fitted on the full training set) - the data of the
    ROADMAP.md:104-109 VQC vs classical-FL comparison."""
    base = load_synthetic_images_federated(num_clients, n_classes, samples_per_client, test_samples, alpha, seed,
                                           clients)
    if images:
        return base
    every = synthetic_images_shards(num_clients, n_classes, samples_per_client, alpha, seed)
    _, tf = make_features(torch.cat([x for x, _ in every]), features, n_features)
    shards = [(make_features(x, features, n_features, tf)[0], y) for x, y in base.clients]
    Xt, yt = base.test
    return FederatedData(shards, base.client_ids, (make_features(Xt, features, n_features, tf)[0], yt), n_classes,
                         n_features, num_clients, tf)


def pool_clients(data: FederatedData, keep: bool) -> FederatedData:
    """Centralized baseline (ROADMAP.md:109): every client's shard pooled into ONE client (id 0), held by the
    rank with ``keep``; FedAvg over one client trained on all the data is centralized training, and the round
    loop, optimizer, DP and evaluation stay exactly those of the federated runs it is compared with."""
    X = torch.cat([x for x, _ in data.clients]) if data.clients else None
    y = torch.cat([t for _, t in data.clients]) if data.clients else None
    clients = [(X, y)] if keep else []
    return FederatedData(clients, [0] if keep else [], data.test, data.n_classes, data.n_features, 1,
                         data.transformer)


def build_federated_data(cfg, clients: Optional[list[int]] = None, images: bool = False) -> FederatedData:
    """Dispatch on ``cfg.data.dataset`` (ExperimentConfig).  ``train.mode=centralized`` pools every client's
    shard into one client (``pool_clients``); ``clients`` then only says whether this rank holds it (rank 0)."""
    if getattr(cfg.train, "mode", "federated") == "centralized":
        import copy
        c2 = copy.deepcopy(cfg)
        c2.train.mode = "federated"
        return pool_clients(build_federated_data(c2, None, images), clients is None or 0 in clients)
    d, m, t = cfg.data, cfg.model, cfg.train
    non_iid = d.partition_type.lower() != "iid"
    amp = getattr(m, "kind", "vqc") == "vqc" and str(getattr(m, "feature_map", "")).lower() == "amplitude"
    nf = d.n_features if d.n_features > 0 else ((1 << m.n_qubits) if amp else m.n_qubits)
    if d.dataset == "synthetic_digits":
        return load_synthetic_digits_federated(d.num_clients, m.n_classes, d.samples_per_client, d.test_samples,
                                               d.alpha, t.seed, d.features, nf, images or m.kind == "tinycnn",
                                               clients)
    if d.dataset == "synthetic":
        if images or m.kind == "tinycnn":
            return load_synthetic_images_federated(d.num_clients, m.n_classes, d.samples_per_client,
                                                   d.test_samples, d.alpha, t.seed, clients)
        return load_synthetic_federated(d.num_clients, nf,
                                        m.n_classes, d.samples_per_client, d.test_samples, d.alpha,
                                        t.seed, non_iid, clients)
    if d.dataset == "iris":
        return load_iris_federated(d.num_clients, d.partition_type, d.alpha, t.seed, clients=clients)
    if d.dataset == "mnist":
        return load_mnist_federated(d.raw_folder, d.num_clients, tuple(d.digits), d.partition_type,
                                    d.alpha, d.features, nf, t.seed, d.val_split, clients,
                                    keep_images=images or m.kind == "tinycnn")
    raise ValueError(f"unknown dataset '{d.dataset}'")
