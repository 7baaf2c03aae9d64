"""MNIST preprocessing pipeline (``src/CFed/Preprocess.py:137-228``).

Behaviour kept: loads the 4 IDX files (``:157-167``), returns ``None`` on ``FileNotFoundError``
(``:170-172``), digit filter + /255 float32 + channel dim -> [N,1,28,28] (``:176-182``), stratified
``train_test_split(test_size=val_split, random_state=42)`` (``:187-189``), ``torch.save((X f32,
y int64))`` to ``{train,val,test}.pt`` (``:192-199``, bit-compatible layout), partitions
(``:212-214``), the two plots (``:223-224``), returns ``(train, val, test, client_data)`` (``:228``).

Fixed: client shards are returned as torch tensors with int64 labels - the
reference returned numpy arrays with uint8 labels, which crashed ``client_update``'s ``.to()``
(``Classical_FL.py:48``).  ``return_numpy=True`` restores the old types.
"""
from __future__ import annotations

import os
from pathlib import Path
from typing import Optional

import numpy as np
import torch

from .idx import read_idx_images, read_idx_labels
from .partition import partition as _partition
from .viz import plot_class_distribution, visualize_client_data

FILES = {
    "train_images": "train-images.idx3-ubyte",
    "train_labels": "train-labels.idx1-ubyte",
    "test_images": "t10k-images.idx3-ubyte",
    "test_labels": "t10k-labels.idx1-ubyte",
}


def stratified_split(X: np.ndarray, y: np.ndarray, val_split: float, random_state: int = 42):
    from sklearn.model_selection import train_test_split
    return train_test_split(X, y, test_size=val_split, stratify=y, random_state=random_state)


def preprocess_mnist(raw_folder: str, processed_folder: str, digits=(0, 1, 2), val_split=0.1,
                     num_clients=4, partition_type="iid", alpha=0.5, plots: bool = True,
                     results_folder: str = "./results", return_numpy: bool = False,
                     rng: Optional[np.random.Generator] = None, verbose: bool = True):
    Path(processed_folder).mkdir(parents=True, exist_ok=True)
    if plots:
        Path(results_folder).mkdir(parents=True, exist_ok=True)
    try:
        X_train = read_idx_images(os.path.join(raw_folder, FILES["train_images"]))
        y_train = read_idx_labels(os.path.join(raw_folder, FILES["train_labels"]))
        X_test = read_idx_images(os.path.join(raw_folder, FILES["test_images"]))
        y_test = read_idx_labels(os.path.join(raw_folder, FILES["test_labels"]))
        if verbose:
            print(f"\nRaw data loaded: Train {X_train.shape}, Test {X_test.shape}")
    except FileNotFoundError as e:
        print(f"Error loading raw data: {e}")
        return None

    train_mask = np.isin(y_train, digits)
    test_mask = np.isin(y_test, digits)
    X_train = (X_train[train_mask].astype(np.float32) / 255.0)[:, None, :, :]
    y_train = y_train[train_mask]
    X_test = (X_test[test_mask].astype(np.float32) / 255.0)[:, None, :, :]
    y_test = y_test[test_mask]

    X_train, X_val, y_train, y_val = stratified_split(X_train, y_train, val_split, 42)

    datasets = {
        "train": (torch.tensor(X_train), torch.tensor(y_train, dtype=torch.long)),
        "val": (torch.tensor(X_val), torch.tensor(y_val, dtype=torch.long)),
        "test": (torch.tensor(X_test), torch.tensor(y_test, dtype=torch.long)),
    }
    for name, data in datasets.items():
        torch.save(data, os.path.join(processed_folder, f"{name}.pt"))

    if verbose:
        for split_name, y_split in (("Train", y_train), ("Val", y_val), ("Test", y_test)):
            u, c = np.unique(y_split, return_counts=True)
            print(f"  {split_name}: " + ", ".join(f"Digit {a}: {b}" for a, b in zip(u, c)))

    client_np = _partition(X_train, y_train, num_clients, partition_type, alpha, rng)
    if plots:
        visualize_client_data(client_np, os.path.join(results_folder, "client_samples.png"))
        plot_class_distribution(client_np, os.path.join(results_folder, "class_distribution.png"))
    if return_numpy:
        client_data = client_np
    else:
        client_data = [(torch.from_numpy(np.ascontiguousarray(Xc)),
                        torch.from_numpy(np.ascontiguousarray(yc).astype(np.int64)))
                       for Xc, yc in client_np]
    return datasets["train"], datasets["val"], datasets["test"], client_data


def load_processed(processed_folder: str, split: str):
    """Load a ``{split}.pt`` tuple safely (weights_only)."""
    return torch.load(os.path.join(processed_folder, f"{split}.pt"), weights_only=True)
