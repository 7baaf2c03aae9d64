"""Synthetic data generators (MNIST images are absent from the reference snapshot,
``.MISSING_LARGE_BLOBS:4-5``; only the label files ship).

* ``synthetic_digit_images(labels)`` - deterministic 28x28 uint8 "digit-like" images: a per-class
  stroke template (seven-segment style glyph) + random affine jitter + noise.  Paired with the
  REAL reference label files this reproduces the reference pipeline's split sizes exactly
  (train 16 760 / val 1 863 / test 3 147 for digits 0/1/2), since those depend only on labels.
* ``write_synthetic_mnist(raw_folder, label_source)`` - writes the 4 IDX files.
* ``synthetic_client_shards`` - feature-space non-IID shards for VQC benchmarks: class-conditional
  Gaussians in [0,1]^F with Dirichlet(alpha) label skew and Dirichlet quantity skew per client,
  keyed by (seed, client) so any rank can build any client's shard independently.
"""
from __future__ import annotations

import os
from typing import Optional

import numpy as np
import torch

from ..utils.seeding import np_rng
from .idx import read_idx_labels, write_idx_images, write_idx_labels

# seven-segment-ish glyph segments: (r0, c0, r1, c1) boxes on a 28x28 canvas
_SEG = {
    "a": (4, 8, 6, 20), "b": (5, 18, 14, 20), "c": (14, 18, 23, 20), "d": (22, 8, 24, 20),
    "e": (14, 7, 23, 9), "f": (5, 7, 14, 9), "g": (13, 8, 15, 20),
}
_DIGIT_SEGS = {
    0: "abcdef", 1: "bc", 2: "abged", 3: "abgcd", 4: "fgbc",
    5: "afgcd", 6: "afgedc", 7: "abc", 8: "abcdefg", 9: "abcdfg",
}


def _template(d: int) -> np.ndarray:
    img = np.zeros((28, 28), np.float32)
    for s in _DIGIT_SEGS[int(d) % 10]:
        r0, c0, r1, c1 = _SEG[s]
        img[r0:r1, c0:c1] = 1.0
    return img


def synthetic_digit_images(labels: np.ndarray, seed: int = 0) -> np.ndarray:
    labels = np.asarray(labels)
    rng = np_rng(seed, "synthetic", 0)
    n = labels.shape[0]
    out = np.empty((n, 28, 28), np.uint8)
    temps = {d: _template(d) for d in range(10)}
    shifts = rng.integers(-3, 4, size=(n, 2))
    gains = rng.uniform(0.7, 1.0, size=n)
    for i in range(n):
        img = np.roll(temps[int(labels[i]) % 10], tuple(shifts[i]), axis=(0, 1))
        noise = rng.normal(0.0, 0.12, size=(28, 28)).astype(np.float32)
        out[i] = np.clip((img * gains[i] + noise) * 255.0, 0, 255).astype(np.uint8)
    return out


def write_synthetic_mnist(raw_folder: str, label_source: Optional[str] = None, seed: int = 0,
                          n_train: int = 60000, n_test: int = 10000) -> dict:
    """Write train/t10k IDX files; labels copied from ``label_source`` dir when available."""
    os.makedirs(raw_folder, exist_ok=True)
    paths = {}
    for split, n in (("train", n_train), ("t10k", n_test)):
        lab_name = f"{split}-labels.idx1-ubyte"
        img_name = f"{split}-images.idx3-ubyte"
        src = os.path.join(label_source, lab_name) if label_source else None
        if src and os.path.exists(src):
            labels = read_idx_labels(src)
        else:
            labels = np_rng(seed, "synthetic", 1 if split == "train" else 2).integers(0, 10, size=n).astype(np.uint8)
        write_idx_labels(os.path.join(raw_folder, lab_name), labels)
        write_idx_images(os.path.join(raw_folder, img_name),
                         synthetic_digit_images(labels, seed + (0 if split == "train" else 1)))
        paths[split] = (os.path.join(raw_folder, img_name), os.path.join(raw_folder, lab_name))
    return paths


def _class_means(n_classes: int, n_features: int, seed: int) -> np.ndarray:
    rng = np_rng(seed, "synthetic", 100)
    return rng.uniform(0.15, 0.85, size=(n_classes, n_features))


def synthetic_client_shard(client: int, num_clients: int, n_features: int, n_classes: int,
                           samples: int, alpha: float = 0.5, seed: int = 0,
                           non_iid: bool = True, spread: float = 0.12,
                           quantity_skew: bool = False) -> tuple[torch.Tensor, torch.Tensor]:
    """One client's (X [n, F] float32 in [0,1], y [n] int64).  Independent of other clients."""
    means = _class_means(n_classes, n_features, seed)
    rng = np_rng(seed, "synthetic", 1000 + client)
    if non_iid:
        probs = rng.dirichlet([alpha] * n_classes)
    else:
        probs = np.full(n_classes, 1.0 / n_classes)
    n = samples
    if quantity_skew:
        n = max(8, int(samples * rng.uniform(0.5, 1.5)))
    y = rng.choice(n_classes, size=n, p=probs)
    X = means[y] + rng.normal(0.0, spread, size=(n, n_features))
    X = np.clip(X, 0.0, 1.0)
    return torch.from_numpy(X.astype(np.float32)), torch.from_numpy(y.astype(np.int64))


def synthetic_test_set(n_features: int, n_classes: int, samples: int, seed: int = 0,
                       spread: float = 0.12) -> tuple[torch.Tensor, torch.Tensor]:
    means = _class_means(n_classes, n_features, seed)
    rng = np_rng(seed, "synthetic", 999)
    y = rng.integers(0, n_classes, size=samples)
    X = np.clip(means[y] + rng.normal(0.0, spread, size=(samples, n_features)), 0.0, 1.0)
    return torch.from_numpy(X.astype(np.float32)), torch.from_numpy(y.astype(np.int64))


def synthetic_client_shards(num_clients: int, n_features: int, n_classes: int, samples: int,
                            alpha: float = 0.5, seed: int = 0, non_iid: bool = True,
                            clients: Optional[list[int]] = None, **kw):
    ids = range(num_clients) if clients is None else clients
    return [synthetic_client_shard(c, num_clients, n_features, n_classes, samples, alpha, seed,
                                   non_iid, **kw) for c in ids]


def synthetic_images_shards(num_clients: int, n_classes: int, samples: int, alpha: float = 0.5,
                            seed: int = 0, clients: Optional[list[int]] = None):
    """Image-space (MNIST-shaped [n,1,28,28]) non-IID shards for the CFed TinyCNN path."""
    out = []
    ids = range(num_clients) if clients is None else clients
    for c in ids:
        rng = np_rng(seed, "synthetic", 5000 + c)
        probs = rng.dirichlet([alpha] * n_classes)
        y = rng.choice(n_classes, size=samples, p=probs).astype(np.int64)
        imgs = synthetic_digit_images(y, seed=seed * 7919 + c)
        X = torch.from_numpy(imgs.astype(np.float32) / 255.0)[:, None]
        out.append((X, torch.from_numpy(y)))
    return out
