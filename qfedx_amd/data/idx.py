"""IDX (MNIST) file readers/writers.

Reference: ``read_idx_images`` skips a 16-byte header and reshapes to (-1, 28, 28) without
checking the magic number (``src/CFed/Preprocess.py:11-14``); ``read_idx_labels`` skips 8 bytes
(``:17-20``).  Same signatures and outputs here; ``strict=True`` additionally validates the
magic/dims header (the reference never does), and the writers let tests and the synthetic-data
generator produce byte-compatible files (the reference snapshot ships labels only,
``.MISSING_LARGE_BLOBS:1-5``).
"""
from __future__ import annotations

import os
import struct

import numpy as np

IMAGES_MAGIC = 0x00000803
LABELS_MAGIC = 0x00000801


def read_idx_images(filename: str, strict: bool = False) -> np.ndarray:
    with open(filename, "rb") as f:
        header = f.read(16)
        if strict:
            magic, n, h, w = struct.unpack(">IIII", header)
            if magic != IMAGES_MAGIC:
                raise ValueError(f"{filename}: bad IDX image magic {magic:#x}")
            data = np.frombuffer(f.read(), dtype=np.uint8)
            return data.reshape(n, h, w)
        return np.frombuffer(f.read(), dtype=np.uint8).reshape(-1, 28, 28)


def read_idx_labels(filename: str, strict: bool = False) -> np.ndarray:
    with open(filename, "rb") as f:
        header = f.read(8)
        if strict:
            magic, n = struct.unpack(">II", header)
            if magic != LABELS_MAGIC:
                raise ValueError(f"{filename}: bad IDX label magic {magic:#x}")
        return np.frombuffer(f.read(), dtype=np.uint8)


def write_idx_images(filename: str, images: np.ndarray) -> None:
    images = np.ascontiguousarray(images, dtype=np.uint8)
    n, h, w = images.shape
    os.makedirs(os.path.dirname(os.path.abspath(filename)), exist_ok=True)
    with open(filename, "wb") as f:
        f.write(struct.pack(">IIII", IMAGES_MAGIC, n, h, w))
        f.write(images.tobytes())


def write_idx_labels(filename: str, labels: np.ndarray) -> None:
    labels = np.ascontiguousarray(labels, dtype=np.uint8)
    os.makedirs(os.path.dirname(os.path.abspath(filename)), exist_ok=True)
    with open(filename, "wb") as f:
        f.write(struct.pack(">II", LABELS_MAGIC, labels.shape[0]))
        f.write(labels.tobytes())
