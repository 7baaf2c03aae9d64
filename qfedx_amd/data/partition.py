"""Client partitioners: IID and Dirichlet non-IID.

Reference: ``create_iid_partition`` (``src/CFed/Preprocess.py:23-37``) shuffles indices with the
GLOBAL python ``random`` and gives ``n//K`` items per client, the remainder to the last;
``create_non_iid_partition`` (``:40-68``) draws, per class, ``np.random.dirichlet([alpha]*K)``
and gives ``int(len*p_k)`` items per client, the remainder to the last.

Parity: when no ``rng`` is passed the same global generators are consumed in the same order, so
``random.seed(s); np.random.seed(s)`` reproduces the reference partition exactly.

Fixed quirks:
  * #3: the reference loops ``for class_label in range(num_classes)`` (``:51``), which drops all
    data when the digit set is not ``{0..C-1}`` (digits=(3,5) keeps 0 of 11 552 samples).  Here the
    loop runs over the sorted ACTUAL labels - identical RNG call sequence for contiguous labels.
  * #4: any ``partition_type`` other than ``'iid'`` silently became non-IID (``:213``); unknown
    types now raise.
"""
from __future__ import annotations

import random
from collections import defaultdict
from typing import Optional

import numpy as np

NON_IID_ALIASES = ("non_iid", "noniid", "non-iid", "dirichlet")


def create_iid_partition(X_data, y_data, num_clients: int, rng: Optional[np.random.Generator] = None):
    indices = list(range(len(X_data)))
    if rng is None:
        random.shuffle(indices)
    else:
        indices = list(rng.permutation(len(X_data)))
    num_items = len(X_data) // num_clients
    client_data = []
    for i in range(num_clients):
        start = i * num_items
        end = len(X_data) if i == num_clients - 1 else (i + 1) * num_items
        idx = indices[start:end]
        client_data.append((X_data[idx], y_data[idx]))
    return client_data


def dirichlet_indices(y_data, num_clients: int, alpha: float = 0.5,
                      rng: Optional[np.random.Generator] = None) -> list[list[int]]:
    """Per-client index lists of a Dirichlet(alpha) label-skew partition."""
    y = np.asarray(y_data)
    class_indices = defaultdict(list)
    for idx, label in enumerate(y.tolist()):
        class_indices[label].append(idx)
    client_indices: list[list[int]] = [[] for _ in range(num_clients)]
    for class_label in sorted(class_indices.keys()):
        class_data = class_indices[class_label]
        if rng is None:
            random.shuffle(class_data)
            proportions = np.random.dirichlet([alpha] * num_clients)
        else:
            class_data = [class_data[i] for i in rng.permutation(len(class_data))]
            proportions = rng.dirichlet([alpha] * num_clients)
        start = 0
        for cid in range(num_clients):
            end = start + int(len(class_data) * proportions[cid])
            if cid == num_clients - 1:
                end = len(class_data)
            client_indices[cid].extend(class_data[start:end])
            start = end
    return client_indices


def create_non_iid_partition(X_data, y_data, num_clients: int, alpha: float = 0.5,
                             rng: Optional[np.random.Generator] = None):
    parts = dirichlet_indices(y_data, num_clients, alpha, rng)
    return [(X_data[idx], y_data[idx]) for idx in parts]


def partition(X_data, y_data, num_clients: int, partition_type: str = "iid", alpha: float = 0.5,
              rng: Optional[np.random.Generator] = None):
    pt = partition_type.lower()
    if pt == "iid":
        return create_iid_partition(X_data, y_data, num_clients, rng)
    if pt in NON_IID_ALIASES:
        return create_non_iid_partition(X_data, y_data, num_clients, alpha, rng)
    raise ValueError(f"unknown partition_type '{partition_type}' (use 'iid' or 'non_iid')")
