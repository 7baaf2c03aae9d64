"""Plots: client sample grid, class distribution (``src/CFed/Preprocess.py:71-134``) and the
ROADMAP reporting plots (accuracy vs epsilon / qubits, speedup vs clients, ``ROADMAP.md:120``).
Uses the non-interactive Agg backend (the reference's ``plt.show()`` blocks, ``testEncoder.py:109``).
"""
from __future__ import annotations

from pathlib import Path

import numpy as np


def _plt():
    import matplotlib
    matplotlib.use("Agg")
    import matplotlib.pyplot as plt
    return plt


def _np(a):
    try:
        import torch
        if isinstance(a, torch.Tensor):
            return a.detach().cpu().numpy()
    except ImportError:  # pragma: no cover
        pass
    return np.asarray(a)


def visualize_client_data(client_data, save_path="./results/client_samples.png", samples_per_client=5):
    plt = _plt()
    Path(save_path).parent.mkdir(parents=True, exist_ok=True)
    num_clients = len(client_data)
    fig, axes = plt.subplots(num_clients, samples_per_client, figsize=(12, 2.5 * num_clients))
    axes = np.atleast_2d(axes)
    if num_clients == 1 and axes.shape[0] != 1:
        axes = axes[None, :]
    for i, (X_client, y_client) in enumerate(client_data):
        X_client, y_client = _np(X_client), _np(y_client)
        for j in range(samples_per_client):
            ax = axes[i, j]
            if j < len(X_client):
                image = X_client[j, 0] if X_client.ndim == 4 else X_client[j]
                ax.imshow(image, cmap="gray")
                ax.set_title(f"Label: {y_client[j]}")
            ax.axis("off")
    plt.suptitle("Sample Images from Each Client", fontsize=16)
    plt.tight_layout()
    plt.savefig(save_path, dpi=150, bbox_inches="tight")
    plt.close(fig)
    print(f"\nClient sample visualization saved to {save_path}")


def class_distribution(client_data) -> tuple[list, np.ndarray]:
    """(classes, counts[num_classes, num_clients]) - the matrix the bar chart plots."""
    all_classes = set()
    for _, y in client_data:
        all_classes.update(_np(y).tolist())
    classes = sorted(all_classes)
    dist = np.zeros((len(classes), len(client_data)), dtype=np.int64)
    pos = {c: i for i, c in enumerate(classes)}
    for k, (_, y) in enumerate(client_data):
        u, c = np.unique(_np(y), return_counts=True)
        for cls, cnt in zip(u.tolist(), c.tolist()):
            dist[pos[cls], k] = cnt
    return classes, dist


def plot_class_distribution(client_data, save_path="./results/class_distribution.png"):
    plt = _plt()
    Path(save_path).parent.mkdir(parents=True, exist_ok=True)
    classes, dist = class_distribution(client_data)
    names = [f"Client {i + 1}" for i in range(len(client_data))]
    colors = plt.cm.Set3(np.linspace(0, 1, max(1, len(classes))))
    fig, ax = plt.subplots(figsize=(10, 6))
    bottom = np.zeros(len(client_data))
    for i, cls in enumerate(classes):
        ax.bar(names, dist[i], bottom=bottom, label=f"Digit {cls}", color=colors[i], alpha=0.8)
        bottom += dist[i]
    ax.set_xlabel("Clients")
    ax.set_ylabel("Number of Samples")
    ax.set_title("Class Distribution Across Clients")
    ax.legend()
    plt.tight_layout()
    plt.savefig(save_path, dpi=150, bbox_inches="tight")
    plt.close(fig)
    print(f"Class distribution plot saved to {save_path}")


def plot_series(xs, ys_by_label: dict, xlabel: str, ylabel: str, title: str, save_path: str,
                yerr_by_label: dict | None = None):
    """Generic line plot used for acc-vs-eps, acc-vs-qubits, speedup-vs-clients (ROADMAP:120)."""
    plt = _plt()
    Path(save_path).parent.mkdir(parents=True, exist_ok=True)
    fig, ax = plt.subplots(figsize=(7, 4.5))
    for label, ys in ys_by_label.items():
        err = (yerr_by_label or {}).get(label)
        ax.errorbar(xs, ys, yerr=err, marker="o", capsize=3, label=label)
    ax.set_xlabel(xlabel)
    ax.set_ylabel(ylabel)
    ax.set_title(title)
    ax.grid(alpha=0.3)
    ax.legend()
    plt.tight_layout()
    plt.savefig(save_path, dpi=150)
    plt.close(fig)
