"""Feature pipelines feeding the quantum encoders.

* ``downsample_image`` - block average with floor boundaries and empty-block guard
  (``src/QFed/testEncoder.py:20-40``), plus a batched torch version (``downsample_batch``).
* ``pool_to_n_features`` - contiguous-chunk means, zero-pad when n >= L, last chunk absorbs the
  remainder (``src/QFed/qAngle.py:9-24``; duplicated verbatim at ``testEncoder.py:42-56`` - one
  copy here), plus a batched torch version.
* ``StandardPCA`` - standardize + PCA(k) with a saved transformer (``ROADMAP.md:17-19``).
* ``angle_scale`` - per-sample min-max to [0, pi] (reference ``qAngle.py:36-41``) or the ROADMAP
  global map ``alpha * x`` (``ROADMAP.md:126``).
"""
from __future__ import annotations

import math

import numpy as np
import torch


def downsample_image(img: np.ndarray, out_shape=(4, 4)) -> np.ndarray:
    img = np.asarray(img, dtype=float)
    in_h, in_w = img.shape
    out_h, out_w = out_shape
    h_step, w_step = in_h / out_h, in_w / out_w
    out = np.zeros(out_shape)
    for i in range(out_h):
        h0, h1 = int(np.floor(i * h_step)), int(np.floor((i + 1) * h_step))
        if h1 <= h0:
            h1 = min(in_h, h0 + 1)
        for j in range(out_w):
            w0, w1 = int(np.floor(j * w_step)), int(np.floor((j + 1) * w_step))
            if w1 <= w0:
                w1 = min(in_w, w0 + 1)
            patch = img[h0:h1, w0:w1]
            out[i, j] = patch.mean() if patch.size > 0 else 0.0
    return out


def _block_bounds(n_in: int, n_out: int) -> list[tuple[int, int]]:
    step = n_in / n_out
    out = []
    for i in range(n_out):
        a, b = int(math.floor(i * step)), int(math.floor((i + 1) * step))
        if b <= a:
            b = min(n_in, a + 1)
        out.append((a, b))
    return out


def downsample_batch(x: torch.Tensor, out_shape=(4, 4)) -> torch.Tensor:
    """[N, (1,) H, W] -> [N, oh*ow] with exactly ``downsample_image``'s block boundaries."""
    if x.dim() == 4:
        x = x[:, 0]
    n, h, w = x.shape
    oh, ow = out_shape
    # averaging matrices Ah [oh, h], Aw [ow, w]
    ah = torch.zeros(oh, h, dtype=torch.float64)
    for i, (a, b) in enumerate(_block_bounds(h, oh)):
        ah[i, a:b] = 1.0 / (b - a)
    aw = torch.zeros(ow, w, dtype=torch.float64)
    for j, (a, b) in enumerate(_block_bounds(w, ow)):
        aw[j, a:b] = 1.0 / (b - a)
    y = torch.einsum("ih,nhw,jw->nij", ah.to(x), x, aw.to(x))
    return y.reshape(n, oh * ow)


def pool_to_n_features(vec: np.ndarray, n_features: int) -> np.ndarray:
    v = np.asarray(vec, dtype=float).reshape(-1)
    L = v.size
    if n_features >= L:
        out = np.zeros(n_features)
        out[:L] = v
        return out
    chunk = L // n_features
    out = np.zeros(n_features)
    for i in range(n_features):
        start = i * chunk
        end = (i + 1) * chunk if i < n_features - 1 else L
        out[i] = v[start:end].mean()
    return out


def pool_batch(x: torch.Tensor, n_features: int) -> torch.Tensor:
    """Batched ``pool_to_n_features`` on [N, L] (identical chunking)."""
    x = x.reshape(x.shape[0], -1)
    n, L = x.shape
    if n_features >= L:
        out = x.new_zeros(n, n_features)
        out[:, :L] = x
        return out
    chunk = L // n_features
    m = torch.zeros(L, n_features, dtype=x.dtype, device=x.device)
    for i in range(n_features):
        a = i * chunk
        b = (i + 1) * chunk if i < n_features - 1 else L
        m[a:b, i] = 1.0 / (b - a)
    return x @ m


def angle_scale(x: torch.Tensor, mode: str = "scale", alpha: float = math.pi) -> torch.Tensor:
    """Map features to rotation angles.

    ``minmax``: reference per-sample min-max to [0,1] then * pi, constant rows -> 0
    (``qAngle.py:36-41``).  ``scale``: ``alpha * x`` (ROADMAP ``RY(alpha * x_i)``).
    """
    if mode == "minmax":
        mn = x.min(dim=-1, keepdim=True).values
        mx = x.max(dim=-1, keepdim=True).values
        rng = mx - mn
        normed = torch.where(rng > 0, (x - mn) / torch.where(rng > 0, rng, torch.ones_like(rng)),
                             torch.zeros_like(x))
        return normed * math.pi
    if mode == "scale":
        return alpha * x
    raise ValueError(f"unknown angle scaling '{mode}'")


class StandardPCA:
    """standardize -> PCA(k) transformer with save/load (ROADMAP.md:18 'save transformer')."""

    def __init__(self, n_components: int):
        self.k = n_components
        self.mean_ = None
        self.std_ = None
        self.components_ = None
        self.out_min_ = None
        self.out_max_ = None

    def fit(self, X: torch.Tensor) -> "StandardPCA":
        X = X.reshape(X.shape[0], -1).double()
        self.mean_ = X.mean(0)
        self.std_ = X.std(0).clamp_min(1e-8)
        Z = (X - self.mean_) / self.std_
        # economy SVD of the standardized data
        _, _, vh = torch.linalg.svd(Z, full_matrices=False)
        comps = vh[: self.k]
        # deterministic sign convention: largest-|.| loading positive
        signs = torch.sign(comps[torch.arange(comps.shape[0]), comps.abs().argmax(1)])
        self.components_ = comps * signs[:, None]
        proj = Z @ self.components_.T
        self.out_min_ = proj.min(0).values
        self.out_max_ = proj.max(0).values
        return self

    def transform(self, X: torch.Tensor, to_unit: bool = True) -> torch.Tensor:
        X = X.reshape(X.shape[0], -1).double()
        proj = ((X - self.mean_) / self.std_) @ self.components_.T
        if to_unit:  # fixed (train-fitted) min-max to [0,1] so angles are comparable across clients
            rng = (self.out_max_ - self.out_min_).clamp_min(1e-8)
            proj = ((proj - self.out_min_) / rng).clamp(0.0, 1.0)
        return proj.float()

    def fit_transform(self, X: torch.Tensor, to_unit: bool = True) -> torch.Tensor:
        return self.fit(X).transform(X, to_unit)

    def state_dict(self) -> dict:
        return {"k": torch.tensor(self.k), "mean": self.mean_, "std": self.std_,
                "components": self.components_, "out_min": self.out_min_, "out_max": self.out_max_}

    def save(self, path: str) -> None:
        torch.save(self.state_dict(), path)

    @classmethod
    def load(cls, path: str) -> "StandardPCA":
        sd = torch.load(path, weights_only=True)
        t = cls(int(sd["k"]))
        t.mean_, t.std_, t.components_ = sd["mean"], sd["std"], sd["components"]
        t.out_min_, t.out_max_ = sd["out_min"], sd["out_max"]
        return t


def make_features(X: torch.Tensor, method: str, n_features: int, fitted=None):
    """[N,1,28,28] or [N,L] -> [N, n_features] in [0,1]; returns (features, transformer)."""
    if method == "pool":
        f = pool_batch(X.reshape(X.shape[0], -1).float(), n_features)
        return f, None
    if method == "downsample":
        side = int(round(math.sqrt(n_features)))
        if side * side != n_features:
            raise ValueError("downsample features need a square n_features")
        return downsample_batch(X.reshape(X.shape[0], X.shape[-2], X.shape[-1]).float(), (side, side)), None
    if method == "pca":
        t = fitted or StandardPCA(n_features).fit(X)
        return t.transform(X), t
    if method == "raw":
        return X.reshape(X.shape[0], -1).float(), None
    raise ValueError(f"unknown feature method '{method}'")
