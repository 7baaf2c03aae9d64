"""TinyCNN - the CFed classical baseline (reference ``src/CFed/Classical_FL.py:21-38``).

conv1 1->16 k5 p2 -> ReLU -> maxpool2 -> conv2 16->32 k5 p2 -> ReLU -> maxpool2 -> flatten(1568)
-> fc1 1568->64 -> ReLU -> Dropout(0.5) -> fc2 64->C.  state_dict keys/shapes are the reference's
(``conv1.weight[16,1,5,5]`` ... ``fc2.bias[C]``; 113 859 fp32 params for C=3).

``TinyCNN`` is the nn.Module (reference API).  ``BatchedTinyCNN`` is the MI355X layout: the
parameters of K clients live in ONE flat [K, P] buffer (one row per client, reference key order),
and one forward evaluates all K clients at once - grouped convolutions (client = group) and batched
GEMMs - instead of K sequential models (``Classical_FL.py:132-140``).  On the HIP backend the
layers run as the fused gfx950 kernels of ``ops/cnn_hip.py``.
"""
from __future__ import annotations

import math
from collections import OrderedDict

import torch
import torch.nn as nn
import torch.nn.functional as F


class TinyCNN(nn.Module):
    def __init__(self, num_classes: int = 3):
        super().__init__()
        self.conv1 = nn.Conv2d(1, 16, kernel_size=5, padding=2)
        self.conv2 = nn.Conv2d(16, 32, kernel_size=5, padding=2)
        self.fc1 = nn.Linear(32 * 7 * 7, 64)
        self.fc2 = nn.Linear(64, num_classes)
        self.dropout = nn.Dropout(0.5)

    def forward(self, x):
        x = F.max_pool2d(F.relu(self.conv1(x)), 2)
        x = F.max_pool2d(F.relu(self.conv2(x)), 2)
        x = x.view(-1, 32 * 7 * 7)
        x = self.dropout(F.relu(self.fc1(x)))
        return self.fc2(x)


def param_shapes(num_classes: int = 3) -> "OrderedDict[str, tuple]":
    return OrderedDict([
        ("conv1.weight", (16, 1, 5, 5)), ("conv1.bias", (16,)),
        ("conv2.weight", (32, 16, 5, 5)), ("conv2.bias", (32,)),
        ("fc1.weight", (64, 1568)), ("fc1.bias", (64,)),
        ("fc2.weight", (num_classes, 64)), ("fc2.bias", (num_classes,)),
    ])


def n_params(num_classes: int = 3) -> int:
    return sum(math.prod(s) for s in param_shapes(num_classes).values())


def layer_boundaries(num_classes: int = 3) -> list[int]:
    """Flat offsets of each tensor (bucket boundaries for the layer-bucketed all-reduce)."""
    out = [0]
    for s in param_shapes(num_classes).values():
        out.append(out[-1] + math.prod(s))
    return out


def flat_to_state_dict(flat: torch.Tensor, num_classes: int = 3) -> "OrderedDict[str, torch.Tensor]":
    sd = OrderedDict()
    off = 0
    for k, s in param_shapes(num_classes).items():
        n = math.prod(s)
        sd[k] = flat[off: off + n].reshape(s).clone()
        off += n
    return sd


def state_dict_to_flat(sd: dict, num_classes: int = 3) -> torch.Tensor:
    return torch.cat([sd[k].reshape(-1).float() for k in param_shapes(num_classes)])


def init_flat(num_classes: int = 3, seed: int = 0) -> torch.Tensor:
    """PyTorch default init of TinyCNN (kaiming-uniform weights, uniform biases), keyed by seed."""
    g = torch.Generator().manual_seed(seed)
    with torch.random.fork_rng(devices=[]):
        torch.manual_seed(int(torch.randint(0, 2 ** 31 - 1, (1,), generator=g)))
        m = TinyCNN(num_classes)
    return state_dict_to_flat(m.state_dict(), num_classes)


def views(params: torch.Tensor, num_classes: int = 3) -> dict:
    """Per-layer views [K, ...] into a flat [K, P] client parameter buffer."""
    K = params.shape[0]
    out = {}
    off = 0
    for k, s in param_shapes(num_classes).items():
        n = math.prod(s)
        out[k] = params[:, off: off + n].reshape((K,) + s)
        off += n
    return out


def batched_forward(params: torch.Tensor, x: torch.Tensor, num_classes: int = 3,
                    dropout_mask: torch.Tensor | None = None) -> torch.Tensor:
    """All clients at once.  params [K, P], x [K, B, 1, 28, 28] -> logits [K, B, C].

    ``dropout_mask`` [K, B, 64] (values 0 or 2 = 1/(1-p)) applies inverted dropout after fc1+ReLU;
    None = eval mode.
    """
    K, B = x.shape[:2]
    v = views(params, num_classes)
    h = x.reshape(K, B, 28, 28).transpose(0, 1)                          # [B, K, 28, 28]
    h = F.conv2d(h, v["conv1.weight"].reshape(K * 16, 1, 5, 5), v["conv1.bias"].reshape(-1), padding=2,
                 groups=K)
    h = F.max_pool2d(F.relu(h), 2)                                        # [B, K*16, 14, 14]
    h = F.conv2d(h, v["conv2.weight"].reshape(K * 32, 16, 5, 5), v["conv2.bias"].reshape(-1), padding=2,
                 groups=K)
    h = F.max_pool2d(F.relu(h), 2)                                        # [B, K*32, 7, 7]
    h = h.reshape(B, K, 1568).transpose(0, 1)                             # [K, B, 1568]
    h = torch.baddbmm(v["fc1.bias"][:, None, :], h, v["fc1.weight"].transpose(1, 2))
    h = F.relu(h)
    if dropout_mask is not None:
        h = h * dropout_mask
    return torch.baddbmm(v["fc2.bias"][:, None, :], h, v["fc2.weight"].transpose(1, 2))


def dropout_keys(K_ids, seed: int, round_num: int) -> torch.Tensor:
    """Host int64 [K, 2] Philox keys of the clients' dropout streams in round ``round_num`` (step = stream)."""
    from ..utils.seeding import philox_keys
    return torch.tensor(philox_keys(seed, ("dropout", round_num), [int(c) for c in K_ids]), dtype=torch.int64)


def dropout_masks(K_ids, B: int, seed: int, round_num: int, step: int, device, p: float = 0.5) -> torch.Tensor:
    """Inverted-dropout masks [K, B, 64] keyed by (seed, round, client, step) - rank-count invariant."""
    from ..quantum.noise import uniforms
    from ..utils.device import h2d
    keys = h2d(dropout_keys(K_ids, seed, round_num), device)
    u = uniforms(keys, B * 64, stream=step)      # HIP Philox kernel on GPU, bit-identical torch oracle on CPU
    return ((u >= p).float() / (1 - p)).reshape(len(K_ids), B, 64)
