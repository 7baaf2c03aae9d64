"""Per-client DP: clip the update to l2 norm C, add N(0, sigma^2 C^2 I) (ROADMAP.md:47,50-51).

Noise is drawn from Philox4x32-10 keyed by (seed, 'dp_noise', round, client) - counter-based, so
a client's noise is the same whichever rank (and however many ranks) processes it; the gfx950
fused aggregation kernel (``csrc/fedavg.hip``) draws the identical stream on device.
"""
from __future__ import annotations

import torch

from ..utils.seeding import philox_key, philox_normal


def clip_factors(deltas: torch.Tensor, clip_norm: float) -> tuple[torch.Tensor, torch.Tensor]:
    """deltas [K, P] -> (scale [K] = min(1, C/||d||), norms [K])."""
    norms = deltas.double().norm(dim=-1)
    scale = torch.clamp(clip_norm / torch.clamp(norms, min=1e-12), max=1.0)
    return scale.to(deltas.dtype), norms.to(deltas.dtype)


def dp_noise(P: int, seed: int, round_num: int, client: int, device="cpu") -> torch.Tensor:
    key = philox_key(seed, "dp_noise", round_num, client)
    return philox_normal(P, key).to(device)


def clip_and_noise(deltas: torch.Tensor, clip_norm: float, noise_multiplier: float, seed: int,
                   round_num: int, client_ids, add_noise: bool = True) -> tuple[torch.Tensor, torch.Tensor]:
    """Torch reference of the fused DP step.  Returns (privatised deltas [K,P], pre-clip norms [K])."""
    scale, norms = clip_factors(deltas, clip_norm)
    out = deltas * scale[:, None]
    if add_noise and noise_multiplier > 0:
        std = noise_multiplier * clip_norm
        noise = torch.stack([dp_noise(deltas.shape[1], seed, round_num, int(c), deltas.device)
                             for c in client_ids])
        out = out + std * noise.to(out.dtype)
    return out, norms
