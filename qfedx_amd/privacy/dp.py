"""Per-client DP: clip the update to l2 norm C, add N(0, sigma^2 C^2 I) (ROADMAP.md:47,50-51).

Noise is drawn from Philox4x32-10 keyed by (noise_seed, 'dp_noise', round, client) - counter-based,
so a client's noise is the same whichever rank (and however many ranks) processes it; the gfx950
fused aggregation kernel (``csrc/train_kernels.hip``) draws the identical stream on device.

``noise_seed`` is a per-run SECRET (:func:`draw_noise_seed`): 63 bits of OS randomness drawn on
rank 0 and broadcast, held in memory only - never written to the config, metrics, tracking store
or checkpoints.  Keying the noise by the public ``train.seed`` would let anyone holding the config
and successive released models regenerate and subtract it, voiding the accountant's epsilon; that
mode exists only behind ``privacy.deterministic_noise`` (tests of rank-count invariance / resume).
"""
from __future__ import annotations

import secrets

import torch

from ..utils.seeding import philox_key, philox_normal


def draw_noise_seed(world, deterministic: bool = False, public_seed: int = 0) -> int:
    """Root key of the DP noise and DP client-sampling streams, identical on every rank.

    ``deterministic=True`` returns ``public_seed`` (reproducible; NOT private)."""
    if deterministic:
        return int(public_seed)
    from ..parallel.dist import broadcast_
    s = secrets.randbits(63) if world.is_main else 0
    t = torch.tensor([s], dtype=torch.int64, device=world.device)
    broadcast_(t, world)
    return int(t.item())


def clip_factors(deltas: torch.Tensor, clip_norm: float) -> tuple[torch.Tensor, torch.Tensor]:
    """deltas [K, P] -> (scale [K] = min(1, C/||d||), norms [K])."""
    norms = deltas.double().norm(dim=-1)
    scale = torch.clamp(clip_norm / torch.clamp(norms, min=1e-12), max=1.0)
    return scale.to(deltas.dtype), norms.to(deltas.dtype)


def dp_noise(P: int, seed: int, round_num: int, client: int, device="cpu") -> torch.Tensor:
    key = philox_key(seed, "dp_noise", round_num, client)
    return philox_normal(P, key).to(device)


def noise_scale(mode: str, live: int) -> float:
    """Per-client factor on the noise std sigma C.  ``local`` (ROADMAP.md:50-51): 1 - every client adds the full
    N(0, sigma^2 C^2), so a sum of m clients carries sigma C sqrt(m).  ``distributed``: 1 / sqrt(m) for the round's m
    live participants - the (SecAgg-hidden) sum carries exactly the N(0, sigma^2 C^2) the accountant charges for
    sensitivity C, while no single share is private on its own."""
    if mode == "local":
        return 1.0
    if mode == "distributed":
        return 1.0 / float(max(1, live)) ** 0.5
    raise ValueError(f"privacy.noise_mode must be local | distributed, got {mode!r}")


def clip_and_noise(deltas: torch.Tensor, clip_norm: float, noise_multiplier: float, seed: int,
                   round_num: int, client_ids, add_noise: bool = True,
                   scale_k: float = 1.0) -> tuple[torch.Tensor, torch.Tensor]:
    """Torch reference of the fused DP step (``scale_k``: ``noise_scale`` of the round).  Returns (privatised
    deltas [K,P], pre-clip norms [K])."""
    scale, norms = clip_factors(deltas, clip_norm)
    out = deltas * scale[:, None]
    if add_noise and noise_multiplier > 0:
        # the same float32 factor the device kernel multiplies by (sigma x dps[k] x C)
        std = float(noise_multiplier) * float(torch.tensor(scale_k, dtype=torch.float32)) * clip_norm
        noise = torch.stack([dp_noise(deltas.shape[1], seed, round_num, int(c), deltas.device)
                             for c in client_ids])
        out = out + std * noise.to(out.dtype)
    return out, norms
