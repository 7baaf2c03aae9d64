"""Python entry points of the fused aggregation / optimizer kernels (``csrc/train_kernels.hip``)."""
from __future__ import annotations

import os

import torch

from ..utils.device import h2d
from ..utils.seeding import philox_keys
from ._ext import ext


def adam_step(params, grads, m, v, t_in, t_out, active, lr, b1, b2, eps) -> None:
    """Fused client-batched Adam; step counters read from ``t_in``, ``t_in + active`` written to ``t_out``."""
    ext().adam(params, grads.float().contiguous(), m, v, t_in, t_out, active.float().contiguous(), lr, b1, b2, eps)


def sgdm_step(params, grads, buf, t_in, t_out, active, lr, mu, keep_state: bool = True) -> None:
    """Fused client-batched SGD-momentum; ``keep_state=False`` (a round's last local step) skips the buffer store."""
    ext().sgdm(params, grads.float().contiguous(), buf, t_in, t_out, active.float().contiguous(), lr, mu, keep_state)


_NO_KEYS = {}
_NO_PACK = {}
_PAIRSYM = os.environ.get("QFEDX_SECAGG_PAIRSYM", "1") != "0"   # A/B knob: per-client mask generation


def dp_noise_keys(client_ids, round_num, seed) -> torch.Tensor:
    """Host int32 [K, 2] Philox keys of the clients' DP noise in round ``round_num``."""
    return torch.tensor(philox_keys(seed, ("dp_noise", round_num), [int(c) for c in client_ids]),
                        dtype=torch.int64).reshape(-1, 2).to(torch.int32)


def fused_local_reduce(theta_k, theta_g, weights, angle_mask, client_ids, round_num, seed, wrap, dp, clip_norm,
                       noise_multiplier, out=None, keys=None, pack=None, sat=None, secagg=None, norm_cid=None,
                       apply=None, dp_scale=None):
    """[sum_k w_k priv(wrap(theta_k - theta_g)) | sum_k w_k] as exact int64 fixed point (scale 2^32)
    [P+1] (per-client terms rounded before the sum -> rank-count invariant), plus norms [K].
    ``angle_mask`` uint8 [P] on the device; ``out`` an optional int64 [P+1] destination (e.g. the head
    of the round's all-reduce buffer).  DP noise keys are only built / uploaded when DP is on; ``keys``
    (device int32 [K, 2], ``dp_noise_keys``) passes them in already on the device, which keeps the launch
    free of host values that change per round (capturable into a round graph).  ``pack`` = (buf, loss,
    correct, nvalid, act): ``out`` is the head of the round's [P + 6] all-reduce buffer ``buf`` and one more
    block of the same launch packs the round metrics into its tail (what ``round_pack`` does on its own).
    ``sat``: int64 [1] device counter that receives the number of fixed-point terms clamped at 2^53 (with
    ``pack``: ``buf[P + 5]``, zeroed by ``round_apply``; else a fresh zero counter).
    ``secagg`` = (seeds int32 [K, N, 2], sign int32 [K, N], round int32 [1] device tensors, scale, bits[,
    pairsym]): the [P + 1] head holds SecAgg ring elements instead, each client's term masked in the kernel
    (``SecureAggregator.round_tables``).  ``pairsym``: the table is square (full graph, row k = client k, every
    client a row) - each pair's mask stream is generated once for both of its clients (``QFEDX_SECAGG_PAIRSYM=0``
    turns it off; bitwise the same masks).  ``norm_cid`` (device int32 [K] global client ids; needs ``pack`` and
    DP): the pack block scatters the clients' pre-clip norms into ``buf[P + 6 + id]`` (CC6).
    ``apply`` = (theta [P] float32, outs float64 [6 + n_norms], counter int32 [1] zeroed, bits, ring scale,
    n_norms): single-rank rounds (no collective between reduce and apply) - the launch's last block also does
    ``round_apply``'s work (needs ``pack``).  ``dp_scale`` (device float32 [K], DP only): per-client factor on the
    noise std (distributed DP: 1 / sqrt(live participants), uploaded with the round's tables).
    Returns (out, norms, sat)."""
    K, P = theta_k.shape
    dev = theta_k.device
    if dp and keys is not None:
        if keys.numel() < 2 * K or keys.dtype != torch.int32 or keys.device != dev:
            raise ValueError("DP keys must be a device int32 [K, 2] tensor")
        keys = keys.reshape(-1).contiguous()
    elif dp:
        keys = h2d(dp_noise_keys(client_ids, round_num, seed).reshape(-1), dev)
    else:
        keys = _NO_KEYS.setdefault(dev, torch.zeros(0, dtype=torch.int32, device=dev))
    norms = torch.empty(ext().fedavg_norm_scratch(K, P), dtype=torch.float64, device=dev)   # [K] + scratch
    if out is None:
        out = torch.empty(P + 1, dtype=torch.int64, device=dev)
    if angle_mask.dtype != torch.uint8:
        angle_mask = angle_mask.to(torch.uint8)
    if pack is not None:
        sat = pack[0][P + 5: P + 6]
    elif sat is None:
        sat = torch.zeros(1, dtype=torch.int64, device=dev)
    if pack is None:
        e = _NO_PACK.setdefault(dev, (torch.zeros(0, dtype=torch.int64, device=dev),
                                      torch.zeros(0, dtype=torch.float32, device=dev)))
        pack = (e[0], e[1], e[1], e[1], e[1])
    ext().fedavg(theta_k.float().contiguous(), theta_g.float().contiguous(), angle_mask.contiguous(),
                 weights.double().contiguous(), norms, keys, bool(wrap), bool(dp), float(clip_norm),
                 float(noise_multiplier) if dp else 0.0, out, *pack, sat,
                 *((secagg[0].contiguous(), secagg[1].contiguous(), secagg[2].contiguous(), float(secagg[3]),
                    int(secagg[4]), torch.empty(K * (P + 1), dtype=torch.int64, device=dev))
                   if secagg is not None else (None, None, None, 1.0, 48, None)),
                 norm_cid, *(apply if apply is not None else (None, None, None, 0, 1.0, 0)),
                 dp_scale.float().contiguous() if (dp and dp_scale is not None) else None,
                 bool(secagg is not None and len(secagg) > 5 and secagg[5] and _PAIRSYM))
    return out, (norms[:K] if dp else None), sat
