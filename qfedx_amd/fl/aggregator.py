"""Server-side aggregation: Delta -> angle wrap -> DP clip+noise -> SecAgg mask -> weighted sum.

Reference FedAvg (``Classical_FL.py:66-81``): sum_k (n_k / sum n) * theta_k over each
state_dict key, averaging WEIGHTS.  ROADMAP (``:36-37``) wants clients to return Delta-theta with
angle deltas wrapped to [-pi, pi].  Both are provided: ``aggregate='delta'`` (default) and
``aggregate='weights'`` (no wrap; algebraically identical to the reference formula).

Per round on each rank (SURVEY §3.2, K8/K17/K18/K20 fused on GPU):
    local = sum_{k on this rank, fixed order} w_k * priv(wrap(theta_k - theta_g))   (+ masks)
    global = all_reduce(local)             # one message per rank, RCCL over xGMI
    theta_g += global[:P] / global[P]
"""
from __future__ import annotations

import math
from typing import Optional

import torch

from ..privacy.dp import clip_and_noise
from ..privacy.secure_agg import SecureAggregator


EXACT_SCALE = float(2 ** 32)   # fixed-point scale of the exact (rank-count invariant) aggregation
SAT_LIMIT = float(2 ** 53)     # largest fixed-point term (|w * Delta| <= 2^21): exact in float64, 2^10 terms fit int64


def wrap_angles(d: torch.Tensor) -> torch.Tensor:
    """Wrap to [-pi, pi) (ROADMAP.md:37 periodicity of rotation angles)."""
    return torch.remainder(d + math.pi, 2 * math.pi) - math.pi


def federated_averaging(client_updates):
    """Reference-compatible FedAvg over ``[(state_dict, n_samples), ...]`` (``Classical_FL.py:66-81``).

    Fixed: the reference's ``+=`` of a float into ``zeros_like`` breaks on integer buffers; here
    non-floating entries (e.g. BatchNorm counters) are taken from the first client.
    """
    total = sum(n for _, n in client_updates)
    first = client_updates[0][0]
    out = {}
    for key, ref in first.items():
        if not torch.is_floating_point(ref):
            out[key] = ref.clone()
            continue
        acc = torch.zeros_like(ref, dtype=torch.float64)
        for params, n in client_updates:
            acc += (n / total) * params[key].double()
        out[key] = acc.to(ref.dtype)
    return out


def _scale_table(dp_scale, K: int, device):
    """The HIP reduce's per-client noise-scale table: None (local DP), a device table as given, or a float broadcast."""
    if dp_scale is None or torch.is_tensor(dp_scale):
        return dp_scale
    return torch.full((K,), float(dp_scale), dtype=torch.float32, device=device)


class Aggregator:
    def __init__(self, n_params: int, angle_mask: Optional[torch.Tensor], device, backend: str = "torch",
                 aggregate: str = "delta", wrap: bool = True, dp: bool = False, clip_norm: float = 1.0,
                 noise_multiplier: float = 1.0, secure_agg: bool = False, secagg: Optional[SecureAggregator] = None,
                 seed: int = 0, num_clients: int = 0):
        self.P = n_params
        self.num_clients = num_clients      # all clients of the federation (SecAgg sign / seed tables)
        self.device = torch.device(device)
        self.backend = backend
        self.aggregate = aggregate
        self.wrap = wrap and aggregate == "delta" and angle_mask is not None
        self.angle_mask = (angle_mask.to(self.device).bool() if angle_mask is not None
                           else torch.zeros(n_params, dtype=torch.bool, device=self.device))
        self.dp = dp
        self.clip_norm = clip_norm
        self.noise_multiplier = noise_multiplier
        self.secure_agg = secure_agg
        self.secagg = secagg
        self.seed = seed
        self.last_norms: Optional[torch.Tensor] = None
        self.last_saturation: Optional[torch.Tensor] = None   # [1] count of clamped fixed-point terms

    def local_reduce(self, theta_k: torch.Tensor, theta_g: torch.Tensor, weights: torch.Tensor,
                     round_num: int, client_ids: list, participants: Optional[list] = None,
                     dropped: Optional[list] = None, out: Optional[torch.Tensor] = None,
                     keys: Optional[torch.Tensor] = None, pack: Optional[tuple] = None,
                     secagg_tabs: Optional[tuple] = None, norm_cid: Optional[torch.Tensor] = None,
                     apply: Optional[tuple] = None, dp_scale=None) -> torch.Tensor:
        """This rank's contribution [P+1] = [sum_k w_k priv(Delta_k) | sum_k w_k].

        float64 normally; int64 ring elements (mod 2^bits, masked) under secure aggregation.
        ``dropped`` clients (subset of participants, possibly on other ranks) had agreed masks but
        never deliver: survivors on this rank add the orphan-mask corrections.
        ``pack`` (HIP fast path only): (buf, loss, correct, nvalid, act) - the same launch also packs the round
        metrics into the tail of the all-reduce buffer ``buf`` whose head is ``out``.  ``apply`` (with ``pack``,
        single-rank rounds): the same launch also applies the round to the global params
        (``fedavg_hip.fused_local_reduce``).  ``dp_scale``: the round's per-client noise factor
        (``privacy.dp.noise_scale``; distributed DP) - a float, or a device float32 [K] table on the HIP path.
        """
        if self.backend == "hip":
            from ..ops import fedavg_hip
            if getattr(self, "_mask_u8", None) is None:
                self._mask_u8 = self.angle_mask.to(torch.uint8).contiguous()
            sa = None
            if self.secure_agg:
                # the fused kernel masks every client's ring element itself (K18 on the device); ``secagg_tabs``
                # = (seeds, sign, round) device tables (uploaded with the round), else built and uploaded here
                if secagg_tabs is None:
                    from ..utils.device import h2d
                    parts = list(participants if participants is not None else client_ids)
                    n_all = max([self.num_clients] + [int(c) + 1 for c in parts + list(client_ids)])
                    seeds, sign = self.secagg.round_tables(client_ids, parts, dropped or [], n_all, round_num)
                    secagg_tabs = (h2d(seeds, self.device), h2d(sign, self.device),
                                   h2d(torch.tensor([round_num], dtype=torch.int32), self.device))
                # a square full-graph table (row k = client k, all clients here) lets the kernel generate each
                # pair's mask stream once for both clients
                ids = [int(c) for c in client_ids]
                pairsym = (getattr(self.secagg, "graph", "full") == "full" and ids == list(range(len(ids)))
                           and secagg_tabs[1].dim() == 2 and tuple(secagg_tabs[1].shape) == (len(ids), len(ids))
                           and len(ids) <= 128)
                sa = (*secagg_tabs, self.secagg.scale, self.secagg.bits, pairsym)
            out, norms, sat = fedavg_hip.fused_local_reduce(
                theta_k, theta_g, weights, self._mask_u8, client_ids, round_num, self.seed,
                wrap=self.wrap, dp=self.dp, clip_norm=self.clip_norm,
                noise_multiplier=self.noise_multiplier, out=out, keys=keys, pack=pack, secagg=sa,
                norm_cid=norm_cid, apply=apply, dp_scale=_scale_table(dp_scale, len(client_ids), self.device))
            self.last_norms = norms
            self.last_saturation = sat
            return out
        if pack is not None or apply is not None:
            raise ValueError("the metric pack and the apply are fused into the HIP reduce only")
        delta = theta_k.double() - theta_g.double()[None, :]
        if self.wrap:
            delta = torch.where(self.angle_mask[None, :], wrap_angles(delta), delta)
        if self.dp:
            sk = 1.0 if dp_scale is None else float(dp_scale if not torch.is_tensor(dp_scale) else dp_scale.reshape(-1)[0])
            delta, norms = clip_and_noise(delta, self.clip_norm, self.noise_multiplier, self.seed,
                                          round_num, client_ids, scale_k=sk)
            self.last_norms = norms
        else:
            self.last_norms = delta.norm(dim=-1)
        w = weights.double().to(delta.device)
        weighted = torch.cat([delta * w[:, None], w[:, None]], -1)    # [K, P+1]
        if not self.secure_agg:
            # per-client fixed point BEFORE summation: integer sums are associative, so the aggregate
            # is bitwise identical however clients are sharded over ranks.  Terms are
            # held to 2^53 (as the HIP kernel does) and the clamped ones counted, never wrapped.
            v = weighted * EXACT_SCALE
            bad = ~(v.abs() <= SAT_LIMIT)
            self.last_saturation = bad.sum().reshape(1)
            v = torch.where(torch.isnan(v), torch.zeros_like(v), v).clamp(-SAT_LIMIT, SAT_LIMIT)
            return torch.round(v).to(torch.int64).sum(0)
        sa = self.secagg
        parts = list(participants if participants is not None else client_ids)
        sa._require_ok(parts, dropped or [], round_num)        # no survivor may be left without live mask neighbours
        total = torch.zeros(self.P + 1, dtype=torch.int64, device=delta.device)
        for k, cid in enumerate(client_ids):
            total = torch.remainder(total + sa.mask(weighted[k], int(cid), parts, round_num), sa.modulus)
        from ..privacy.secure_agg import prg_mask
        for d in dropped or []:
            nb = set(sa.neighbors(int(d), parts, round_num))
            for cid in client_ids:
                if int(cid) not in nb:
                    continue
                m = prg_mask(sa.registry.pair_seed(int(cid), int(d)), round_num, self.P + 1, sa.bits, delta.device)
                total = total - m if int(cid) < int(d) else total + m
            total = torch.remainder(total, sa.modulus)
        return total

    def finalize(self, reduced: torch.Tensor) -> tuple[torch.Tensor, torch.Tensor]:
        """Decode the all-reduced [P+1] vector -> (mean update [P] float64, weight sum (0-d tensor)).

        Stays on the device (no host read-back), so a round can be enqueued without a sync."""
        if self.secure_agg:
            from ..privacy.secure_agg import decode_fixed
            vals = decode_fixed(reduced, self.secagg.scale, self.secagg.bits)
        elif reduced.dtype == torch.int64:
            vals = reduced.double() / EXACT_SCALE
        else:
            vals = reduced.double()
        wsum = vals[self.P]
        return vals[: self.P] / wsum.clamp(min=1e-300), wsum

    def apply(self, theta_g: torch.Tensor, mean_update: torch.Tensor, server_lr: float = 1.0,
              wsum: Optional[torch.Tensor] = None) -> torch.Tensor:
        """theta_g + lr * mean_update; a round with zero total weight (everyone dropped) keeps theta_g."""
        new = theta_g.double() + server_lr * mean_update.to(theta_g.device)
        if wsum is not None:
            new = torch.where(wsum.to(new.device) > 0, new, theta_g.double())
        return new.to(theta_g.dtype)

