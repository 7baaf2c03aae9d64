"""Pairwise-mask secure aggregation (ROADMAP.md:52-55,61,137-138: ``secure_agg.py`` with a seed
exchange API simulating DH key agreement at registration).

Protocol (Bonawitz et al. style, single round, honest-but-curious server):
  * registration: each client draws a secret ``sk_i`` from OS randomness (``secrets``), held only by
    the rank hosting that client, and publishes ``pk_i = g^sk_i mod p``; ranks exchange public keys
    only (``SecureAggregator.setup``: one all-gather).  A pair seed is ``s_ij = H(g^(sk_i sk_j) mod p)``
    - both ends derive it; the aggregate (server side) sees public keys and masked sums only.
    Passing an integer ``session_seed`` instead derives every secret from it (reproducible simulation
    for tests - whoever knows the seed can unmask, so it is not a confidentiality setting).
  * masking: the update is encoded in the fixed-point ring Z_{2^bits} (default 2^48, scale 2^24), then client i
    adds ``+PRG(s_ij, round)`` for every peer j>i and ``-PRG(s_ij, round)`` for j<i.
  * aggregation: masked vectors are summed mod 2^bits - pair masks cancel EXACTLY (integer ring,
    no float rounding), then decoded.
  * dropouts: if a masked client drops before its vector arrives, surviving peers reveal their pair
    seeds with the dropped client and the server removes the orphan masks (ROADMAP:91).

PRG = Philox4x32-10 keyed by the pair seed, counter = (element/4, round) - the same generator the
HIP aggregation kernel uses on device: ``round_tables`` gives the fused FedAvg kernel
(``csrc/train_kernels.hip``, ``secagg_masks``) every local client's pair-seed key words and mask signs for a
round, and the kernel masks each client's encoded update itself (the round stays on the hipGraph path).
"""
from __future__ import annotations

import hashlib
import secrets
from typing import Iterable, Optional

import numpy as np
import torch

from ..utils.seeding import MASK32, derive_seed, philox4x32

# RFC 3526 group 14 would be realistic; a 127-bit Mersenne prime keeps the simulation fast.
_P = (1 << 127) - 1
_G = 3


def _hash_int(*vals: int) -> int:
    h = hashlib.blake2b(digest_size=8)
    for v in vals:
        h.update(int(v).to_bytes(16, "little", signed=False))
    return int.from_bytes(h.digest(), "little")


class KeyRegistry:
    """Simulated Diffie-Hellman key agreement (registration phase).

    Holds the secret keys of the clients registered HERE and the public keys of every client."""

    def __init__(self, session_seed: Optional[int] = None):
        self.session_seed = session_seed
        self._sk: dict[int, int] = {}
        self.public: dict[int, int] = {}

    def register(self, client: int) -> int:
        if self.session_seed is None:
            sk = secrets.randbelow(_P - 2) + 1
        else:
            sk = derive_seed(self.session_seed, "secagg", 0xD4, client) % (_P - 2) + 1
        self._sk[client] = sk
        self.public[client] = pow(_G, sk, _P)
        return self.public[client]

    def add_public(self, client: int, pk: int) -> None:
        if client not in self._sk:
            self.public[client] = int(pk)

    def pair_seed(self, me: int, peer: int) -> int:
        """Computed by client ``me`` from its own secret and the peer's public key."""
        if me not in self._sk:
            if self.session_seed is None:
                raise KeyError(f"client {me}'s secret key is not held by this process")
            self.register(me)
        if peer not in self.public:
            if self.session_seed is None:
                raise KeyError(f"no public key registered for client {peer}")
            self.register(peer)
        shared = pow(self.public[peer], self._sk[me], _P)
        return _hash_int(shared)


def prg_mask(pair_seed: int, round_num: int, P: int, bits: int = 48, device="cpu") -> torch.Tensor:
    """Uniform mask in [0, 2^bits) as int64 [P] (Philox keyed by the pair seed).

    bits <= 32 uses one Philox word per element, bits in (32, 62] combines two words.
    """
    words_per = 1 if bits <= 32 else 2
    nw = P * words_per
    nblk = (nw + 3) // 4
    idx = torch.arange(nblk, dtype=torch.int64)
    ctr = torch.stack([idx & MASK32, (idx >> 32) & MASK32,
                       torch.full_like(idx, round_num & MASK32), torch.full_like(idx, 0x5EC)], -1)
    out = philox4x32(ctr, pair_seed & MASK32, (pair_seed >> 32) & MASK32).reshape(-1)[:nw]
    if words_per == 2:
        out = out[0::2] | (out[1::2] << 32)
    if bits < 64:
        out = out & ((1 << bits) - 1)
    return out.to(device)


def encode_fixed(x: torch.Tensor, scale: float, bits: int = 48) -> torch.Tensor:
    q = torch.round(x.double() * scale).to(torch.int64)
    return torch.remainder(q, 1 << bits)


def decode_fixed(v: torch.Tensor, scale: float, bits: int = 48) -> torch.Tensor:
    v = torch.remainder(v, 1 << bits)
    half = 1 << (bits - 1)
    signed = torch.where(v >= half, v - (1 << bits), v)
    return signed.double() / scale


class SecureAggregator:
    def __init__(self, session_seed: Optional[int] = None, bits: int = 48, scale: float = 2.0 ** 24):
        self.registry = KeyRegistry(session_seed)
        self.bits = bits
        self.scale = scale
        self.modulus = 1 << bits

    def register(self, clients: Iterable[int]) -> None:
        for c in clients:
            self.registry.register(int(c))

    def setup(self, local_clients: Iterable[int], world) -> None:
        """Register this rank's clients (secrets stay here) and all-gather every client's public key:
        rows [client, pk words 0..3] (127-bit keys as four 32-bit words)."""
        from ..parallel.dist import all_gather_cat
        rows = []
        for c in local_clients:
            pk = self.registry.register(int(c))
            rows.append([int(c)] + [(pk >> (32 * i)) & 0xFFFFFFFF for i in range(4)])
        t = torch.tensor(rows, dtype=torch.int64).reshape(-1).to(world.device)
        allrows = all_gather_cat(t, world).cpu().reshape(-1, 5).tolist()
        for c, *w in allrows:
            self.registry.add_public(int(c), sum(int(x) << (32 * i) for i, x in enumerate(w)))

    def client_mask(self, client: int, participants: Iterable[int], round_num: int, P: int,
                    device="cpu") -> torch.Tensor:
        total = torch.zeros(P, dtype=torch.int64, device=device)
        for j in participants:
            j = int(j)
            if j == client:
                continue
            m = prg_mask(self.registry.pair_seed(client, j), round_num, P, self.bits, device)
            total = total + m if client < j else total - m
        return torch.remainder(total, self.modulus)

    def mask(self, update: torch.Tensor, client: int, participants: Iterable[int], round_num: int) -> torch.Tensor:
        enc = encode_fixed(update, self.scale, self.bits)
        return torch.remainder(enc + self.client_mask(client, participants, round_num, update.numel(),
                                                      update.device).view_as(enc), self.modulus)

    def seed_matrix(self, rows: Iterable[int], num_clients: int) -> np.ndarray:
        """uint64 [len(rows), num_clients] pair seeds s_{i,j} of clients ``rows`` (held here) with every client j
        (diagonal 0).  Pair seeds do not depend on the round, so they are derived once (modular exponentiations)
        and cached."""
        cache = self.__dict__.setdefault("_seed_rows", {})
        out = np.zeros((len(list(rows)), num_clients), dtype=np.uint64)
        for r, i in enumerate(rows):
            i = int(i)
            row = cache.get(i)
            if row is None or row.shape[0] != num_clients:
                row = np.array([self.registry.pair_seed(i, j) if j != i else 0 for j in range(num_clients)],
                               dtype=np.uint64)
                cache[i] = row
            out[r] = row
        return out

    def round_tables(self, clients: list[int], participants: Iterable[int], dropped: Iterable[int],
                     num_clients: int) -> tuple[torch.Tensor, torch.Tensor]:
        """Device-kernel tables of one round for the masking clients ``clients`` (rows): pair-seed key words
        int32 [K, N, 2] (lo, hi 32-bit halves) and mask signs int32 [K, N] over ALL N clients: +1 toward
        participating peers j > i, -1 toward j < i, 0 for the client itself and non-participants.  A dropped
        peer d's orphan mask is removed by the correction the survivors enable (``aggregate``); that exactly
        cancels the survivor's mask toward d mod 2^bits, so its sign is 0 (net)."""
        K = len(clients)
        live = np.zeros(num_clients, dtype=bool)
        live[[int(c) for c in participants]] = True
        live[[int(d) for d in dropped]] = False
        cid = np.asarray([int(c) for c in clients], dtype=np.int64)[:, None]
        j = np.arange(num_clients, dtype=np.int64)[None, :]
        sign = np.where(live[None, :] & (j != cid), np.where(j > cid, 1, -1), 0).astype(np.int32)
        seeds = self.seed_matrix(clients, num_clients)
        words = np.stack([seeds & np.uint64(0xFFFFFFFF), seeds >> np.uint64(32)], -1).astype(np.uint32)
        return (torch.from_numpy(words.view(np.int32).reshape(K, num_clients, 2).copy()),
                torch.from_numpy(sign.reshape(K, num_clients)))

    def aggregate(self, masked: list[torch.Tensor], survivors: list[int], dropped: Optional[list[int]] = None,
                  round_num: int = 0) -> torch.Tensor:
        """Sum surviving masked vectors; remove orphan masks of ``dropped`` clients; decode."""
        total = torch.zeros_like(masked[0])
        for m in masked:
            total = torch.remainder(total + m, self.modulus)
        for d in dropped or []:
            # survivors reveal s_{i,d}: remove the mask each survivor i added toward d
            for i in survivors:
                m = prg_mask(self.registry.pair_seed(i, d), round_num, total.numel(), self.bits, total.device)
                total = total - m if i < d else total + m
            total = torch.remainder(total, self.modulus)
        return decode_fixed(total, self.scale, self.bits)
