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
  * mask graph: ``graph="full"`` (default) pairs every two participants - K (K - 1) / 2 pair masks per round, each
    P elements long.  ``graph="sparse"`` is the SecAgg+ construction (Bell et al., CCS 2020): each participant pairs
    only with its 2 ceil(log2 K) neighbours in a circulant graph over a round-keyed public permutation of the
    participants, so the round generates O(K log K) masks instead of O(K^2).  Masks still cancel exactly and orphan
    masks of dropped clients are removed the same way (only their graph neighbours reveal seeds).  The guarantee is
    SecAgg+'s: the sum stays hidden unless the server corrupts or drops enough of a client's neighbourhood, a weaker
    statement than the complete graph's.
  * live-neighbour threshold: a surviving participant whose mask neighbours all dropped would send its ring element
    with no mask left in it (after the orphan masks are removed the server holds that client's update).  Every
    surviving participant must therefore keep at least ``min_live`` live neighbours (default: half its degree on the
    sparse graph, as SecAgg+ requires; one on the complete graph); otherwise the round is aborted (``SecAggAbort``)
    - ``round_tables`` and ``aggregate`` refuse it, and the server skips the round's aggregation on every rank.

PRG = Philox4x32-10 keyed by the pair seed, counter = (element/4, round) - the same generator the
HIP aggregation kernel uses on device: ``round_tables`` gives the fused FedAvg kernel
(``csrc/train_kernels.hip``, ``secagg_masks``) every local client's pair-seed key words and mask signs for a
round, and the kernel masks each client's encoded update itself (the round stays on the hipGraph path).
"""
from __future__ import annotations

import hashlib
import math
import secrets
from typing import Iterable, Optional

import numpy as np
import torch

from ..utils.seeding import MASK32, derive_seed, np_rng, philox4x32

GRAPH_KEY = 0x5EC6A   # the neighbour graph is public (a server could announce it): keyed by round, not by a secret


class SecAggAbort(ValueError):
    """The round's surviving participants do not keep enough live mask neighbours: aggregating would unmask one."""


def secagg_degree(k: int) -> int:
    """SecAgg+ neighbours per participant among ``k``: 2 ceil(log2 k), at most k - 1 (then the graph is complete)."""
    if k <= 1:
        return 0
    return min(k - 1, 2 * max(1, math.ceil(math.log2(k))))

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
        # pair seeds do not depend on the round: one modular exponentiation per (client, peer, peer key), cached
        # (the sparse graph re-pairs clients every round, so its tables would otherwise pay one per edge per round)
        cache = self.__dict__.setdefault("_pair_cache", {})
        pk = self.public[peer]
        hit = cache.get((me, peer))
        if hit is not None and hit[0] == pk and hit[1] == self._sk[me]:
            return hit[2]
        seed = _hash_int(pow(pk, self._sk[me], _P))
        cache[(me, peer)] = (pk, self._sk[me], seed)
        return seed


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
    def __init__(self, session_seed: Optional[int] = None, bits: int = 48, scale: float = 2.0 ** 24,
                 graph: str = "full", min_live: int = 0):
        if graph not in ("full", "sparse"):
            raise ValueError(f"secagg graph must be full | sparse, got {graph!r}")
        self.registry = KeyRegistry(session_seed)
        self.bits = bits
        self.scale = scale
        self.modulus = 1 << bits
        self.graph = graph
        self.min_live = int(min_live)
        self._nb = (None, None)

    def live_threshold(self, num_participants: int) -> int:
        """Live mask neighbours every surviving participant must keep (``min_live``, or auto: half the sparse
        graph's degree, rounded up, as SecAgg+ requires; one on the complete graph)."""
        if self.min_live > 0:
            return self.min_live
        if self.graph == "sparse" and secagg_degree(num_participants) < num_participants - 1:
            return max(1, (secagg_degree(num_participants) + 1) // 2)
        return 1

    def live_counts(self, participants: Iterable[int], dropped: Iterable[int], round_num: int) -> dict:
        """survivor -> number of its mask neighbours that survived the round."""
        parts = sorted({int(c) for c in participants})
        gone = {int(d) for d in dropped}
        surv = [c for c in parts if c not in gone]
        if self.graph == "full" or secagg_degree(len(parts)) >= len(parts) - 1:
            return {c: len(surv) - 1 for c in surv}           # complete graph: every other survivor
        pt, nbm = self._neighbor_matrix(tuple(parts), round_num)
        dead = np.zeros(int(pt.max()) + 1, dtype=bool)
        idx = [d for d in gone if d <= int(pt.max())]
        dead[idx] = True
        live = (~dead[nbm]).sum(1)
        return {int(c): int(n) for c, n, d in zip(pt, live, dead[pt]) if not d}

    def round_ok(self, participants: Iterable[int], dropped: Iterable[int], round_num: int) -> bool:
        """Every surviving participant keeps at least ``live_threshold`` live neighbours (public information: the
        participant set, the dropouts and the round-keyed graph, so every rank decides alike).  Decided once per
        (participants, dropouts, round): the server asks, then ``round_tables`` asks again."""
        parts = sorted({int(c) for c in participants})
        key = (tuple(parts), tuple(sorted({int(d) for d in dropped})), int(round_num))
        memo = self.__dict__.setdefault("_ok_memo", {})
        if key in memo:
            return memo[key]
        t = self.live_threshold(len(parts))
        self.check_threshold(len(parts))
        cnt = self.live_counts(parts, dropped, round_num)
        ok = all(v >= t for v in cnt.values())
        memo.clear()
        memo[key] = ok
        return ok

    def check_threshold(self, num_participants: int) -> None:
        """A ``min_live`` above the mask graph's degree (sparse degree, or K - 1 on the complete graph) fails every
        round even with no dropout: the server would silently turn every round into an aborted no-op.  Raised
        instead (a configuration error, not a privacy event)."""
        if num_participants < 2:
            return
        deg = num_participants - 1
        if self.graph == "sparse":
            deg = min(deg, secagg_degree(num_participants))
        if self.live_threshold(num_participants) > deg:
            raise ValueError(f"privacy.secagg_min_live={self.min_live} exceeds the mask graph degree {deg} of a "
                             f"{num_participants}-participant round ({self.graph} graph): every round would abort")

    def _require_ok(self, participants, dropped, round_num) -> None:
        if not self.round_ok(participants, dropped, round_num):
            parts = sorted({int(c) for c in participants})
            cnt = self.live_counts(parts, dropped, round_num)
            t = self.live_threshold(len(parts))
            low = sorted(c for c, v in cnt.items() if v < t)
            raise SecAggAbort(f"round {round_num}: survivors {low[:8]} keep fewer than {t} live mask neighbours; "
                              "aggregating would expose their updates")

    def neighbors(self, client: int, participants: Iterable[int], round_num: int) -> list[int]:
        """The peers ``client`` shares pair masks with this round (sorted).  Full graph: every other participant.
        Sparse graph: the secagg_degree(K) / 2 predecessors and successors of ``client`` on a circle of the K
        participants in a round-keyed public order - symmetric (j is i's neighbour iff i is j's), the same on every
        rank without communication."""
        client = int(client)
        parts = tuple(sorted({int(c) for c in participants}))
        if self.graph == "full" or secagg_degree(len(parts)) >= len(parts) - 1:
            return [j for j in parts if j != client]
        return list(self._neighbor_map(parts, round_num)[client])

    def _neighbor_matrix(self, parts: tuple, round_num: int):
        """(participants [K], their sorted sparse-graph neighbours [K, 2h]) for the sorted participant tuple ``parts``:
        the h predecessors and successors on the round's circle (cached per round; vectorised - the per-client
        Python sets cost ~1 ms a round at 128 clients, on the host path of every SecAgg round)."""
        key = (parts, int(round_num))
        if self._nb[0] != key:
            K = len(parts)
            pt = np.asarray(parts, dtype=np.int64)
            order = pt[np_rng(GRAPH_KEY, "secagg_graph", int(round_num), K).permutation(K)]
            pos = np.zeros(int(pt.max()) + 1, dtype=np.int64)
            pos[order] = np.arange(K)
            h = secagg_degree(K) // 2
            d = np.concatenate([np.arange(1, h + 1), -np.arange(1, h + 1)])
            self._nb = (key, (pt, np.sort(order[(pos[pt][:, None] + d[None, :]) % K], axis=1)))
        return self._nb[1]

    def _neighbor_map(self, parts: tuple, round_num: int) -> dict:
        """client -> sorted sparse-graph neighbours for the sorted participant tuple ``parts``."""
        pt, nbm = self._neighbor_matrix(parts, round_num)
        return {int(c): [int(j) for j in row] for c, row in zip(pt, nbm)}

    def table_width(self, num_clients: int) -> int:
        """Peer columns of ``round_tables``: every client (full graph) or the largest neighbourhood any round
        can have (sparse: the degree grows with the participant count, so this is its value at all clients - fixed,
        so the round's hipGraph keeps one shape)."""
        return num_clients if self.graph == "full" else max(1, secagg_degree(num_clients))

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
        for j in self.neighbors(client, participants, round_num):
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
        rows = [int(i) for i in rows]
        key = (tuple(rows), int(num_clients))
        whole = self.__dict__.get("_seed_whole")
        if whole is not None and whole[0] == key:
            return whole[1]                                  # the same rows every round: one stacked copy
        cache = self.__dict__.setdefault("_seed_rows", {})
        out = np.zeros((len(rows), num_clients), dtype=np.uint64)
        for r, i in enumerate(rows):
            i = int(i)
            row = cache.get(i)
            if row is None or row.shape[0] != num_clients:
                row = np.array([self.registry.pair_seed(i, j) if j != i else 0 for j in range(num_clients)],
                               dtype=np.uint64)
                cache[i] = row
            out[r] = row
        out.setflags(write=False)
        self._seed_whole = (key, out)
        return out

    def round_tables(self, clients: list[int], participants: Iterable[int], dropped: Iterable[int],
                     num_clients: int, round_num: int = 0) -> tuple[torch.Tensor, torch.Tensor]:
        """Device-kernel tables of one round for the masking clients ``clients`` (rows): pair-seed key words
        int32 [K, W, 2] (lo, hi 32-bit halves) and mask signs int32 [K, W], W = ``table_width``.  Full graph: column
        j is client j; +1 toward participating peers j > i, -1 toward j < i, 0 for the client itself and
        non-participants.  Sparse graph: row i lists its live neighbours (sign 0 pads).  A dropped peer d's orphan
        mask is removed by the correction the survivors enable (``aggregate``); that exactly cancels the survivor's
        mask toward d mod 2^bits, so its sign is 0 (net)."""
        self._require_ok(participants, dropped, round_num)
        if self.graph == "sparse":
            return self._sparse_tables(clients, participants, dropped, num_clients, round_num)
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

    def _sparse_tables(self, clients, participants, dropped, num_clients, round_num):
        W = self.table_width(num_clients)
        parts = list(participants)
        gone = {int(d) for d in dropped}
        # the graph is re-drawn every round, so over a run every pair is used: the clients' full seed rows are
        # derived once (cached, as for the full graph) and each round only gathers its neighbours' columns
        full = self.seed_matrix(clients, num_clients)
        pt = np.asarray(sorted({int(c) for c in parts}), dtype=np.int64)
        cl = np.asarray([int(c) for c in clients], dtype=np.int64)
        K = len(pt)
        if K == 0:
            nb = np.full((len(cl), 0), -1, dtype=np.int64)
        elif secagg_degree(K) >= K - 1:
            nb = np.where((pt[None, :] != cl[:, None]) & np.isin(cl, pt)[:, None], pt[None, :], -1)   # all others
        else:
            # the round's circle (_neighbor_matrix, shared with round_ok): rows of this rank's clients
            ptm, nbm = self._neighbor_matrix(tuple(int(c) for c in pt), round_num)
            row = np.full(max(int(pt.max()), int(cl.max(initial=0))) + 1, -1, dtype=np.int64)
            row[ptm] = np.arange(K)
            r = row[cl]
            nb = np.where((r >= 0)[:, None], nbm[np.maximum(r, 0)], -1)       # non-participants mask nothing
        if len(gone):
            nb = np.where(np.isin(nb, np.asarray(sorted(gone), dtype=np.int64)), -1, nb)
        # live neighbours first (ascending), -1 pads
        key = np.where(nb < 0, np.iinfo(np.int64).max, nb)
        nb = np.take_along_axis(nb, np.argsort(key, axis=1, kind="stable"), axis=1)
        cnt = (nb >= 0).sum(1)
        if len(cnt) and int(cnt.max()) > W:
            raise ValueError(f"a client has {int(cnt.max())} live neighbours, table width {W}")
        nb = nb[:, :W] if nb.shape[1] >= W else np.pad(nb, ((0, 0), (0, W - nb.shape[1])), constant_values=-1)
        ok = nb >= 0
        seeds = np.where(ok, np.take_along_axis(full, np.where(ok, nb, 0), axis=1), np.uint64(0)).astype(np.uint64)
        sign = np.where(ok, np.where(nb > cl[:, None], 1, -1), 0).astype(np.int32)
        words = np.stack([seeds & np.uint64(0xFFFFFFFF), seeds >> np.uint64(32)], -1).astype(np.uint32)
        return (torch.from_numpy(words.view(np.int32).reshape(len(clients), W, 2).copy()),
                torch.from_numpy(sign))

    def orphan_pairs(self, survivors: Iterable[int], dropped: Iterable[int], participants: Iterable[int],
                     round_num: int) -> list[tuple[int, int]]:
        """(survivor i, dropped d) pairs whose seeds the survivors reveal: d is i's graph neighbour."""
        parts = list(participants)
        out = []
        for d in dropped:
            nb = set(self.neighbors(int(d), parts, round_num))
            out += [(int(i), int(d)) for i in survivors if int(i) in nb]
        return out

    def aggregate(self, masked: list[torch.Tensor], survivors: list[int], dropped: Optional[list[int]] = None,
                  round_num: int = 0) -> torch.Tensor:
        """Sum surviving masked vectors; remove orphan masks of ``dropped`` clients; decode.  Refuses a round in
        which a survivor kept fewer than ``live_threshold`` live neighbours (``SecAggAbort``)."""
        self._require_ok(list(survivors) + list(dropped or []), dropped or [], round_num)
        total = torch.zeros_like(masked[0])
        for m in masked:
            total = torch.remainder(total + m, self.modulus)
        parts = list(survivors) + list(dropped or [])
        for d in dropped or []:
            # survivors reveal s_{i,d}: remove the mask each neighbouring survivor i added toward d
            nb = set(self.neighbors(int(d), parts, round_num))
            for i in survivors:
                if int(i) not in nb:
                    continue
                m = prg_mask(self.registry.pair_seed(i, d), round_num, total.numel(), self.bits, total.device)
                total = total - m if i < d else total + m
            total = torch.remainder(total, self.modulus)
        return decode_fixed(total, self.scale, self.bits)
