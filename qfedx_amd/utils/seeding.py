"""Reproducibility: one root seed -> counter-based streams keyed by purpose.

Reference behaviour: ``set_seeds`` seeds python/numpy/torch globals
(``/root/reference/src/CFed/Classical_FL.py:12-18``, also at import time, ``:18``;
``src/CFed/Preprocess.py:232-236``; ``src/QFed/testEncoder.py:60-62``).

MI355X-first redesign: the hot path never touches global RNG state.  Every random draw
(client sampling, minibatch order, dropout masks, DP noise, SecAgg masks, shot noise) is
keyed by ``(root_seed, purpose, round, client, ...)`` and produced by Philox4x32-10, the
same counter-based generator the HIP kernels run on device.  Results are therefore
invariant to the number of GPUs / ranks a run is sharded over.
"""
from __future__ import annotations

import hashlib
import random
import numpy as np
import torch

# Purpose tags (stable integers: they are part of the on-device RNG key).
PURPOSE = {
    "init": 1,
    "sample_clients": 2,
    "batch": 3,
    "dropout": 4,
    "dp_noise": 5,
    "secagg": 6,
    "shots": 7,
    "noise_traj": 8,
    "partition": 9,
    "synthetic": 10,
    "spsa": 11,
    "client_drop": 12,
}

PHILOX_M0 = 0xD2511F53
PHILOX_M1 = 0xCD9E8D57
PHILOX_W0 = 0x9E3779B9
PHILOX_W1 = 0xBB67AE85
MASK32 = 0xFFFFFFFF


def set_seeds(seed: int = 42) -> None:
    """Seed python, numpy and torch global generators (reference-compatible)."""
    random.seed(seed)
    np.random.seed(seed)
    torch.manual_seed(seed)
    if torch.cuda.is_available():
        torch.cuda.manual_seed_all(seed)


def derive_seed(root: int, *keys: int | str) -> int:
    """Stable 64-bit seed from a root seed and a tuple of keys (str or int)."""
    h = hashlib.blake2b(digest_size=8)
    h.update(int(root).to_bytes(8, "little", signed=False))
    for k in keys:
        if isinstance(k, str):
            k = PURPOSE[k] if k in PURPOSE else int.from_bytes(
                hashlib.blake2b(k.encode(), digest_size=8).digest(), "little")
        h.update(int(k & 0xFFFFFFFFFFFFFFFF).to_bytes(8, "little", signed=False))
    return int.from_bytes(h.digest(), "little")


def generator(root: int, *keys: int | str, device: str | torch.device = "cpu") -> torch.Generator:
    g = torch.Generator(device=device)
    g.manual_seed(derive_seed(root, *keys) & 0x7FFFFFFFFFFFFFFF)
    return g


def np_rng(root: int, *keys: int | str) -> np.random.Generator:
    return np.random.Generator(np.random.Philox(key=derive_seed(root, *keys)))


def philox_key(root: int, *keys: int | str) -> tuple[int, int]:
    """Two 32-bit key words for the device Philox stream of a purpose."""
    s = derive_seed(root, *keys)
    return s & MASK32, (s >> 32) & MASK32


def philox_keys(root: int, prefix: tuple, last: list) -> list[tuple[int, int]]:
    """``[philox_key(root, *prefix, k) for k in last]`` (bitwise the same): the hash state of (root, *prefix) is built
    once and copied per key - a round's per-client keys (128 clients) cost ~0.2 ms of host time per round otherwise."""
    h0 = hashlib.blake2b(digest_size=8)
    h0.update(int(root).to_bytes(8, "little", signed=False))
    for k in prefix:
        if isinstance(k, str):
            k = PURPOSE[k] if k in PURPOSE else int.from_bytes(
                hashlib.blake2b(k.encode(), digest_size=8).digest(), "little")
        h0.update(int(k & 0xFFFFFFFFFFFFFFFF).to_bytes(8, "little", signed=False))
    out = []
    for k in last:
        h = h0.copy()
        h.update(int(int(k) & 0xFFFFFFFFFFFFFFFF).to_bytes(8, "little", signed=False))
        s = int.from_bytes(h.digest(), "little")
        out.append((s & MASK32, (s >> 32) & MASK32))
    return out


# ---------------------------------------------------------------------------
# Philox4x32-10, vectorised in torch int64 (CPU oracle of csrc/philox.h)
# ---------------------------------------------------------------------------

def _philox4x32_np(c: np.ndarray, k0, k1, rounds: int = 10) -> np.ndarray:
    """numpy uint64 Philox4x32: the product of two 32-bit words is exact in uint64 (no limb split)."""
    m = np.uint64(MASK32)
    c0, c1, c2, c3 = (c[..., i].astype(np.uint64) & m for i in range(4))
    k0 = np.broadcast_to(np.asarray(k0, dtype=np.uint64) & m, c0.shape).copy()
    k1 = np.broadcast_to(np.asarray(k1, dtype=np.uint64) & m, c0.shape).copy()
    M0, M1 = np.uint64(PHILOX_M0), np.uint64(PHILOX_M1)
    W0, W1 = np.uint64(PHILOX_W0), np.uint64(PHILOX_W1)
    s32 = np.uint64(32)
    for _ in range(rounds):
        p0 = c0 * M0
        p1 = c2 * M1
        c0, c1, c2, c3 = ((p1 >> s32) ^ c1 ^ k0) & m, p1 & m, ((p0 >> s32) ^ c3 ^ k1) & m, p0 & m
        k0 = (k0 + W0) & m
        k1 = (k1 + W1) & m
    return np.stack([c0, c1, c2, c3], axis=-1)


def philox4x32(counter: torch.Tensor, key0: int, key1: int, rounds: int = 10) -> torch.Tensor:
    """Philox4x32 on an int64 tensor ``counter[..., 4]`` of 32-bit words.

    Returns int64 tensor [..., 4] of 32-bit outputs.  Bit-identical to the device
    implementation in ``qfedx_amd/csrc/philox.h``.  CPU tensors use the numpy uint64 path; device
    tensors a limb-split int64 torch path (both tested against the known-answer vectors).
    """
    if counter.device.type == "cpu":
        k0 = key0.numpy() if isinstance(key0, torch.Tensor) else key0
        k1 = key1.numpy() if isinstance(key1, torch.Tensor) else key1
        out = _philox4x32_np(counter.to(torch.int64).numpy(), k0, k1, rounds)
        return torch.from_numpy(out.astype(np.int64))
    return _philox4x32_torch(counter, key0, key1, rounds)


def _philox4x32_torch(counter: torch.Tensor, key0, key1, rounds: int = 10) -> torch.Tensor:
    """int64 torch Philox (16-bit limb products: no uint64 multiply in torch), any device."""
    c0, c1, c2, c3 = (counter[..., i].to(torch.int64) & MASK32 for i in range(4))
    if isinstance(key0, torch.Tensor):   # per-row keys, broadcast against the counter
        k0 = (key0.to(torch.int64) & MASK32).expand_as(c0).clone()
        k1 = (key1.to(torch.int64) & MASK32).expand_as(c0).clone()
    else:
        k0 = torch.full_like(c0, key0 & MASK32)
        k1 = torch.full_like(c0, key1 & MASK32)

    def mul32(a, m):
        # a, m < 2^32: compute 64-bit product split into hi/lo using 16-bit limbs
        a_lo = a & 0xFFFF
        a_hi = a >> 16
        m_lo = m & 0xFFFF
        m_hi = m >> 16
        lo_lo = a_lo * m_lo
        hi_lo = a_hi * m_lo
        lo_hi = a_lo * m_hi
        hi_hi = a_hi * m_hi
        cross = (lo_lo >> 16) + (hi_lo & 0xFFFF) + (lo_hi & 0xFFFF)
        lo = ((cross & 0xFFFF) << 16) | (lo_lo & 0xFFFF)
        hi = hi_hi + (hi_lo >> 16) + (lo_hi >> 16) + (cross >> 16)
        return hi & MASK32, lo & MASK32

    for _ in range(rounds):
        hi0, lo0 = mul32(c0, PHILOX_M0)
        hi1, lo1 = mul32(c2, PHILOX_M1)
        c0, c1, c2, c3 = (hi1 ^ c1 ^ k0) & MASK32, lo1, (hi0 ^ c3 ^ k1) & MASK32, lo0
        k0 = (k0 + PHILOX_W0) & MASK32
        k1 = (k1 + PHILOX_W1) & MASK32
    return torch.stack([c0, c1, c2, c3], dim=-1)


def philox_uniform(n: int, key: tuple[int, int], stream: int = 0, offset: int = 0) -> torch.Tensor:
    """n uniform float32 in (0, 1] from Philox counter (offset+i//4, stream, 0, 0)."""
    nblk = (n + 3) // 4
    idx = torch.arange(nblk, dtype=torch.int64) + offset
    ctr = torch.stack([idx & MASK32, (idx >> 32) & MASK32,
                       torch.full_like(idx, stream & MASK32), torch.zeros_like(idx)], -1)
    out = philox4x32(ctr, key[0], key[1]).reshape(-1)[:n]
    # (x + 1) * 2^-32 in (0, 1]; computed in float64 then rounded like the device does
    return ((out.to(torch.float64) + 1.0) * (1.0 / 4294967296.0)).to(torch.float32)


def philox_uniform_rows(keys: torch.Tensor, n: int, stream: int = 0) -> torch.Tensor:
    """[K, n] uniforms, row k from key ``keys[k]`` (int64 [K, 2]); runs on keys.device (GPU ok).

    Row k equals ``philox_uniform(n, tuple(keys[k]), stream)`` exactly.
    """
    K = keys.shape[0]
    nblk = (n + 3) // 4
    idx = torch.arange(nblk, dtype=torch.int64, device=keys.device)
    ctr = torch.stack([idx & MASK32, (idx >> 32) & MASK32, torch.full_like(idx, stream & MASK32),
                       torch.zeros_like(idx)], -1)[None].expand(K, nblk, 4)
    out = philox4x32(ctr, keys[:, 0:1], keys[:, 1:2]).reshape(K, -1)[:, :n]
    return ((out.to(torch.float64) + 1.0) * (1.0 / 4294967296.0)).to(torch.float32)


def philox_normal(n: int, key: tuple[int, int], stream: int = 0, offset: int = 0) -> torch.Tensor:
    """n standard normals via Box-Muller on Philox uniforms (pairs)."""
    m = n + (n & 1)
    u = philox_uniform(m, key, stream, offset).to(torch.float64)
    u1, u2 = u[0::2], u[1::2]
    r = torch.sqrt(-2.0 * torch.log(u1))
    z = torch.stack([r * torch.cos(2 * np.pi * u2), r * torch.sin(2 * np.pi * u2)], -1).reshape(-1)
    return z[:n].to(torch.float32)


def keyed_permutation(n: int, root: int, *keys: int | str) -> torch.Tensor:
    return torch.randperm(n, generator=generator(root, *keys))

