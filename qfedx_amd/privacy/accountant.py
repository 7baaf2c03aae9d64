"""RDP privacy accountant for the subsampled Gaussian mechanism.

ROADMAP.md:56-58,62,140-141 asks for epsilon(q, sigma, T, delta) "with Opacus"; Opacus is not
installed here, so this implements the same mathematics directly (Mironov, Talwar, Zhang 2019,
"Renyi Differential Privacy of the Sampled Gaussian Mechanism": integer orders by the binomial
expansion, fractional orders by the two-sided erfc series) and the RDP -> (eps, delta)
conversion of Balle et al. 2020 (``improved``, Opacus' default) or Mironov 2017 (``classic``).

State is tiny (orders + accumulated rdp) and checkpointable.
"""
from __future__ import annotations

import functools
import math
from typing import Iterable, Optional

import numpy as np
from scipy import special

DEFAULT_ORDERS = [1.0 + x / 10.0 for x in range(1, 100)] + [float(a) for a in range(12, 64)]


def _logadd(a: float, b: float) -> float:
    if a == -np.inf:
        return b
    if b == -np.inf:
        return a
    hi, lo = max(a, b), min(a, b)
    return hi + math.log1p(math.exp(lo - hi))


def _logsub(a: float, b: float) -> float:
    if b == -np.inf:
        return a
    if a < b:
        raise ValueError("log-sub of a larger number")
    if a == b:
        return -np.inf
    return a + math.log1p(-math.exp(b - a))


def _log_erfc(x: float) -> float:
    return math.log(2.0) + float(special.log_ndtr(-x * math.sqrt(2.0)))


def _log_a_int(q: float, sigma: float, alpha: int) -> float:
    acc = -np.inf
    for i in range(alpha + 1):
        term = (math.log(special.binom(alpha, i)) + i * math.log(q) + (alpha - i) * math.log1p(-q)
                + (i * i - i) / (2.0 * sigma ** 2))
        acc = _logadd(acc, term)
    return acc


def _log_a_frac(q: float, sigma: float, alpha: float) -> float:
    a0, a1 = -np.inf, -np.inf
    z0 = sigma ** 2 * math.log(1.0 / q - 1.0) + 0.5
    i = 0
    while True:
        coef = special.binom(alpha, i)
        lc = math.log(abs(coef))
        j = alpha - i
        t0 = lc + i * math.log(q) + j * math.log1p(-q)
        t1 = lc + j * math.log(q) + i * math.log1p(-q)
        e0 = math.log(0.5) + _log_erfc((i - z0) / (math.sqrt(2.0) * sigma))
        e1 = math.log(0.5) + _log_erfc((z0 - j) / (math.sqrt(2.0) * sigma))
        s0 = t0 + (i * i - i) / (2.0 * sigma ** 2) + e0
        s1 = t1 + (j * j - j) / (2.0 * sigma ** 2) + e1
        if coef > 0:
            a0, a1 = _logadd(a0, s0), _logadd(a1, s1)
        else:
            a0, a1 = _logsub(a0, s0), _logsub(a1, s1)
        i += 1
        if max(s0, s1) < -30:
            break
    return _logadd(a0, a1)


def rdp_sampled_gaussian(q: float, sigma: float, alpha: float) -> float:
    """RDP of one step of the sampled Gaussian mechanism at order alpha."""
    if q == 0:
        return 0.0
    if sigma == 0:
        return np.inf
    if q == 1.0:
        return alpha / (2.0 * sigma ** 2)
    if np.isinf(alpha):
        return np.inf
    if float(alpha).is_integer():
        return _log_a_int(q, sigma, int(alpha)) / (alpha - 1)
    return _log_a_frac(q, sigma, alpha) / (alpha - 1)


@functools.lru_cache(maxsize=256)
def _rdp_curve(q: float, sigma: float, orders: tuple) -> np.ndarray:
    # one step of the sampled Gaussian at every order: depends only on (q, sigma), so a training run
    # (fixed q, sigma every round) evaluates the series once instead of once per round
    out = np.array([rdp_sampled_gaussian(q, sigma, a) for a in orders])
    out.setflags(write=False)
    return out


def compute_rdp(q: float, sigma: float, steps: int, orders: Iterable[float] = DEFAULT_ORDERS) -> np.ndarray:
    return _rdp_curve(float(q), float(sigma), tuple(float(a) for a in orders)) * steps


def eps_from_rdp(orders, rdp, delta: float, conversion: str = "improved") -> tuple[float, float]:
    orders = np.asarray(orders, dtype=float)
    rdp = np.asarray(rdp, dtype=float)
    if conversion == "classic":
        eps = rdp - math.log(delta) / (orders - 1)
    else:
        eps = rdp - (math.log(delta) + np.log(orders)) / (orders - 1) + np.log((orders - 1) / orders)
    eps = np.where(np.isnan(eps), np.inf, eps)
    i = int(np.argmin(eps))
    return float(max(eps[i], 0.0)), float(orders[i])


class RDPAccountant:
    """Accumulates (q, sigma) steps; ``get_epsilon(delta)`` after each round (ROADMAP:57)."""

    def __init__(self, orders: Optional[list] = None):
        self.orders = list(orders or DEFAULT_ORDERS)
        self.rdp = np.zeros(len(self.orders))
        self.history: list[tuple[float, float, int]] = []

    def step(self, q: float, sigma: float, steps: int = 1) -> None:
        if sigma <= 0:
            self.rdp = self.rdp + np.inf
        else:
            self.rdp = self.rdp + compute_rdp(q, sigma, steps, self.orders)
        if self.history and self.history[-1][:2] == (q, sigma):
            self.history[-1] = (q, sigma, self.history[-1][2] + steps)
        else:
            self.history.append((q, sigma, steps))

    def get_epsilon(self, delta: float, conversion: str = "improved") -> float:
        if not self.history:
            return 0.0
        return eps_from_rdp(self.orders, self.rdp, delta, conversion)[0]

    def state_dict(self) -> dict:
        return {"orders": list(self.orders), "rdp": self.rdp.tolist(), "history": self.history}

    def load_state_dict(self, sd: dict) -> None:
        self.orders = list(sd["orders"])
        self.rdp = np.asarray(sd["rdp"], dtype=float)
        self.history = [tuple(h) for h in sd.get("history", [])]


def epsilon(q: float, sigma: float, steps: int, delta: float, conversion: str = "improved") -> float:
    acc = RDPAccountant()
    acc.step(q, sigma, steps)
    return acc.get_epsilon(delta, conversion)
