"""Client-batched local optimizers on flat parameter buffers [K, P] (one row per client).

Reference: a fresh ``SGD(lr, momentum=0.9)`` per client per round (``Classical_FL.py:53``), so
momentum resets every round.  ROADMAP.md:38 adds Adam and SPSA.  State is allocated per round
(reset) by default, matching the reference; ``persistent=True`` keeps it across rounds.

On GPU the update runs as one fused kernel over all clients (``qfx_adam_kernel`` /
``qfx_sgdm_kernel`` in ``csrc/train_kernels.hip``; the per-client step counter ping-pongs between two
buffers so the counter update needs no launch of its own); the torch version is the CPU path / oracle.
Rows with ``active[k] == 0`` are left untouched (clients whose local epochs are exhausted).
"""
from __future__ import annotations

from typing import Optional

import torch


class BatchedOptimizer:
    def __init__(self, kind: str, shape, device, lr: float, momentum: float = 0.9,
                 betas=(0.9, 0.999), eps: float = 1e-8, backend: str = "torch", zero_init: bool = True):
        self.kind = kind.lower()
        self.lr = lr
        self.momentum = momentum
        self.b1, self.b2 = betas
        self.eps = eps
        self.backend = backend
        # zero_init=False: the state is left unset until init_round() (the round prologue kernel zeroes it)
        alloc = torch.zeros if zero_init else torch.empty
        self.m = alloc(shape, dtype=torch.float32, device=device)
        self.v = alloc(shape, dtype=torch.float32, device=device) if self.kind == "adam" else None
        self._t = alloc(2, shape[0], dtype=torch.float32, device=device)
        self._phase = 0
        self._fresh = zero_init

    @property
    def t(self) -> torch.Tensor:
        return self._t[self._phase]

    def reset(self) -> None:
        self.m.zero_()
        if self.v is not None:
            self.v.zero_()
        self._t.zero_()
        self._phase = 0
        self._fresh = True

    def init_round(self, params: torch.Tensor, theta: torch.Tensor) -> None:
        """params[k] = theta for every client row and the optimizer state reset (HIP: one kernel)."""
        if self.backend == "hip":
            from ..ops._ext import ext
            # SGD-momentum never reads its buffer on a client's first active step: only Adam's moments are zeroed
            m = self.m if self.kind == "adam" else None
            ext().round_init(theta.float().contiguous(), params, m, self.v, self._t)
            self._phase = 0
            self._fresh = True
            return
        params.copy_(theta[None, :].expand_as(params))
        self.reset()

    def init_state(self):
        """(m, v, t) for a round-prologue kernel that does ``init_round``'s work itself (HIP backend): the
        optimizer counts as freshly reset once that kernel is queued."""
        if self.backend != "hip":
            raise RuntimeError("init_state() is for the fused HIP round prologue")
        self._phase = 0
        self._fresh = True
        return (self.m if self.kind == "adam" else None), self.v, self._t

    def fused_adam(self, params: torch.Tensor, active: torch.Tensor):
        """Hand this step's Adam update to a kernel that fuses it (the MFMA engine's gradient reduction,
        ``hea_grad_reduce``): returns ([m, v, t_in, t_out, active], [lr, b1, b2, eps]) and does ``step``'s
        bookkeeping (counter ping-pong), or None when that path does not apply (not HIP Adam)."""
        if self.kind != "adam" or self.backend != "hip" or not params.is_cuda:
            return None
        if not self._fresh:
            raise RuntimeError("BatchedOptimizer(zero_init=False): call init_round() or reset() first")
        t_in, t_out = self._t[self._phase], self._t[1 - self._phase]
        self._phase ^= 1
        return ([self.m, self.v, t_in, t_out, active.float().contiguous()],
                [float(self.lr), float(self.b1), float(self.b2), float(self.eps)])

    def fused_sgdm(self, last: bool = False) -> Optional[dict]:
        """Hand this step's SGD-momentum update to the kernels that produce the gradient (the CFed step kernels'
        sink, csrc/cnn_args.h): returns the state they update (momentum rows, step-counter ping-pong, lr, mu, keep)
        and does ``step``'s bookkeeping, or None when that path does not apply (not HIP SGD)."""
        if self.kind not in ("sgd", "sgdm", "spsa") or self.backend != "hip" or not self.m.is_cuda:
            return None
        if not self._fresh:
            raise RuntimeError("BatchedOptimizer(zero_init=False): call init_round() or reset() first")
        t_in, t_out = self._t[self._phase], self._t[1 - self._phase]
        self._phase ^= 1
        return {"buf": self.m, "t_in": t_in, "t_out": t_out, "lr": float(self.lr), "mu": float(self.momentum),
                "keep": not last}

    @torch.no_grad()
    def step(self, params: torch.Tensor, grads: torch.Tensor, active: Optional[torch.Tensor] = None,
             last: bool = False) -> None:
        """One update of every active client row.  ``last``: no later step of this round reads the optimizer
        state (it is reset by the next ``init_round``), so the HIP SGD-momentum path skips storing its buffer."""
        if active is None:
            active = torch.ones(params.shape[0], device=params.device)
        active = active.to(params.dtype)
        if not self._fresh:
            raise RuntimeError("BatchedOptimizer(zero_init=False): call init_round() or reset() first")
        if self.backend == "hip":
            from ..ops import fedavg_hip
            t_in, t_out = self._t[self._phase], self._t[1 - self._phase]
            if self.kind == "adam":
                fedavg_hip.adam_step(params, grads, self.m, self.v, t_in, t_out, active, self.lr, self.b1,
                                     self.b2, self.eps)
            else:
                fedavg_hip.sgdm_step(params, grads, self.m, t_in, t_out, active, self.lr, self.momentum,
                                     keep_state=not last)
            self._phase ^= 1
            return
        a = active[:, None]
        if self.kind == "adam":
            self._t[self._phase] += active
            t = self.t.clamp(min=1.0)[:, None]
            m_new = self.b1 * self.m + (1 - self.b1) * grads
            v_new = self.b2 * self.v + (1 - self.b2) * grads * grads
            self.m = torch.where(a > 0, m_new, self.m)
            self.v = torch.where(a > 0, v_new, self.v)
            mhat = self.m / (1 - self.b1 ** t)
            vhat = self.v / (1 - self.b2 ** t)
            params -= a * self.lr * mhat / (vhat.sqrt() + self.eps)
        elif self.kind in ("sgd", "sgdm", "spsa"):
            # torch.optim.SGD semantics: buf = mu*buf + g ; p -= lr*buf (first step buf = g)
            first = (self.t == 0)[:, None]
            buf = torch.where(first, grads, self.momentum * self.m + grads)
            self.m = torch.where(a > 0, buf, self.m)
            self._t[self._phase] += active
            params -= a * self.lr * self.m
        else:
            raise ValueError(f"unknown optimizer '{self.kind}'")
