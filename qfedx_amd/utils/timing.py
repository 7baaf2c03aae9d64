"""Phase timers and profiler ranges (SURVEY §5 "Tracing / profiling").

The reference has no tracing.  ``PhaseTimer`` brackets the federated phases (local-train,
aggregate, comm, eval) with HIP events on GPU (no host sync inside the hot loop; the events
are resolved once per report) and ``time.perf_counter`` on CPU, and wraps each phase in a
``torch.profiler.record_function`` range so rocprofv3/roctracer and torch.profiler traces
carry the same names.
"""
from __future__ import annotations

import contextlib
import time
from collections import defaultdict

import torch


class PhaseTimer:
    # pending event pairs are folded into the totals once this many accumulate (bounded memory on long runs;
    # a blocking drain only if the GPU is a further MAX_PENDING phases behind)
    MAX_PENDING = 256

    def __init__(self, device: torch.device | str = "cpu", enabled: bool = True, every: int = 1):
        self.device = torch.device(device)
        self.enabled = enabled
        # GPU phases are timed on every ``every``-th round only (``step``): each HIP event recorded between two
        # round-graph launches idles the GPU for ~5 us on this stack (scripts/graph_gap.py)
        self.every = max(1, int(every))
        self.active = True
        self.gpu = self.device.type == "cuda"
        self._pending: list[tuple[str, object, object]] = []
        self.totals: dict[str, float] = defaultdict(float)
        self.counts: dict[str, int] = defaultdict(int)

    def step(self, round_num: int) -> None:
        self.active = round_num % self.every == 0

    def per_phase(self) -> dict[str, float]:
        """Mean milliseconds per timed occurrence of each phase (syncs once on GPU)."""
        tot = self.resolve()
        return {k: v / max(self.counts[k], 1) for k, v in tot.items()}

    @contextlib.contextmanager
    def phase(self, name: str):
        if not (self.enabled and self.active):
            yield
            return
        with torch.profiler.record_function(f"qfedx::{name}"):
            if self.gpu:
                s = torch.cuda.Event(enable_timing=True)
                e = torch.cuda.Event(enable_timing=True)
                s.record()
                yield
                e.record()
                self._pending.append((name, s, e))
                if len(self._pending) >= self.MAX_PENDING:
                    self._drain(block=len(self._pending) >= 2 * self.MAX_PENDING)
            else:
                t0 = time.perf_counter()
                yield
                self.totals[name] += (time.perf_counter() - t0) * 1e3
                self.counts[name] += 1

    def _drain(self, block: bool) -> None:
        """Fold finished phases into the totals, oldest first.  Non-blocking: stops at the first phase whose
        end event the GPU has not reached (``block``: waits for every pending phase)."""
        if block and self._pending:
            self._pending[-1][2].synchronize()
        done = 0
        for name, s, e in self._pending:
            if not block and not e.query():
                break
            self.totals[name] += s.elapsed_time(e)
            self.counts[name] += 1
            done += 1
        del self._pending[:done]

    def resolve(self) -> dict[str, float]:
        """Return accumulated milliseconds per phase (syncs once on GPU)."""
        self._drain(block=True)
        return dict(self.totals)

    def reset(self) -> None:
        self._pending.clear()
        self.totals.clear()
        self.counts.clear()


def sync(device) -> None:
    if torch.device(device).type == "cuda":
        torch.cuda.synchronize()
