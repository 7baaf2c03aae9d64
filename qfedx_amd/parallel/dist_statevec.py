"""Distributed statevector over ranks: one state sharded across GPUs by its top qubits.

With W = 2^g ranks, an n-qubit state is stored as W shards of 2^(n-g) amplitudes: physical bit positions
0..n-g-1 are *local* (inside a shard), positions n-g..n-1 are *global* (the rank index bits).  A logical
qubit -> physical position map ``perm`` lets the layout change as the circuit runs:

* a gate on local qubits runs inside the rank's shard.  Runs of such gates form *segments* executed by the
  single-GPU engine (HIP load-from-state plans on a GPU, the torch executor on CPU);
* SWAP gates are pure relabels of ``perm`` (no data moves);
* diagonal gates on a global qubit are per-rank phases.  CZ/CX *controlled* by a global qubit become a
  local Z/X on ranks whose control bit is 1.  These need no communication;
* any other gate on a global qubit first exchanges that qubit with a local one (the local qubit whose
  next use is furthest away, Belady).  The exchange is pairwise: rank r swaps the half of its shard whose
  local bit differs from its rank bit with partner r ^ 2^j.  That is one ``batch_isend_irecv`` of half a
  shard, which on MI355X goes over the direct xGMI link between the two GPUs (no ring, no all-to-all).

<Z_q> reductions are one all-reduce of [S, C] partial sums.  288 GB of HBM per GPU holds a 35-qubit
complex64 state, so W GPUs simulate 35 + log2(W) qubits.  Gradients: the parameter-shift rule over batched
parameter rows (``param_shift``), forward passes only.  The reference has no multi-device simulation
(ROADMAP.md:85-87 plans "statevector <= 20q; tensor network / cuQuantum beyond").
"""
from __future__ import annotations

import math
from dataclasses import dataclass
from typing import Optional

import torch
import torch.distributed as dist

from ..quantum.circuit import Circuit, DIAGONAL, ParamExpr, gate_matrix

_DIAG1 = DIAGONAL - {"cz"}


@dataclass
class _Seg:
    circuit: Circuit


@dataclass
class _Swap:
    j: int          # global bit (rank bit) index
    l: int          # local physical bit


@dataclass
class _Phase:
    name: str       # diagonal 1q gate applied to a global qubit with rank bit = 1 (d1) or 0 (d0)
    angle: object   # float or ParamExpr
    bit: int        # this rank's bit value of that qubit ("cz2": cz on two global qubits, both bits 1 -> -1)


class DistributedStatevector:
    """Batched n-qubit circuit simulation sharded over the ranks of ``torch.distributed``.

        ds = DistributedStatevector(circuit, world_size, rank, device)
        z = ds.expectation_z(values, readout)          # [S, C] on every rank
        g = ds.param_shift(values, w, readout)         # d(sum_c w <Z_c>)/dvalues [S, n_slots]
    """

    def __init__(self, circuit: Circuit, world_size: int, rank: int, device="cpu", backend: str = "auto",
                 slots: Optional[list] = None, group=None):
        if world_size & (world_size - 1):
            raise ValueError("world size must be a power of two")
        self.circuit = circuit
        self.n = circuit.n_qubits
        self.W, self.rank, self.group = world_size, rank, group
        self.g = int(math.log2(world_size))
        self.nl = self.n - self.g
        if self.nl < 2:
            raise ValueError(f"{self.n} qubits over {world_size} ranks leaves < 2 local qubits")
        self.device = torch.device(device)
        self.backend = ("hip" if self.device.type == "cuda" else "torch") if backend == "auto" else backend
        names = slots or []
        if not names:
            for p in circuit.parameters:
                if p.name not in names:
                    names.append(p.name)
        sizes: dict = {}
        for p in circuit.parameters:
            sizes[p.name] = max(sizes.get(p.name, 0), p.index + 1)
        self.slot_of, off = {}, 0
        for nm in names:
            self.slot_of[nm] = off
            off += sizes.get(nm, 0)
        self.n_slots = max(off, 1)
        self.steps, self.final_perm = self._schedule()
        self._execs: dict = {}

    # ------------------------------------------------------------------ schedule
    def _schedule(self):
        nl, ins = self.nl, self.circuit.instructions
        perm = list(range(self.n))                       # logical qubit -> physical position
        phys = list(range(self.n))                       # physical position -> logical qubit
        steps: list = []
        seg = Circuit(nl)

        def flush():
            nonlocal seg
            if seg.instructions:
                steps.append(_Seg(seg))
                seg = Circuit(nl)

        def bit_of(q):                                   # this rank's value of a global logical qubit
            return (self.rank >> (perm[q] - nl)) & 1

        def next_use(q, i0):
            for i in range(i0, len(ins)):
                if q in ins[i].qubits:
                    return i
            return len(ins) + 1

        for i, g in enumerate(ins):
            qs = g.qubits
            glob = [q for q in qs if perm[q] >= nl]
            if g.name == "swap":                         # relabel only
                a, b = perm[qs[0]], perm[qs[1]]
                perm[qs[0]], perm[qs[1]] = b, a
                phys[a], phys[b] = qs[1], qs[0]
                continue
            if glob and g.name in _DIAG1:
                flush()
                steps.append(_Phase(g.name, g.angle, bit_of(qs[0])))
                continue
            if glob and g.name == "cz":
                if len(glob) == 2:
                    if bit_of(qs[0]) and bit_of(qs[1]):
                        flush()
                        steps.append(_Phase("cz2", None, 1))
                    continue
                loc = qs[0] if glob[0] == qs[1] else qs[1]
                if bit_of(glob[0]):
                    seg.append("z", (perm[loc],))
                continue
            if glob and g.name == "cx" and perm[qs[1]] < nl and perm[qs[0]] >= nl:
                if bit_of(qs[0]):
                    seg.append("x", (perm[qs[1]],))
                continue
            for q in glob:                               # bring q local: swap with the furthest-used local
                busy = {perm[x] for x in qs}
                cand = [p for p in range(nl) if p not in busy]
                victim = max(cand, key=lambda p: (next_use(phys[p], i), -p))
                flush()
                j = perm[q] - nl
                steps.append(_Swap(j, victim))
                lq = phys[victim]
                perm[q], perm[lq] = victim, nl + j
                phys[victim], phys[nl + j] = q, lq
            seg.append(g.name, tuple(perm[q] for q in qs), g.angle, g.matrix)
        flush()
        return steps, perm

    @property
    def n_swaps(self) -> int:
        return sum(isinstance(s, _Swap) for s in self.steps)

    # ------------------------------------------------------------------ execution
    def _exec(self, k: int):
        ex = self._execs.get(k)
        if ex is None:
            seg = self.steps[k].circuit
            ops, coef = seg.to_program(self.slot_of)
            if self.backend == "hip":
                from ..ops.statevec_hip import HipProgram
                ex = HipProgram(ops, coef, self.nl, [0], self.device, n_theta=self.n_slots, x_width=1)
            else:
                from ..ops.statevec_torch import TorchProgram
                ex = TorchProgram(ops, coef, self.nl, self.device, torch.complex128)
            self._execs[k] = ex
        return ex

    def _angle(self, a, v: torch.Tensor) -> torch.Tensor:
        if isinstance(a, ParamExpr):
            return a.scale * v[:, self.slot_of[a.param.name] + a.param.index].double() + a.offset
        return torch.full((v.shape[0],), float(a or 0.0), dtype=torch.float64, device=v.device)

    def _exchange(self, psi: torch.Tensor, j: int, l: int) -> None:
        S = psi.shape[0]
        b = (self.rank >> j) & 1
        view = psi.view(S, -1, 2, 1 << l)[:, :, 1 - b, :]
        partner = self.rank ^ (1 << j)
        send = view.contiguous()
        recv = torch.empty_like(send)
        staged = dist.get_backend(self.group) == "gloo" and send.is_cuda
        if staged:                                       # gloo has no device p2p: stage through the host
            send, recv = send.cpu(), recv.cpu()
        reqs = dist.batch_isend_irecv([dist.P2POp(dist.isend, send, partner, self.group),
                                       dist.P2POp(dist.irecv, recv, partner, self.group)])
        for r in reqs:
            r.wait()
        view.copy_(recv.to(psi.device) if staged else recv)

    def initial_shard(self, S: int, initial_state: Optional[torch.Tensor] = None) -> torch.Tensor:
        dt = torch.complex64 if self.backend == "hip" else torch.complex128
        L = 1 << self.nl
        if initial_state is not None:                    # full logical states [S, 2^n] (identity layout)
            st = torch.as_tensor(initial_state).reshape(S, -1)
            return st[:, self.rank * L:(self.rank + 1) * L].to(self.device, dt).contiguous()
        psi = torch.zeros(S, L, dtype=dt, device=self.device)
        if self.rank == 0:
            psi[:, 0] = 1.0
        return psi

    def run(self, values, initial_state: Optional[torch.Tensor] = None) -> torch.Tensor:
        """Final local shards [S, 2^(n-g)] in the physical layout ``final_perm``."""
        v = torch.as_tensor(values, dtype=torch.float32, device=self.device)
        v = v[None] if v.dim() == 1 else v
        if v.shape[1] < self.n_slots:
            v = torch.cat([v, v.new_zeros(v.shape[0], self.n_slots - v.shape[1])], 1)
        S = v.shape[0]
        psi = self.initial_shard(S, initial_state)
        for k, st in enumerate(self.steps):
            if isinstance(st, _Seg):
                ex = self._exec(k)
                if self.backend == "hip":
                    psi = ex.statevector(torch.zeros(S, 1, 1, device=self.device), v.contiguous(), psi)[0]
                else:
                    psi = ex.run(v.double(), state=psi)
            elif isinstance(st, _Swap):
                self._exchange(psi, st.j, st.l)
            else:                                        # per-rank diagonal phase
                if st.name == "cz2":                     # cz on two global qubits, both bits 1
                    psi = -psi
                    continue
                d = torch.as_tensor(
                    [[complex(x) for x in gate_matrix(st.name, float(a)).diagonal()]
                     for a in self._angle(st.angle, v).tolist()], dtype=psi.dtype, device=psi.device)
                psi = psi * d[:, st.bit, None]
        return psi

    def expectation_z(self, values, readout: list, initial_state=None) -> torch.Tensor:
        psi = self.run(values, initial_state)
        return self.expz_from_shard(psi, readout)

    def expz_from_shard(self, psi: torch.Tensor, readout: list) -> torch.Tensor:
        p = psi.abs().pow(2).double()                    # [S, L]
        L = p.shape[1]
        idx = torch.arange(L, device=p.device)
        cols = []
        for q in readout:
            pos = self.final_perm[q]
            if pos < self.nl:
                sgn = 1.0 - 2.0 * ((idx >> pos) & 1).double()
                cols.append(p @ sgn)
            else:
                bit = (self.rank >> (pos - self.nl)) & 1
                cols.append(p.sum(1) * (1.0 - 2.0 * bit))
        z = torch.stack(cols, 1) if cols else p.new_zeros(p.shape[0], 0)
        if self.W > 1:
            zz = z.cpu() if (dist.get_backend(self.group) == "gloo" and z.is_cuda) else z
            dist.all_reduce(zz, group=self.group)
            z = zz.to(z.device)
        return z.float()

    def gather(self, psi: torch.Tensor) -> torch.Tensor:
        """Full logical states [S, 2^n] on every rank (tests / small n): all-gather + undo ``final_perm``."""
        parts = [torch.empty_like(psi) for _ in range(self.W)]
        if self.W > 1:
            src = psi.cpu() if (dist.get_backend(self.group) == "gloo" and psi.is_cuda) else psi
            parts = [torch.empty_like(src) for _ in range(self.W)]
            dist.all_gather(parts, src.contiguous(), group=self.group)
        else:
            parts = [psi]
        full = torch.cat([x.to(psi.device) for x in parts], 1)          # physical index = rank * L + local
        S = full.shape[0]
        # physical tensor axes (little-endian bit p <-> axis n-1-p); permute to logical order
        t = full.reshape(S, *([2] * self.n))
        phys_axis = {p: self.n - p for p in range(self.n)}              # +1 for the batch axis
        order = [0] + [phys_axis[self.final_perm[q]] for q in reversed(range(self.n))]
        return t.permute(order).reshape(S, -1)

    def param_shift(self, values, w, readout: list) -> torch.Tensor:
        """d(sum_c w[s,c] <Z_c>)/d values [S, n_slots] by the two-term shift rule.  Needs every slot to drive
        RX/RY/RZ/P gates with unit scale; a slot used by several gates is shifted per occurrence."""
        v = torch.as_tensor(values, dtype=torch.float32, device=self.device)
        v = v[None] if v.dim() == 1 else v
        w = torch.as_tensor(w, dtype=torch.float64, device=self.device).reshape(v.shape[0], len(readout))
        occ = [(i, g) for i, g in enumerate(self.circuit.instructions) if isinstance(g.angle, ParamExpr)]
        for _, g in occ:
            if g.name not in ("rx", "ry", "rz", "p") or abs(g.angle.scale - 1.0) > 1e-12:
                raise ValueError("param_shift needs unit-scale rx/ry/rz/p parametric gates")
        counts: dict = {}
        for _, g in occ:
            key = self.slot_of[g.angle.param.name] + g.angle.param.index
            counts[key] = counts.get(key, 0) + 1
        if any(c > 1 for c in counts.values()):
            raise ValueError("param_shift: each slot must drive one gate (shift rows are slot shifts)")
        S = v.shape[0]
        keys = sorted(counts)
        rows = v.repeat(2 * len(keys), 1)                                  # [(2J) S, P]
        for jj, key in enumerate(keys):
            rows[(2 * jj) * S:(2 * jj + 1) * S, key] += math.pi / 2
            rows[(2 * jj + 1) * S:(2 * jj + 2) * S, key] -= math.pi / 2
        z = self.expectation_z(rows, readout).double().view(len(keys), 2, S, -1)
        d = 0.5 * (z[:, 0] - z[:, 1])                                      # [J, S, C]
        grad = torch.zeros(S, self.n_slots, dtype=torch.float64, device=self.device)
        for jj, key in enumerate(keys):
            grad[:, key] = (d[jj] * w).sum(-1)
        return grad.float()
