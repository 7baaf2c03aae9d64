"""Tables of the generic MPS HIP kernel (csrc/mps_mpo.hip) and its torch emulator.

The einsum MPS (``quantum/mps.py``) applies a two-qubit gate as the bond-2 MPO |0><0| (x) I + |1><1| (x) U.  When
no recompression ever happens (``MPSProgram.autograd_ok``: at most log2(chi_max) two-qubit gates across any cut)
the final MPS is known in closed form, column by column:

* bit i of the bond word on cut c (between qubits c and c + 1) is k_g of the i-th two-qubit gate g, in program
  order, whose qubit span crosses c;
* qubit q's tensor for left / right words (a, b) is A_q[a, :, b] = E_m ... E_1 |0>, over q's own events in program
  order: its 1-qubit gates, the projector P_{k_g} where q is g's control (CX) or first qubit (CZ), X^{k_g} / Z^{k_g}
  where q is g's target;
* the column is zero unless every gate passing over q (crossing both of q's cuts) has the same bit in a and b.

``compile_mpo`` turns a lowered program (``Circuit.to_program`` / ``VQCSpec.program`` rows kind, q0, q1, slot) into
the kernel's int32 tables; ``site_tensors`` builds the same MPS with torch (CPU tests check it against the dense
statevector, so the bond-bit bookkeeping is verified without a GPU).  Bond words use the kernel's own bit order, not
the einsum network's; the state is the same.
"""
from __future__ import annotations

from typing import Dict, List, Sequence

import torch

from ..ops.statevec_torch import CX, CZ, P, PAULI, RX, RY, RZ, _u1

EV_GATE, EV_CTRL, EV_X, EV_Z = 0, 1, 2, 3
DMAX_BITS = 4                        # bond <= 16 (QFX_MPO_DMAX)
MAX_ROT_PER_QUBIT = 64               # QFX_MPO_MAXPG
ONE_QUBIT_KINDS = set(range(13)) | {PAULI}
ROTATIONS = (RX, RY, RZ, P)


def compile_mpo(ops_list: Sequence[Sequence[int]], n: int) -> Dict[str, torch.Tensor]:
    """-> {gkind [G], events [E], sinfo [n, 8], nbits [n - 1]} (int32, CPU).  Raises ValueError when a cut carries
    more than 4 two-qubit gates or an op kind is outside the kernel's set."""
    if n < 2:
        raise ValueError("the MPO kernel needs at least two qubits")
    cross: List[List[int]] = [[] for _ in range(n - 1)]
    for g, (kind, q0, q1, _) in enumerate(ops_list):
        if kind in (CX, CZ):
            for c in range(min(q0, q1), max(q0, q1)):
                cross[c].append(g)
        elif kind not in ONE_QUBIT_KINDS:
            raise ValueError(f"MPO kernel: unsupported op kind {kind}")
    nbits = [len(c) for c in cross]
    if max(nbits, default=0) > DMAX_BITS:
        raise ValueError(f"MPO kernel: a cut carries {max(nbits)} two-qubit gates (bond > 16)")
    pos = [{g: i for i, g in enumerate(c)} for c in cross]
    events: List[List[int]] = [[] for _ in range(n)]
    passes: List[List[tuple]] = [[] for _ in range(n)]
    nrot = [0] * n
    for g, (kind, q0, q1, _) in enumerate(ops_list):
        if kind in (CX, CZ):
            lo, hi = min(q0, q1), max(q0, q1)
            for q in range(lo, hi + 1):
                if lo < q < hi:                       # passes over q: same bit on both of q's cuts
                    passes[q].append((pos[q - 1][g], pos[q][g]))
                    continue
                side, bit = (1, pos[q][g]) if q == lo else (0, pos[q - 1][g])
                typ = EV_CTRL if q == q0 else (EV_X if kind == CX else EV_Z)
                events[q].append(typ | side << 2 | bit << 3 | g << 8)
        else:
            events[q0].append(EV_GATE | g << 8)
            nrot[q0] += kind in ROTATIONS
    if max(nrot) > MAX_ROT_PER_QUBIT:
        raise ValueError("MPO kernel: more than 64 rotations on one qubit")
    flat, sinfo = [], []
    for q in range(n):
        pt = 0
        for p, (i, j) in enumerate(passes[q]):
            pt |= (i | j << 2) << (4 * p)
        sinfo.append([len(flat), len(events[q]), pt, len(passes[q]), nrot[q], 0, 0, 0])
        flat.extend(events[q])
    i32 = dict(dtype=torch.int32)
    return {"gkind": torch.tensor([int(r[0]) for r in ops_list], **i32),
            "events": torch.tensor(flat or [0], **i32),
            "sinfo": torch.tensor(sinfo, **i32),
            "nbits": torch.tensor(nbits, **i32)}


def site_tensors(tab: Dict[str, torch.Tensor], ang: torch.Tensor, dtype=torch.complex128) -> List[torch.Tensor]:
    """The kernel's MPS built with torch: [B, Dl, 2, Dr] per qubit from the event tables (tests, small B)."""
    B = ang.shape[0]
    gkind = tab["gkind"].tolist()
    events = tab["events"].tolist()
    sinfo = tab["sinfo"].tolist()
    nbits = tab["nbits"].tolist()
    n = len(sinfo)
    rdt = torch.float64 if dtype == torch.complex128 else torch.float32
    out = []
    for q in range(n):
        off, cnt, pt, npt = sinfo[q][:4]
        Dl = 1 if q == 0 else 1 << nbits[q - 1]
        Dr = 1 if q == n - 1 else 1 << nbits[q]
        A = torch.zeros(B, Dl, 2, Dr, dtype=dtype)
        for a in range(Dl):
            for b in range(Dr):
                if any(((a >> ((pt >> 4 * p) & 3)) ^ (b >> ((pt >> (4 * p + 2)) & 3))) & 1 for p in range(npt)):
                    continue
                v0 = torch.ones(B, dtype=dtype)
                v1 = torch.zeros(B, dtype=dtype)
                for e in events[off:off + cnt]:
                    typ = e & 3
                    if typ == EV_GATE:
                        u = _u1(gkind[e >> 8], ang[:, e >> 8].to(rdt), dtype)
                        v0, v1 = u[0] * v0 + u[1] * v1, u[2] * v0 + u[3] * v1
                        continue
                    k = (((b if (e >> 2) & 1 else a) >> ((e >> 3) & 3)) & 1)
                    if typ == EV_CTRL:
                        v0, v1 = (v0 * 0, v1) if k else (v0, v1 * 0)
                    elif typ == EV_X and k:
                        v0, v1 = v1, v0
                    elif typ == EV_Z and k:
                        v1 = -v1
                A[:, a, 0, b] = v0
                A[:, a, 1, b] = v1
        out.append(A)
    return out
