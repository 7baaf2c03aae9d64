"""Float64 statevector oracle (CPU, numpy complex128).

Replaces Qiskit's ``Statevector.from_instruction`` (``src/QFed/qAmplitude.py:44-46``; callers read
``.data``, ``testEncoder.py:121``).  This is the golden reference every gfx950 kernel and the
torch engine are tested against (SURVEY §4 "Golden/oracle tests").
"""
from __future__ import annotations

from typing import Optional

import numpy as np

from .circuit import Circuit, gate_matrix


def apply_matrix(state: np.ndarray, U: np.ndarray, qubits, n: int) -> np.ndarray:
    """Apply a 2^k x 2^k matrix on ``qubits`` (little-endian local index) to a 2^n state."""
    k = len(qubits)
    psi = state.reshape([2] * n)  # C-order: tensor axis a <-> qubit n-1-a
    # local index bit j <-> qubits[j]; U as a tensor has out axes then in axes, most significant
    # local bit first, so tensor axis i (and k+i) <-> qubits[k-1-i]
    Ut = U.reshape([2] * (2 * k))
    in_axes_U = list(range(k, 2 * k))
    state_axes = [n - 1 - qubits[k - 1 - i] for i in range(k)]
    out = np.tensordot(Ut, psi, axes=(in_axes_U, state_axes))
    # out axes: U out axes (k, for qubits[k-1..0]) followed by remaining psi axes
    remaining = [a for a in range(n) if a not in state_axes]
    cur_order = state_axes + remaining
    perm = np.argsort(cur_order)
    out = np.transpose(out, perm)
    return out.reshape(-1)


class Statevector:
    def __init__(self, data, dims: Optional[int] = None):
        self.data = np.asarray(data, dtype=np.complex128).reshape(-1)
        n = int(round(np.log2(self.data.size)))
        if 2 ** n != self.data.size:
            raise ValueError("statevector length must be a power of 2")
        self.num_qubits = n

    @classmethod
    def zero(cls, n: int) -> "Statevector":
        v = np.zeros(2 ** n, np.complex128)
        v[0] = 1.0
        return cls(v)

    @classmethod
    def from_instruction(cls, circ: Circuit, values: Optional[dict] = None) -> "Statevector":
        return cls.zero(circ.n_qubits).evolve(circ, values)

    def evolve(self, circ: Circuit, values: Optional[dict] = None) -> "Statevector":
        n = self.num_qubits
        psi = self.data.copy()
        for ins in circ.instructions:
            if ins.name == "initialize":
                if len(ins.qubits) != n or list(ins.qubits) != list(range(n)):
                    # general: reset the sub-register then prepare (only from |0> on those qubits)
                    sub = np.zeros(2 ** n, np.complex128)
                    idx = np.arange(2 ** len(ins.qubits))
                    full = np.zeros_like(idx)
                    for j, q in enumerate(ins.qubits):
                        full |= ((idx >> j) & 1) << q
                    sub[full] = ins.matrix
                    psi = sub
                else:
                    psi = ins.matrix.astype(np.complex128).copy()
                continue
            if ins.name == "unitary":
                U = ins.matrix
            else:
                U = gate_matrix(ins.name, circ.resolve_angle(ins, values))
            psi = apply_matrix(psi, U, list(ins.qubits), n)
        return Statevector(psi)

    def probabilities(self) -> np.ndarray:
        return np.abs(self.data) ** 2

    def expectation_z(self, qubit: int) -> float:
        idx = np.arange(self.data.size)
        sign = 1.0 - 2.0 * ((idx >> qubit) & 1)
        return float(np.sum(self.probabilities() * sign))

    def expectation_z_string(self, qubits) -> float:
        idx = np.arange(self.data.size)
        par = np.zeros_like(idx)
        for q in qubits:
            par ^= (idx >> q) & 1
        return float(np.sum(self.probabilities() * (1.0 - 2.0 * par)))

    def inner(self, other: "Statevector") -> complex:
        return complex(np.vdot(self.data, other.data))

    def equiv(self, other: "Statevector", atol: float = 1e-8) -> bool:
        ov = abs(self.inner(other))
        return abs(ov - 1.0) < atol

    def __repr__(self) -> str:
        return f"Statevector({np.array2string(self.data, precision=4)}, dims={(2,) * self.num_qubits})"


def simulate(circ: Circuit, values: Optional[dict] = None) -> np.ndarray:
    return Statevector.from_instruction(circ, values).data
