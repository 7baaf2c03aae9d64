"""Quantum circuit IR (replaces the Qiskit ``QuantumCircuit`` the reference imports,
``src/QFed/qAmplitude.py:1-2``, ``qAngle.py:1``; Qiskit is not installable here).

Conventions match Qiskit: little-endian (amplitude index ``i``, bit ``k`` of ``i`` is qubit ``k``),
``RX(t) = exp(-i t X/2)`` etc.  Gate angles are affine expressions ``scale * param + offset`` of a
symbolic ``Parameter`` (trainable theta or data feature x) or plain floats.  ``to_program`` lowers a
circuit to the flat integer/float tables consumed by the C++ pass planner and the gfx950 kernels
(``qfedx_amd/csrc/statevec.hip``).
"""
from __future__ import annotations

import math
from dataclasses import dataclass, field
from typing import Optional, Sequence, Union

import numpy as np

# Gate kind codes shared with csrc/qfx_common.h (keep in sync).
KIND = {
    "rx": 0, "ry": 1, "rz": 2, "p": 3, "h": 4, "x": 5, "y": 6, "z": 7, "s": 8, "sdg": 9,
    "t": 10, "tdg": 11, "sx": 12, "cx": 13, "cz": 14, "swap": 15, "unitary": 16, "initialize": 17,
    "pauli": 18,   # noise-trajectory Pauli: the (per-sample) parameter value 0/1/2/3 selects I/X/Y/Z
}
PARAMETRIC = {"rx", "ry", "rz", "p"}
TWO_QUBIT = {"cx", "cz", "swap"}
DIAGONAL = {"rz", "p", "z", "s", "sdg", "t", "tdg", "cz"}
_ALIASES = {"cnot": "cx", "phase": "p", "i": None}


@dataclass(frozen=True)
class Parameter:
    name: str
    index: int = 0

    def __mul__(self, k: float) -> "ParamExpr":
        return ParamExpr(self, float(k), 0.0)

    __rmul__ = __mul__

    def __add__(self, c: float) -> "ParamExpr":
        return ParamExpr(self, 1.0, float(c))

    __radd__ = __add__

    def __str__(self) -> str:
        return f"{self.name}[{self.index}]"


@dataclass(frozen=True)
class ParamExpr:
    param: Parameter
    scale: float = 1.0
    offset: float = 0.0

    def __mul__(self, k: float) -> "ParamExpr":
        return ParamExpr(self.param, self.scale * k, self.offset * k)

    __rmul__ = __mul__

    def __add__(self, c: float) -> "ParamExpr":
        return ParamExpr(self.param, self.scale, self.offset + c)

    __radd__ = __add__

    def __str__(self) -> str:
        s = str(self.param) if self.scale == 1.0 else f"{self.scale:.3g}*{self.param}"
        return s if self.offset == 0 else f"{s}+{self.offset:.3g}"


class ParameterVector(list):
    def __init__(self, name: str, length: int):
        super().__init__(Parameter(name, i) for i in range(length))
        self.name = name


Angle = Union[float, Parameter, ParamExpr]


def _as_expr(a: Angle) -> Union[float, ParamExpr]:
    if isinstance(a, Parameter):
        return ParamExpr(a, 1.0, 0.0)
    if isinstance(a, ParamExpr):
        return a
    return float(a)


@dataclass
class Instruction:
    name: str
    qubits: tuple
    angle: Union[float, ParamExpr, None] = None
    matrix: Optional[np.ndarray] = None      # for 'unitary' / 'initialize' (state vector)

    @property
    def is_parametric(self) -> bool:
        return isinstance(self.angle, ParamExpr)


@dataclass
class Circuit:
    n_qubits: int
    name: str = "circuit"
    instructions: list = field(default_factory=list)

    # ---- construction -------------------------------------------------------
    @property
    def qubits(self) -> list[int]:
        return list(range(self.n_qubits))

    @property
    def num_qubits(self) -> int:
        return self.n_qubits

    def _q(self, q) -> int:
        q = int(q)
        if not 0 <= q < self.n_qubits:
            raise IndexError(f"qubit {q} out of range for {self.n_qubits}-qubit circuit")
        return q

    def append(self, name: str, qubits: Sequence[int], angle: Angle = None, matrix=None) -> "Circuit":
        name = _ALIASES.get(name, name)
        if name not in KIND:
            raise ValueError(f"unknown gate '{name}'")
        qs = tuple(self._q(q) for q in qubits)
        if len(set(qs)) != len(qs):
            raise ValueError("repeated qubit in gate")
        self.instructions.append(Instruction(name, qs, None if angle is None else _as_expr(angle), matrix))
        return self

    def rx(self, t: Angle, q: int): return self.append("rx", (q,), t)
    def ry(self, t: Angle, q: int): return self.append("ry", (q,), t)
    def rz(self, t: Angle, q: int): return self.append("rz", (q,), t)
    def p(self, t: Angle, q: int): return self.append("p", (q,), t)
    def h(self, q: int): return self.append("h", (q,))
    def x(self, q: int): return self.append("x", (q,))
    def y(self, q: int): return self.append("y", (q,))
    def z(self, q: int): return self.append("z", (q,))
    def s(self, q: int): return self.append("s", (q,))
    def sdg(self, q: int): return self.append("sdg", (q,))
    def t(self, q: int): return self.append("t", (q,))
    def tdg(self, q: int): return self.append("tdg", (q,))
    def sx(self, q: int): return self.append("sx", (q,))
    def pauli(self, sel: Angle, q: int): return self.append("pauli", (q,), sel)
    def cx(self, c: int, t: int): return self.append("cx", (c, t))
    cnot = cx
    def cz(self, a: int, b: int): return self.append("cz", (a, b))
    def swap(self, a: int, b: int): return self.append("swap", (a, b))

    def unitary(self, U: np.ndarray, qubits: Sequence[int]):
        U = np.asarray(U, dtype=np.complex128)
        if U.shape != (2 ** len(qubits),) * 2:
            raise ValueError("unitary shape mismatch")
        return self.append("unitary", tuple(qubits), None, U)

    def initialize(self, state, qubits=None):
        qubits = self.qubits if qubits is None else [self._q(q) for q in qubits]
        v = np.asarray(state, dtype=np.complex128).reshape(-1)
        if v.size != 2 ** len(qubits):
            raise ValueError("initialize: state size mismatch")
        if not np.isclose(np.linalg.norm(v), 1.0, atol=1e-8):
            raise ValueError("initialize: state must be normalized")
        return self.append("initialize", tuple(qubits), None, v)

    def compose(self, other: "Circuit") -> "Circuit":
        if other.n_qubits != self.n_qubits:
            raise ValueError("compose: qubit count mismatch")
        out = Circuit(self.n_qubits, self.name, list(self.instructions))
        out.instructions.extend(other.instructions)
        return out

    # ---- parameters ---------------------------------------------------------
    @property
    def parameters(self) -> list[Parameter]:
        seen, out = set(), []
        for ins in self.instructions:
            if ins.is_parametric and ins.angle.param not in seen:
                seen.add(ins.angle.param)
                out.append(ins.angle.param)
        return out

    @property
    def num_parameters(self) -> int:
        return len(self.parameters)

    def depth(self) -> int:
        level = [0] * self.n_qubits
        for ins in self.instructions:
            d = max(level[q] for q in ins.qubits) + 1
            for q in ins.qubits:
                level[q] = d
        return max(level) if level else 0

    def count_ops(self) -> dict:
        out: dict = {}
        for ins in self.instructions:
            out[ins.name] = out.get(ins.name, 0) + 1
        return out

    def resolve_angle(self, ins: Instruction, values: Optional[dict]) -> float:
        a = ins.angle
        if a is None:
            return 0.0
        if isinstance(a, float):
            return a
        if values is None:
            raise ValueError(f"unbound parameter {a.param}")
        key = a.param
        if key in values:
            v = values[key]
        elif a.param.name in values:
            v = values[a.param.name][a.param.index]
        else:
            raise ValueError(f"unbound parameter {a.param}")
        return a.scale * float(v) + a.offset

    # ---- lowering to the kernel program -------------------------------------
    def to_program(self, slot_of: dict) -> tuple[np.ndarray, np.ndarray]:
        """Lower to (ops int32 [G,4] = kind,q0,q1,slot ; coef float32 [G,2] = scale,offset).

        ``slot_of`` maps a parameter vector name to its slot base, e.g. ``{"theta": 0, "x": P}``;
        a constant angle gets slot -1 with the angle in ``offset``.
        """
        ops, coef = [], []
        for ins in self.instructions:
            if ins.name in ("unitary", "initialize"):
                raise ValueError(f"'{ins.name}' is not lowerable to the kernel program")
            if ins.name == "swap":  # SWAP = 3 CNOTs (kernels keep CNOT/diag/1q micro-ops only)
                a, b = ins.qubits
                for c, t in ((a, b), (b, a), (a, b)):
                    ops.append((KIND["cx"], c, t, -1))
                    coef.append((0.0, 0.0))
                continue
            q0 = ins.qubits[0]
            q1 = ins.qubits[1] if len(ins.qubits) > 1 else -1
            if isinstance(ins.angle, ParamExpr):
                base = slot_of[ins.angle.param.name]
                ops.append((KIND[ins.name], q0, q1, base + ins.angle.param.index))
                coef.append((ins.angle.scale, ins.angle.offset))
            else:
                ops.append((KIND[ins.name], q0, q1, -1))
                coef.append((0.0, float(ins.angle or 0.0)))
        return np.asarray(ops, np.int32).reshape(-1, 4), np.asarray(coef, np.float32).reshape(-1, 2)

    # ---- drawing ------------------------------------------------------------
    def draw(self, output: str = "text") -> str:
        if output != "text":
            raise ValueError("only output='text' is supported")
        return TextDrawing(self)

    def __str__(self) -> str:
        return str(self.draw())


class TextDrawing(str):
    """A ``str`` subclass so ``print(qc.draw(output='text'))`` works like Qiskit's."""

    def __new__(cls, circ: Circuit):
        n = circ.n_qubits
        rows = [[f"q_{q}: "] for q in range(n)]
        width = max(len(r[0]) for r in rows)
        rows = [[r[0].rjust(width)] for r in rows]
        for ins in circ.instructions:
            if ins.name == "initialize":
                vals = ",".join(f"{v.real:.3g}" for v in ins.matrix[:4])
                labels = {q: f"Initialize({vals}{',...' if ins.matrix.size > 4 else ''})" for q in ins.qubits}
            elif ins.name == "cx":
                labels = {ins.qubits[0]: "■", ins.qubits[1]: "X"}
            elif ins.name == "cz":
                labels = {ins.qubits[0]: "■", ins.qubits[1]: "■"}
            elif ins.name == "swap":
                labels = {ins.qubits[0]: "x", ins.qubits[1]: "x"}
            else:
                nm = ins.name.upper() if len(ins.name) <= 2 else ins.name.capitalize()
                if ins.angle is not None:
                    a = ins.angle
                    nm += f"({a:.3g})" if isinstance(a, float) else f"({a})"
                labels = {q: nm for q in ins.qubits}
            w = max(len(s) for s in labels.values()) + 2
            lo, hi = min(ins.qubits), max(ins.qubits)
            for q in range(n):
                if q in labels:
                    cell = labels[q].center(w, "─")
                elif lo < q < hi and len(ins.qubits) > 1:
                    cell = "┼".center(w, "─")
                else:
                    cell = "─" * w
                rows[q].append(cell)
        text = "\n".join("".join(r) + "─" for r in rows)
        header = f"{circ.name} ({n} qubits)\n" if circ.name else ""
        return super().__new__(cls, header + text)


def gate_matrix(name: str, angle: float = 0.0) -> np.ndarray:
    """2x2 (or 4x4) complex128 matrix of a gate (Qiskit conventions)."""
    c, s = math.cos(angle / 2), math.sin(angle / 2)
    if name == "rx":
        return np.array([[c, -1j * s], [-1j * s, c]])
    if name == "ry":
        return np.array([[c, -s], [s, c]], dtype=np.complex128)
    if name == "rz":
        return np.array([[np.exp(-0.5j * angle), 0], [0, np.exp(0.5j * angle)]])
    if name == "p":
        return np.array([[1, 0], [0, np.exp(1j * angle)]])
    if name == "pauli":
        return [np.eye(2), np.array([[0, 1], [1, 0]]), np.array([[0, -1j], [1j, 0]]),
                np.diag([1, -1])][int(round(angle))].astype(np.complex128)
    r2 = 1 / math.sqrt(2)
    fixed = {
        "h": np.array([[r2, r2], [r2, -r2]], dtype=np.complex128),
        "x": np.array([[0, 1], [1, 0]], dtype=np.complex128),
        "y": np.array([[0, -1j], [1j, 0]]),
        "z": np.array([[1, 0], [0, -1]], dtype=np.complex128),
        "s": np.array([[1, 0], [0, 1j]]),
        "sdg": np.array([[1, 0], [0, -1j]]),
        "t": np.array([[1, 0], [0, np.exp(0.25j * math.pi)]]),
        "tdg": np.array([[1, 0], [0, np.exp(-0.25j * math.pi)]]),
        "sx": 0.5 * np.array([[1 + 1j, 1 - 1j], [1 - 1j, 1 + 1j]]),
        # two-qubit, basis |q1 q0> with q0 = first listed qubit (control for cx)
        "cx": np.array([[1, 0, 0, 0], [0, 0, 0, 1], [0, 0, 1, 0], [0, 1, 0, 0]], dtype=np.complex128),
        "cz": np.diag([1, 1, 1, -1]).astype(np.complex128),
        "swap": np.array([[1, 0, 0, 0], [0, 0, 1, 0], [0, 1, 0, 0], [0, 0, 0, 1]], dtype=np.complex128),
    }
    return fixed[name]
