"""Amplitude and angle encoders.

Reference API (kept: names, signatures, error text, circuit names, little-endian ordering):
  * ``normalize_for_amplitude`` - float64 L2 normalise, zero vector -> uniform ``1/sqrt(L)``
    (``src/QFed/qAmplitude.py:11-22``)
  * ``amplitude_encode`` - power-of-2 check with the exact ``ValueError`` text (``:32-33``),
    circuit name ``"AmplitudeEncode"`` (``:39``), ``initialize(state, qubits)`` (``:40``)
  * ``get_statevector_from_circuit`` (``:44-46``)
  * ``pool_to_n_features`` / ``angle_encode`` - per-sample min-max -> pi*x, RX/RZ/RY per qubit with
    RY fallback, name ``AngleEncode_{BASIS}`` (``src/QFed/qAngle.py:9-51``)

Batched device versions (``amplitude_states``, ``angle_product_states``) build the encoded
statevectors directly - no gate simulation; on GPU they run as the
``qfx_amplitude_init`` / product-state kernels of the extension.
"""
from __future__ import annotations

import math

import numpy as np
import torch

from ..data.features import pool_to_n_features, angle_scale
from .circuit import Circuit
from .statevector import Statevector


def normalize_for_amplitude(vec: np.ndarray) -> np.ndarray:
    v = np.asarray(vec, dtype=float)
    norm = np.linalg.norm(v)
    if norm == 0:
        return np.ones_like(v) / np.sqrt(v.size)
    return v / norm


def amplitude_encode(vector: np.ndarray) -> Circuit:
    v = np.asarray(vector, dtype=float)
    L = v.size
    if not (L != 0 and ((L & (L - 1)) == 0)):
        raise ValueError("Vector length must be a power of 2 for amplitude encoding. Got {}".format(L))
    n_qubits = int(np.log2(L))
    state = normalize_for_amplitude(v)
    qc = Circuit(n_qubits, name="AmplitudeEncode")
    qc.initialize(state, qc.qubits)
    return qc


def get_statevector_from_circuit(qc: Circuit) -> Statevector:
    return Statevector.from_instruction(qc)


def angle_encode(features: np.ndarray, n_qubits: int = None, basis: str = "ry") -> Circuit:
    f = np.asarray(features, dtype=float)
    if n_qubits is None:
        n_qubits = f.size
    if f.size != n_qubits:
        f = pool_to_n_features(f, n_qubits)
    if f.max() == f.min():
        normed = np.zeros_like(f)
    else:
        normed = (f - f.min()) / (f.max() - f.min())
    angles = normed * np.pi
    qc = Circuit(n_qubits, name=f"AngleEncode_{basis.upper()}")
    for i, ang in enumerate(angles):
        b = basis.lower()
        if b == "rx":
            qc.rx(float(ang), i)
        elif b == "rz":
            qc.rz(float(ang), i)
        else:
            qc.ry(float(ang), i)
    return qc


# ---------------------------------------------------------------------------
# batched torch encoders (complex64 [B, 2^n])
# ---------------------------------------------------------------------------

def amplitude_states(x: torch.Tensor) -> torch.Tensor:
    """[B, L] real -> normalised complex64 states [B, L] (zero rows -> uniform)."""
    L = x.shape[-1]
    if L & (L - 1):
        raise ValueError("Vector length must be a power of 2 for amplitude encoding. Got {}".format(L))
    xd = x.to(torch.float64)
    nrm = xd.norm(dim=-1, keepdim=True)
    uni = torch.full_like(xd, 1.0 / math.sqrt(L))
    out = torch.where(nrm > 0, xd / torch.where(nrm > 0, nrm, torch.ones_like(nrm)), uni)
    return out.to(torch.complex64)


def single_qubit_vectors(angles: torch.Tensor, basis: str = "ry") -> torch.Tensor:
    """angles [B, n] -> per-qubit 2-vectors R(angle)|0> as complex [B, n, 2]."""
    a = angles.to(torch.float64)
    c, s = torch.cos(a / 2), torch.sin(a / 2)
    z = torch.zeros_like(c)
    b = basis.lower()
    if b == "rx":
        v0, v1 = torch.complex(c, z), torch.complex(z, -s)
    elif b == "rz":
        v0, v1 = torch.complex(c, -s), torch.complex(z, z)
    else:
        v0, v1 = torch.complex(c, z), torch.complex(s, z)
    return torch.stack([v0, v1], -1)


def product_state(vecs: torch.Tensor) -> torch.Tensor:
    """Per-qubit 2-vectors [B, n, 2] -> full product state [B, 2^n] (qubit 0 = LSB)."""
    B, n, _ = vecs.shape
    state = vecs[:, n - 1, :]
    for q in range(n - 2, -1, -1):
        state = (state[:, :, None] * vecs[:, q, None, :]).reshape(B, -1)
    return state


def angle_product_states(features: torch.Tensor, basis: str = "ry", mode: str = "minmax",
                         alpha: float = math.pi) -> torch.Tensor:
    """Batched ``angle_encode`` statevectors [B, 2^n] (complex128) without gate simulation."""
    ang = angle_scale(features.to(torch.float64), mode, alpha)
    return product_state(single_qubit_vectors(ang, basis))
