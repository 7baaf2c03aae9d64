"""Exact column-environment contraction of the CNOT-chain hardware-efficient VQC (the MPS fast path).

Circuit (models/vqc.py): F(x_q)|0> on every qubit, then L layers of  RZ(phi_lq) RX(theta_lq)  on every qubit followed
by the chain CNOT(0,1) CNOT(1,2) ... CNOT(n-2,n-1).  Write CNOT(q, q+1) = sum_k |k><k|_q (x) X^k_{q+1}: the index k
is a bond between column q and column q+1, one per layer.  Qubit q's column then maps its left bond word a (bit l =
the layer-l CNOT from q-1) and right bond word b (bit l = the layer-l CNOT to q+1) to a 2-vector,

    A_q[a, :, b] = P_{b_L} X^{a_L} G_L ... P_{b_1} X^{a_1} G_1 F(x_q) |0>,      G_l = RZ(phi_lq) RX(theta_lq),

which is an EXACT matrix-product state of bond D = 2^L (q = 0 has no left bond, q = n - 1 no right bond and no
projectors).  Every column is built independently, with no MPO application, no QR and no SVD.

Readout and gradients run on transfer environments of the doubled network, D x D matrices per cut:
    Rp_q = sum_s A_q[s]^* Rp_{q+1} A_q[s]^T-ish (right, no observable),  Lp_q (left),
    LO_q / RO_q = the same with one term w_c Z_c of O = sum_c w_c Z_c on the left / right of the cut,
    <Z_c> = contraction of Lp_c, A_c^* Z A_c, Rp_{c+1};
    d<O>/dx = 2 Re sum conj(A[a,s,b]) dA[a',s,b'] (Lp[a,a'] RO[b,b'] + LO[a,a'] Rp[b,b'] + w_q z_s Lp Rp)  for a
    parameter x of column q (reverse mode through the column's 2 x 2 chain gives dA for all 2L angles at once).
Cost per sample O(n D^3), no state vector, no tensor-network library calls: csrc/mps_chain.hip runs one wave per sample.
This module is the float64 numpy oracle of that kernel (tests/test_mps_chain.py checks it against the dense
statevector; tests/test_gpu_mps_chain.py checks the kernel against it).
"""
from __future__ import annotations

import numpy as np

_FEATURES = {"ry": 0, "rx": 1, "rz": 2}


def eligible(spec) -> bool:
    """The column contraction covers the angle-encoded RX/RZ + CNOT-chain VQC with 1..3 layers (bond <= 8)."""
    return (spec.entangler == "chain" and not spec.amplitude and not getattr(spec, "noisy", False)
            and spec.feature_map.lower() in _FEATURES and 1 <= spec.n_layers <= 3 and spec.n_qubits >= 2
            and spec.n_classes <= 8)


def _rx(t):
    c, s = np.cos(t / 2), np.sin(t / 2)
    return np.array([[c, -1j * s], [-1j * s, c]])


def _rz(p):
    return np.diag([np.exp(-0.5j * p), np.exp(0.5j * p)])


def _feature(x, kind):
    c, s = np.cos(x / 2), np.sin(x / 2)
    if kind == "rx":
        return np.array([c, -1j * s])
    if kind == "rz":
        return np.array([np.exp(-0.5j * x), 0.0])
    return np.array([c, s + 0j])


def _column(xq, th, ph, q, n, L, kind, a, b, deriv=None):
    """A_q[a, :, b] (2-vector); ``deriv`` = (layer, 0 theta | 1 phi) differentiates that gate."""
    v = _feature(xq, kind)
    for ell in range(L):
        rx, rz = _rx(th[ell]), _rz(ph[ell])
        if deriv == (ell, 0):
            rx = -0.5j * np.array([[0, 1], [1, 0]]) @ rx
        if deriv == (ell, 1):
            rz = -0.5j * np.diag([1, -1]) @ rz
        v = rz @ (rx @ v)
        if q > 0 and (a >> ell) & 1:
            v = v[::-1].copy()
        if q < n - 1:
            keep = (b >> ell) & 1
            v = np.array([v[0], 0]) if keep == 0 else np.array([0, v[1]])
    return v


def _site(xq, th, ph, q, n, L, kind, deriv=None):
    Dl = 1 if q == 0 else 1 << L
    Dr = 1 if q == n - 1 else 1 << L
    A = np.zeros((Dl, 2, Dr), dtype=complex)
    for a in range(Dl):
        for b in range(Dr):
            A[a, :, b] = _column(xq, th, ph, q, n, L, kind, a, b, deriv)
    return A


def _env_right(A, R, zsign=None):
    """sum_{s,b,b'} conj(A[a,s,b]) (z_s) A[a',s,b'] R[b,b'] -> [a, a']."""
    Az = A if zsign is None else A * np.array([1, -1])[None, :, None]
    return np.einsum("asb,xsy,by->ax", A.conj(), Az, R)


def _env_left(Lm, A, zsign=None):
    Az = A if zsign is None else A * np.array([1, -1])[None, :, None]
    return np.einsum("ax,asb,xsy->by", Lm, A.conj(), Az)


def chain_columns(x, theta, n, L, readout, feature="ry", w=None):
    """x [S, n] feature angles, theta [S, 2 n L] (RX angle of (layer l, qubit q) at 2 (l n + q), RZ at + 1)
    -> z [S, C] (= <Z_c>), and with ``w`` [S, C] also grad [S, 2 n L] of sum_c w_c <Z_c> (float64 numpy)."""
    x, theta = np.asarray(x, np.float64), np.asarray(theta, np.float64)
    S, C = x.shape[0], len(readout)
    z = np.zeros((S, C))
    grad = np.zeros((S, 2 * n * L)) if w is not None else None
    for si in range(S):
        th = theta[si, 0::2].reshape(L, n)
        ph = theta[si, 1::2].reshape(L, n)
        A = [_site(x[si, q], th[:, q], ph[:, q], q, n, L, feature) for q in range(n)]
        Rp = [None] * (n + 1)
        Rp[n] = np.ones((1, 1), dtype=complex)
        for q in range(n - 1, -1, -1):
            Rp[q] = _env_right(A[q], Rp[q + 1])
        Lp = np.ones((1, 1), dtype=complex)
        for c_i, c in enumerate(readout):
            Lc = np.ones((1, 1), dtype=complex)
            for q in range(c):
                Lc = _env_left(Lc, A[q])
            z[si, c_i] = np.einsum("ax,asb,xsy,by->", Lc, A[c].conj(), A[c] * np.array([1, -1])[None, :, None],
                                   Rp[c + 1]).real
        if w is None:
            continue
        wq = np.zeros(n)
        for c_i, c in enumerate(readout):
            wq[c] += w[si, c_i]
        RO = [None] * (n + 1)
        RO[n] = np.zeros((1, 1), dtype=complex)
        for q in range(n - 1, -1, -1):
            RO[q] = _env_right(A[q], RO[q + 1]) + wq[q] * _env_right(A[q], Rp[q + 1], zsign=True)
        Lp = np.ones((1, 1), dtype=complex)
        LO = np.zeros((1, 1), dtype=complex)
        for q in range(n):
            for ell in range(L):
                for kind_i in range(2):
                    dA = _site(x[si, q], th[:, q], ph[:, q], q, n, L, feature, deriv=(ell, kind_i))
                    t = (np.einsum("ax,asb,xsy,by->", Lp, A[q].conj(), dA, RO[q + 1])
                         + np.einsum("ax,asb,xsy,by->", LO, A[q].conj(), dA, Rp[q + 1])
                         + wq[q] * np.einsum("ax,asb,xsy,by->", Lp, A[q].conj(),
                                             dA * np.array([1, -1])[None, :, None], Rp[q + 1]))
                    grad[si, 2 * (ell * n + q) + kind_i] = 2 * t.real
            Lp, LO = _env_left(Lp, A[q]), _env_left(LO, A[q]) + wq[q] * _env_left(Lp, A[q], zsign=True)
    return z, grad
