"""Tables of the generic MPS HIP kernel (quantum/mps_mpo.py, csrc/mps_mpo.hip) on the CPU: the MPS its event lists
define (built by the torch emulator ``site_tensors``) equals the dense statevector for circuits with long-range CX /
CZ in both directions, ring entanglers and every 1-qubit kind; over-wide programs are refused."""
import numpy as np
import pytest
import torch

from qfedx_amd.models.vqc import VQCSpec
from qfedx_amd.ops.statevec_torch import TorchProgram
from qfedx_amd.quantum.circuit import Circuit, Parameter
from qfedx_amd.quantum.mps import MPS, MPSProgram
from qfedx_amd.quantum.mps_mpo import compile_mpo, site_tensors


def _wide_circuit(n, seed, n2q=6):
    """1-qubit gates of every kind, then CX / CZ between random (possibly distant) qubits, twice."""
    rng = np.random.default_rng(seed)
    c = Circuit(n)
    k = 0
    for _ in range(2):
        for q in range(n):
            g = rng.choice(["rx", "ry", "rz", "p", "h", "x", "y", "z", "s", "sdg", "t", "tdg", "sx"])
            if g in ("rx", "ry", "rz", "p"):
                getattr(c, g)(Parameter("v", k), q)
                k += 1
            else:
                getattr(c, g)(q)
        for _ in range(n2q // 2):
            a, b = rng.choice(n, 2, replace=False)
            (c.cx if rng.random() < 0.5 else c.cz)(int(a), int(b))
    return c, k


def _check(ops, coef, n, rows):
    tab = compile_mpo([tuple(int(v) for v in r) for r in ops.tolist()], n)
    mp = MPSProgram(ops, coef, n, dtype=torch.complex128, chi_max=16)
    ang = mp.angles(rows)
    dense = TorchProgram(ops, coef, n, dtype=torch.complex128).run(rows)
    st = MPS(site_tensors(tab, ang))
    np.testing.assert_allclose(st.to_dense().numpy(), dense.numpy(), atol=1e-12)
    return tab


@pytest.mark.parametrize("seed", [0, 1, 2, 3])
def test_event_tables_define_the_dense_state(seed):
    n = 7
    circ, k = _wide_circuit(n, seed)
    ops, coef = circ.to_program({"v": 0})
    cuts = [0] * (n - 1)
    for kind, q0, q1, _ in ops.tolist():
        if q1 >= 0:
            for c in range(min(q0, q1), max(q0, q1)):
                cuts[c] += 1
    assert max(cuts) <= 4                               # these seeds draw programs within bond 16
    rows = torch.randn(3, k, generator=torch.Generator().manual_seed(seed), dtype=torch.float64)
    _check(ops, coef, n, rows)


def test_ring_vqc_tables_match_dense():
    spec = VQCSpec(6, 2, 3, entangler="ring")
    ops, coef = spec.program()
    g = torch.Generator().manual_seed(1)
    x = spec.encode_features(torch.rand(2, 6, generator=g))
    th = torch.rand(2, spec.n_theta, generator=g, dtype=torch.float64) * 3
    rows = torch.cat([th, x.double()], -1)
    tab = _check(ops, coef, 6, rows)
    assert tab["nbits"].tolist() == [4] * 5             # chain + ring CX per layer: 2 bits per cut per layer


def test_too_wide_and_unsupported_programs_are_refused():
    spec = VQCSpec(6, 3, 3, entangler="ring")            # 6 gates across every cut: bond 64
    ops, _ = spec.program()
    with pytest.raises(ValueError, match="bond > 16"):
        compile_mpo([tuple(int(v) for v in r) for r in ops.tolist()], 6)
    with pytest.raises(ValueError, match="unsupported"):
        compile_mpo([(16, 0, -1, -1)], 3)
