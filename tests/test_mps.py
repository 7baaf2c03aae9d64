"""MPS (tensor-network) backend vs the dense float64 oracle (ROADMAP.md:85-87): amplitudes, <Z>, adjoint
(reverse-mode) and parameter-shift gradients, truncation bookkeeping, engine / simulator / FL integration,
and a 40-qubit circuit checked through its causal light cone against a dense 8-qubit simulation."""
import numpy as np
import pytest
import torch

from qfedx_amd.models.vqc import VQCSpec
from qfedx_amd.ops.engine import VQCEngine
from qfedx_amd.ops.statevec_torch import TorchProgram
from qfedx_amd.quantum.circuit import Circuit, Parameter
from qfedx_amd.quantum.mps import MPS, MPSProgram, program_exact_bond
from qfedx_amd.quantum.simulator import Simulator


def _random_circuit(n, depth, seed):
    rng = np.random.default_rng(seed)
    c = Circuit(n)
    k = 0
    for _ in range(depth):
        for q in range(n):
            g = rng.choice(["rx", "ry", "rz", "p", "h", "s", "t", "sx", "y"])
            if g in ("rx", "ry", "rz", "p"):
                getattr(c, g)(Parameter("v", k), q)
                k += 1
            else:
                getattr(c, g)(q)
        for _ in range(n // 2):
            a, b = rng.choice(n, 2, replace=False)
            (c.cx if rng.random() < 0.6 else c.cz)(int(a), int(b))
    c.swap(0, n - 1)
    return c, k


@pytest.mark.parametrize("seed", [0, 1, 2])
def test_mps_amplitudes_and_grads_match_dense(seed):
    n = 7
    circ, k = _random_circuit(n, 3, seed)
    ops, coef = circ.to_program({"v": 0})
    tp = TorchProgram(ops, coef, n, dtype=torch.complex128)
    mp = MPSProgram(ops, coef, n, dtype=torch.complex128, chi_max=64)
    g = torch.Generator().manual_seed(seed)
    rows = torch.randn(3, k, generator=g, dtype=torch.float64)
    psi = tp.run(rows)
    st = mp.run(rows)
    assert max(st.bonds()) <= 8                                 # lossless trims keep cuts at their Schmidt cap
    np.testing.assert_allclose(st.to_dense().numpy(), psi.numpy(), atol=1e-12)
    ro = [0, 3, 6]
    np.testing.assert_allclose(mp.expz(st, ro).numpy(), tp.expz(psi, ro).numpy(), atol=1e-12)
    w = torch.randn(3, 3, generator=g, dtype=torch.float64)
    ref = tp.adjoint_grads(rows, psi, w, ro)
    np.testing.assert_allclose(mp.adjoint_grads(rows, st, w, ro).numpy(), ref.numpy(), atol=1e-11)
    np.testing.assert_allclose(mp.param_shift_grads(rows, w, ro).numpy(), ref.numpy(), atol=1e-11)


def test_dense_roundtrip_and_initial_state():
    g = torch.Generator().manual_seed(4)
    psi = torch.randn(2, 1 << 6, generator=g, dtype=torch.complex128)
    psi = psi / psi.norm(dim=-1, keepdim=True)
    m = MPS.from_dense(psi)
    assert m.bonds() == [2, 4, 8, 4, 2]
    np.testing.assert_allclose(m.to_dense().numpy(), psi.numpy(), atol=1e-13)
    circ, k = _random_circuit(6, 2, 5)
    ops, coef = circ.to_program({"v": 0})
    rows = torch.randn(2, k, generator=g, dtype=torch.float64)
    tp = TorchProgram(ops, coef, 6, dtype=torch.complex128)
    mp = MPSProgram(ops, coef, 6, dtype=torch.complex128)
    ref = tp.run(rows, state=psi)
    np.testing.assert_allclose(mp.run(rows, state=psi).to_dense().numpy(), ref.numpy(), atol=1e-12)
    w = torch.randn(2, 2, generator=g, dtype=torch.float64)
    np.testing.assert_allclose(mp.adjoint_grads(rows, None, w, [1, 4], init=psi).numpy(),
                               tp.adjoint_grads(rows, ref, w, [1, 4]).numpy(), atol=1e-11)


def test_truncation_bounds_bond_and_tracks_discarded_weight():
    n = 10
    circ, k = _random_circuit(n, 6, 7)
    ops, coef = circ.to_program({"v": 0})
    rows = torch.randn(2, k, generator=torch.Generator().manual_seed(0), dtype=torch.float64)
    exact = MPSProgram(ops, coef, n, dtype=torch.complex128, chi_max=32)
    small = MPSProgram(ops, coef, n, dtype=torch.complex128, chi_max=4)
    assert exact.exact and not small.exact and not small.autograd_ok
    s1, s2 = exact.run(rows), small.run(rows)
    assert max(s2.bonds()) <= 4 and float(s2.trunc_err.min()) > 1e-3 and float(s1.trunc_err.max()) < 1e-20
    z1, z2 = exact.expz(s1, [0, 5]), small.expz(s2, [0, 5])
    assert torch.all(z2.abs() <= 1 + 1e-9)
    assert torch.all((z1 - z2).abs() <= s2.error_bound()[:, None] + 1e-9)
    # gradients under truncation fall back to parameter shift (finite, one per parametric gate)
    g = small.adjoint_grads(rows, s2, torch.ones(2, 2, dtype=torch.float64), [0, 5])
    assert torch.isfinite(g).all()


def test_exact_bond_of_chain_ansatz_is_two_to_the_layers():
    for L in (1, 2, 3, 4):
        ops, _ = VQCSpec(24, L, 3).program()
        assert program_exact_bond([tuple(r) for r in ops.tolist()], 24) == 1 << L


def _lightcone_circuit(n, L):
    c = Circuit(n)
    for q in range(n):
        c.ry(Parameter("v", 500 + q), q)
    for layer in range(L):
        for q in range(n):
            c.rx(Parameter("v", 100 * layer + 2 * q), q)
            c.rz(Parameter("v", 100 * layer + 2 * q + 1), q)
        for q in range(n - 1):
            c.cx(q, q + 1)
    return c


def test_40_qubit_circuit_matches_dense_light_cone():
    """<Z_c> of a CNOT-chain circuit depends only on qubits <= c + L: a 40-qubit MPS run (a 2^40 state
    would need 8 TiB) must equal the dense 8-qubit simulation on the shared parameters."""
    L, ro = 2, [0, 1, 2]
    big, small = Simulator(_lightcone_circuit(40, L), ro, backend="mps"), Simulator(_lightcone_circuit(8, L), ro)
    g = torch.Generator().manual_seed(1)
    v = torch.rand(4, 540, generator=g) * 3
    _, z_big = big.run(v)
    _, z_small = small.run(v)
    np.testing.assert_allclose(z_big.numpy(), z_small.numpy(), atol=2e-5)
    w = torch.randn(4, 3, generator=g)
    _, g_big = big.vjp(v, w)
    _, g_small = small.vjp(v, w)
    np.testing.assert_allclose(g_big[:, :g_small.shape[1]].numpy(), g_small.numpy(), atol=5e-5)


@pytest.mark.parametrize("method", ["adjoint", "param_shift", "autograd"])
def test_engine_mps_matches_statevector(method):
    spec = VQCSpec(6, 2, 3, readout_scale=2.0)
    K, B = 2, 4
    g = torch.Generator().manual_seed(2)
    x = spec.encode_features(torch.rand(K, B, 6, generator=g))
    y = torch.randint(0, 3, (K, B), generator=g)
    w = torch.full((K, B), 1.0 / B)
    params = torch.stack([spec.init_params(k) for k in range(K)]) + 0.3
    ref = VQCEngine(spec, "cpu", "torch").loss_and_grads(x, y, w, params, "adjoint")
    out = VQCEngine(spec, "cpu", "mps").loss_and_grads(x, y, w, params, method)
    np.testing.assert_allclose(out["loss"].numpy(), ref["loss"].numpy(), atol=1e-5)
    np.testing.assert_allclose(out["grad"].numpy(), ref["grad"].numpy(), atol=1e-4)


def test_federated_run_with_mps_simulator():
    from qfedx_amd.api import run_experiment
    from tests.test_fl import small_cfg
    # SGD: Adam would turn float noise on the zero-gradient last-layer RZ angles into +-lr steps
    out = run_experiment(small_cfg(num_rounds=2, simulator="mps", n_qubits=4, optimizer="sgd"))
    ref = run_experiment(small_cfg(num_rounds=2, n_qubits=4, optimizer="sgd"))
    assert np.allclose(out["accuracies"], ref["accuracies"], atol=0.02)
    assert torch.allclose(out["params"], ref["params"], atol=1e-4)
