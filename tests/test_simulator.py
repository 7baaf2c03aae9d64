"""Public batched simulator (quantum/simulator.py) on arbitrary circuits: states, <Z>, adjoint VJP and
initial-state (amplitude encoding) runs vs the float64 oracle; plus the planner's load-from-state mode
through the register-level emulator (what the HIP kernels execute)."""
import numpy as np
import pytest
import torch

from qfedx_amd.quantum.circuit import Circuit, ParameterVector
from qfedx_amd.quantum.simulator import Simulator
from qfedx_amd.quantum.statevector import Statevector


def _random_circuit(n, n_par, seed, gates=40):
    rng = np.random.default_rng(seed)
    th = ParameterVector("theta", n_par)
    qc = Circuit(n)
    for i in range(gates):
        r = rng.random()
        q = int(rng.integers(n))
        if r < 0.4:
            getattr(qc, ["rx", "ry", "rz", "p"][int(rng.integers(4))])(th[i % n_par] * float(rng.uniform(0.5, 1.5)), q)
        elif r < 0.6:
            getattr(qc, ["h", "x", "y", "z", "s", "sdg", "t", "tdg", "sx"][int(rng.integers(9))])(q)
        else:
            a, b = rng.choice(n, 2, replace=False)
            (qc.cx if r < 0.85 else qc.cz)(int(a), int(b))
    return qc


def _oracle(qc, vals, init=None):
    sv = Statevector(np.asarray(init, dtype=complex)) if init is not None else Statevector.zero(qc.n_qubits)
    return sv.evolve(qc, {"theta": vals})


@pytest.mark.parametrize("n,seed", [(3, 0), (5, 1), (7, 2)])
def test_simulator_torch_states_expz_vjp(n, seed):
    qc = _random_circuit(n, 6, seed)
    sim = Simulator(qc, readout=[0, n - 1])
    rng = np.random.default_rng(seed)
    vals = rng.normal(size=(3, 6))
    psi, z = sim.run(torch.tensor(vals))
    for s in range(3):
        ref = _oracle(qc, vals[s])
        assert np.abs(psi[s].numpy() - ref.data).max() < 1e-5
        assert np.allclose(z[s].numpy(), [ref.expectation_z(0), ref.expectation_z(n - 1)], atol=1e-5)
    w = rng.normal(size=(3, 2))
    _, g = sim.vjp(torch.tensor(vals), torch.tensor(w))
    eps = 1e-4
    for j in range(6):                                   # central finite differences on the oracle
        d = np.zeros(6)
        d[j] = eps
        for s in range(3):
            fp, fm = _oracle(qc, vals[s] + d), _oracle(qc, vals[s] - d)
            num = sum(w[s, c] * (fp.expectation_z(q) - fm.expectation_z(q)) / (2 * eps) for c, q in enumerate([0, n - 1]))
            assert abs(num - float(g[s, j])) < 2e-3


def test_simulator_initial_state_amplitude_encoding():
    from qfedx_amd.quantum.encoders import amplitude_states
    n = 4
    qc = _random_circuit(n, 4, 7, gates=20)
    x = torch.rand(2, 16)
    init = amplitude_states(x)
    vals = np.random.default_rng(0).normal(size=(2, 4))
    psi, _ = Simulator(qc, readout=[1]).run(torch.tensor(vals), initial_state=init)
    for s in range(2):
        assert np.abs(psi[s].numpy() - _oracle(qc, vals[s], init[s].numpy()).data).max() < 1e-5


@pytest.mark.parametrize("n,R,kmax", [(6, 4, 5), (9, 16, 7), (12, 16, 12)])
def test_planner_load_mode_emulated(n, R, kmax):
    C = pytest.importorskip("qfedx_amd._qfedx_C", reason="native extension not built")
    from qfedx_amd.ops.plan_tools import emulate_pass, parse_blob
    qc = _random_circuit(n, 5, n, gates=50)
    ops, coef = qc.to_program({"theta": 0})
    info = parse_blob(C.plan(torch.from_numpy(ops), torch.from_numpy(coef), n, R, kmax, [0, n - 1], 5, 1, 3))
    rng = np.random.default_rng(n)
    init = rng.normal(size=1 << n) + 1j * rng.normal(size=1 << n)
    init /= np.linalg.norm(init)
    vals = rng.normal(size=5)
    psi = init.copy()
    for p in info["passes"]:
        out = emulate_pass(info, p, psi, None, vals, np.zeros(1), None, False, None)
    ref = _oracle(qc, vals, init)
    assert np.abs(psi - ref.data).max() < 1e-6
    assert np.allclose(out, [ref.expectation_z(0), ref.expectation_z(n - 1)], atol=1e-6)
