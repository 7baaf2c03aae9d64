"""Circuit IR, float64 oracle, encoders (reference API parity), engine gradients, planner emulation."""
import math

import numpy as np
import pytest
import torch
from hypothesis import given, settings, strategies as st

from qfedx_amd.models.vqc import VQCSpec
from qfedx_amd.ops.engine import VQCEngine
from qfedx_amd.ops.statevec_torch import TorchProgram
from qfedx_amd.quantum.circuit import Circuit, ParameterVector, gate_matrix
from qfedx_amd.quantum.encoders import (amplitude_encode, amplitude_states, angle_encode, angle_product_states,
                                        get_statevector_from_circuit, normalize_for_amplitude)
from qfedx_amd.quantum.statevector import Statevector, apply_matrix


def _kron_1q(U, q, n):
    M = np.array([[1.0]])
    for qq in reversed(range(n)):
        M = np.kron(M, U if qq == q else np.eye(2))
    return M


def test_oracle_matches_kron():
    rng = np.random.default_rng(0)
    psi = rng.normal(size=16) + 1j * rng.normal(size=16)
    for q in range(4):
        U = gate_matrix("ry", 0.37 * (q + 1))
        assert np.allclose(apply_matrix(psi, U, [q], 4), _kron_1q(U, q, 4) @ psi)


def test_bell_and_draw():
    qc = Circuit(2, "bell")
    qc.h(0)
    qc.cx(0, 1)
    sv = Statevector.from_instruction(qc)
    assert np.allclose(sv.data, [1 / math.sqrt(2), 0, 0, 1 / math.sqrt(2)])
    txt = qc.draw(output="text")
    assert "H" in txt and "■" in txt


def test_amplitude_encode_reference_api():
    with pytest.raises(ValueError, match="Vector length must be a power of 2 for amplitude encoding. Got 3"):
        amplitude_encode(np.ones(3))
    qc = amplitude_encode(np.arange(16, dtype=float))
    assert qc.name == "AmplitudeEncode" and qc.num_qubits == 4
    sv = get_statevector_from_circuit(qc)
    assert np.allclose(sv.data, np.arange(16) / np.linalg.norm(np.arange(16)))
    assert np.allclose(normalize_for_amplitude(np.zeros(8)), np.full(8, 1 / math.sqrt(8)))  # zero -> uniform
    assert torch.allclose(amplitude_states(torch.zeros(1, 4)).real, torch.full((1, 4), 0.5))


def test_angle_encode_reference_api():
    f = np.array([0.1, 0.5, 0.9, 0.3])
    for basis in ("ry", "rx", "rz", "RY", "foo"):
        qc = angle_encode(f, 4, basis)
        assert qc.name == f"AngleEncode_{basis.upper()}"
    qc = angle_encode(f, 4, "ry")
    sv = Statevector.from_instruction(qc).data
    ref = angle_product_states(torch.tensor(f)[None], "ry", "minmax")[0].numpy()
    assert np.allclose(sv, ref)
    # constant vector -> all-zero angles -> |0000>
    assert np.isclose(abs(Statevector.from_instruction(angle_encode(np.ones(4), 4)).data[0]), 1)
    assert angle_encode(np.arange(16.0), 4).num_qubits == 4   # pools 16 -> 4


@settings(max_examples=20, deadline=None)
@given(st.integers(1, 5), st.integers(0, 10_000))
def test_unitarity_norm_preserved(n, seed):
    rng = np.random.default_rng(seed)
    qc = Circuit(n)
    for _ in range(8):
        q = int(rng.integers(n))
        g = rng.choice(["rx", "ry", "rz", "h", "sx", "t"])
        if g in ("rx", "ry", "rz"):
            getattr(qc, g)(float(rng.normal()), q)
        else:
            getattr(qc, g)(q)
        if n > 1:
            a, b = rng.choice(n, 2, replace=False)
            qc.cx(int(a), int(b))
    sv = Statevector.from_instruction(qc)
    assert np.isclose(np.linalg.norm(sv.data), 1.0)


def _engine_setup(n=4, L=2, K=2, B=5, seed=0):
    spec = VQCSpec(n_qubits=n, n_layers=L, n_classes=3, init_std=0.8, readout_scale=2.0)
    g = torch.Generator().manual_seed(seed)
    x = torch.rand(K, B, n, generator=g)
    y = torch.randint(0, 3, (K, B), generator=g)
    w = torch.full((K, B), 1.0 / B)
    p = torch.stack([spec.init_params(seed + k) for k in range(K)])
    p[:, : spec.n_theta] += torch.randn(K, spec.n_theta, generator=g)
    return spec, spec.encode_features(x), y, w, p


def test_adjoint_equals_param_shift_equals_autograd():
    """ROADMAP.md:27 - parameter-shift gradients match adjoint within tolerance."""
    spec, x, y, w, p = _engine_setup()
    eng = VQCEngine(spec)
    ga = eng.loss_and_grads(x, y, w, p, "adjoint")["grad"]
    gp = eng.loss_and_grads(x, y, w, p, "param_shift")["grad"]
    gt = eng.loss_and_grads(x, y, w, p, "autograd")["grad"]
    assert torch.allclose(ga, gt, atol=1e-5) and torch.allclose(gp, gt, atol=1e-5)


def test_finite_difference_check():
    spec, x, y, w, p = _engine_setup(n=3, L=1, K=1, B=3)
    eng = VQCEngine(spec)
    g = eng.loss_and_grads(x, y, w, p, "adjoint")["grad"][0]
    eps = 1e-3
    for i in [0, 2, spec.n_theta - 1, spec.n_theta]:
        pp, pm = p.clone().double(), p.clone().double()
        pp[0, i] += eps
        pm[0, i] -= eps
        lp = eng.loss_and_grads(x, y, w, pp.float(), "autograd")["loss"]
        lm = eng.loss_and_grads(x, y, w, pm.float(), "autograd")["loss"]
        assert abs(float((lp - lm) / (2 * eps)) - float(g[i])) < 2e-3


def test_spsa_is_unbiased_direction():
    spec, x, y, w, p = _engine_setup()
    eng = VQCEngine(spec)
    g = eng.loss_and_grads(x, y, w, p, "adjoint")["grad"][:, : spec.n_theta]
    est = torch.stack([eng.loss_and_grads(x, y, w, p, "spsa", spsa_c=0.01, rng_keys=(s,))["grad"][:, : spec.n_theta]
                       for s in range(60)]).mean(0)
    cos = torch.nn.functional.cosine_similarity(est.reshape(-1), g.reshape(-1), dim=0)
    assert cos > 0.5


def test_engine_matches_oracle():
    spec, x, y, w, p = _engine_setup(n=5, L=2, K=1, B=2)
    eng = VQCEngine(spec)
    z = eng.expz(x, p[:, : spec.n_theta])
    sv = Statevector.from_instruction(spec.circuit(), {"theta": p[0, : spec.n_theta].double().numpy(),
                                                        "x": x[0, 1].double().numpy()})
    assert np.allclose(z[0, 1].numpy(), [sv.expectation_z(c) for c in spec.readout], atol=1e-5)


def test_generic_program_torch_engine_matches_oracle():
    rng = np.random.default_rng(5)
    n = 4
    th = ParameterVector("theta", 6)
    qc = Circuit(n)
    qc.h(0)
    qc.rx(th[0], 1)
    qc.ry(th[1], 2)
    qc.cz(0, 3)
    qc.p(th[2], 3)
    qc.sx(1)
    qc.swap(1, 2)
    qc.rz(2.0 * th[3] + 0.1, 0)
    qc.t(2)
    qc.cx(3, 1)
    qc.y(0)
    vals = rng.normal(size=6)
    ops, coef = qc.to_program({"theta": 0})
    prog = TorchProgram(ops, coef, n, dtype=torch.complex128)
    st = prog.run(torch.from_numpy(vals)[None])[0].numpy()
    assert np.allclose(st, Statevector.from_instruction(qc, {"theta": vals}).data)
