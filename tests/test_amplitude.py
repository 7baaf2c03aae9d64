"""Amplitude-encoded VQC (model.feature_map=amplitude): the 2^n features are the normalised initial state
(reference ``amplitude_encode``, src/QFed/qAmplitude.py:25-41) and the trainable ansatz runs from it.
Checks: spec/program shape, torch adjoint vs complex128 autograd vs the float64 Statevector oracle,
planner load-mode emulation of the VQC program, and an end-to-end federated run on CPU."""
import numpy as np
import pytest
import torch

from qfedx_amd.models.vqc import VQCSpec
from qfedx_amd.ops.engine import VQCEngine
from qfedx_amd.quantum.statevector import Statevector


def _amp_setup(n=4, L=2, C=3, K=2, B=5, seed=0, ent="chain"):
    spec = VQCSpec(n_qubits=n, n_layers=L, n_classes=C, feature_map="amplitude", init_std=1.0,
                   entangler=ent, readout_scale=2.0)
    g = torch.Generator().manual_seed(seed)
    x = torch.rand(K, B, (1 << n) - 3, generator=g)        # short rows are zero-padded to 2^n
    y = torch.randint(0, C, (K, B), generator=g)
    w = torch.full((K, B), 1.0 / B)
    params = torch.stack([spec.init_params(seed + k) for k in range(K)])
    params[:, : spec.n_theta] += torch.randn(K, spec.n_theta, generator=g)
    return spec, x, y, w, params


def test_amplitude_spec_shape():
    spec = VQCSpec(n_qubits=5, n_layers=2, n_classes=3, feature_map="amplitude")
    assert spec.amplitude and spec.n_features == 32 and spec.x_width == 1
    ang = VQCSpec(n_qubits=5, n_layers=2, n_classes=3)
    assert spec.n_theta == ang.n_theta
    assert len(spec.circuit().instructions) == len(ang.circuit().instructions) - 5           # no feature-map rotations
    x = torch.rand(3, 7)
    init = spec.initial_states(x)
    assert init.shape == (3, 32) and torch.allclose(init.abs().pow(2).sum(-1), torch.ones(3))
    assert torch.allclose(spec.initial_states(torch.zeros(1, 32)).real, torch.full((1, 32), 32 ** -0.5))
    assert ang.initial_states(x) is None


def test_amplitude_engine_adjoint_matches_autograd_and_oracle():
    spec, x, y, w, params = _amp_setup()
    eng = VQCEngine(spec, "cpu", "torch")
    xa = spec.encode_features(x)
    init = spec.initial_states(x)
    adj = eng.loss_and_grads(xa, y, w, params, "adjoint", init=init)
    ag = eng.loss_and_grads(xa, y, w, params, "autograd", init=init)
    assert torch.allclose(adj["loss"], ag["loss"], atol=1e-5)
    assert torch.allclose(adj["grad"], ag["grad"], atol=1e-4)
    th = spec.split(params)[0]
    qc = spec.circuit()
    for k in range(2):
        for b in range(5):
            sv = Statevector(init[k, b].numpy().astype(complex)).evolve(
                qc, {"theta": th[k].double().numpy(), "x": np.zeros(spec.n_qubits)})
            z = [sv.expectation_z(q) for q in spec.readout]
            assert np.allclose(adj["expz"][k, b].numpy(), z, atol=1e-5)
    with pytest.raises(ValueError):
        eng.loss_and_grads(xa, y, w, params, "adjoint")                  # init is mandatory


@pytest.mark.parametrize("method", ["param_shift", "spsa"])
def test_amplitude_other_grad_methods(method):
    spec, x, y, w, params = _amp_setup(n=3, seed=2)
    eng = VQCEngine(spec, "cpu", "torch")
    xa, init = spec.encode_features(x), spec.initial_states(x)
    res = eng.loss_and_grads(xa, y, w, params, method, init=init)
    if method == "param_shift":
        ref = eng.loss_and_grads(xa, y, w, params, "adjoint", init=init)
        assert torch.allclose(res["grad"], ref["grad"], atol=1e-4)
    assert torch.isfinite(res["grad"]).all()


def test_amplitude_vqc_plan_load_mode_emulated():
    C = pytest.importorskip("qfedx_amd._qfedx_C", reason="native extension not built")
    from qfedx_amd.ops.plan_tools import FIN_READOUT, FIN_STORE, emulate_pass, parse_blob
    spec, x, *_ , params = _amp_setup(n=7, L=2, K=1, B=1, seed=3, ent="ring")
    ops, coef = spec.program()
    info = parse_blob(C.plan(torch.from_numpy(ops), torch.from_numpy(coef), spec.n_qubits, 16, 6, spec.readout,
                             spec.n_theta, 1, FIN_STORE | FIN_READOUT))
    init = spec.initial_states(x[0])[0].numpy().astype(complex)
    vals = spec.split(params)[0][0].double().numpy()
    psi = init.copy()
    for p in info["passes"]:
        out = emulate_pass(info, p, psi, None, vals, np.zeros(1), None, False, None)
    ref = Statevector(init).evolve(spec.circuit(), {"theta": vals, "x": np.zeros(spec.n_qubits)})
    assert np.abs(psi - ref.data).max() < 1e-6
    assert np.allclose(out, [ref.expectation_z(q) for q in spec.readout], atol=1e-6)


def test_amplitude_federated_run_cpu():
    from tests.test_fl import small_cfg
    from qfedx_amd.api import run_experiment
    out = run_experiment(small_cfg(num_rounds=3, feature_map="amplitude", n_qubits=3))
    assert np.isfinite(out["accuracies"][-1])
    assert out["history"][-1]["train_loss"] < out["history"][0]["train_loss"] + 1e-6


def test_amplitude_raw_init_equals_states():
    spec, x, y, w, params = _amp_setup(n=4, seed=5)
    eng = VQCEngine(spec, "cpu", "torch")
    xa = spec.encode_features(x)
    a = eng.loss_and_grads(xa, y, w, params, "adjoint", init=x)
    b = eng.loss_and_grads(xa, y, w, params, "adjoint", init=spec.initial_states(x))
    assert torch.equal(a["grad"], b["grad"]) and torch.equal(a["loss"], b["loss"])
    with pytest.raises(ValueError):
        eng.loss_and_grads(xa, y, w, params, "adjoint", init=torch.rand(2, 5, 17))   # > 2^n raw amplitudes
