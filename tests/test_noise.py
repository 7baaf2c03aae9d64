"""Quantum noise model (ROADMAP.md:64-73): Pauli trajectories vs the exact density
matrix, readout confusion / shots statistics, and 'noise degrades accuracy' (ROADMAP.md:72-73).
The reference ships no noise implementation, so parity is against our own float64 density-matrix
oracle (parity unpinned w.r.t. the reference)."""
import math

import numpy as np
import pytest
import torch

from qfedx_amd.models.vqc import VQCSpec
from qfedx_amd.ops.engine import VQCEngine
from qfedx_amd.quantum.noise import NoiseModel, density_expz, pauli_probs, uniforms
from qfedx_amd.utils.seeding import philox_key, philox_uniform_rows


def _keys(n, purpose="noise_traj"):
    return torch.tensor([philox_key(7, purpose, 0, c) for c in range(n)], dtype=torch.int64)


@pytest.mark.parametrize("kind,p,gamma", [("depolarizing", 0.15, 0.0), ("amplitude_twirl", 0.0, 0.3)])
def test_trajectory_average_matches_density_matrix(kind, p, gamma):
    px, py, pz = pauli_probs(kind, p, gamma)
    nm = NoiseModel(px, py, pz)
    clean = VQCSpec(3, 1, 2, readout=[0, 2])
    noisy = VQCSpec(3, 1, 2, readout=[0, 2], noisy=True)
    g = torch.Generator().manual_seed(3)
    theta = torch.randn(1, clean.n_theta, generator=g) * 0.9
    x = torch.rand(1, 1, 3, generator=g) * 2.0
    M = 12000
    eng = VQCEngine(noisy, "cpu", "torch", noise=nm)
    xs = x.expand(1, M, 3)
    xa = eng.augment(xs, _keys(1), step=0)
    z = eng.expz(xa, theta)[0].double()                      # [M, C] one trajectory per row
    est, se = z.mean(0).numpy(), (z.std(0) / math.sqrt(M)).numpy()
    ops, coef = clean.program()
    slots = np.concatenate([theta[0].double().numpy(), x[0, 0].double().numpy()])
    exact = density_expz(ops, coef, 3, slots, clean.readout, (px, py, pz))
    ideal = density_expz(ops, coef, 3, slots, clean.readout, (0.0, 0.0, 0.0))
    assert np.all(np.abs(est - exact) < 4.5 * se + 1e-3), (est, exact, se)
    assert np.max(np.abs(exact - ideal)) > 0.02               # the channel is actually visible


def test_pauli_selector_frequencies():
    nm = NoiseModel(0.1, 0.05, 0.2)
    sel = nm.pauli_columns(_keys(4), B=500, n_ops=20, step=3)
    f = [(sel == v).float().mean().item() for v in (1, 2, 3)]
    assert abs(f[0] - 0.1) < 0.01 and abs(f[1] - 0.05) < 0.01 and abs(f[2] - 0.2) < 0.012


def test_uniform_stream_keyed_and_reproducible():
    k = _keys(3)
    a = uniforms(k, 100, 5)
    assert torch.equal(a, philox_uniform_rows(k, 100, 5)) and not torch.equal(a, uniforms(k, 100, 6))
    assert float(a.min()) > 0.0 and float(a.max()) <= 1.0


def test_readout_confusion_and_shots_statistics():
    z = torch.tensor([[[0.6, -0.2, 1.0]]]).expand(1, 4000, 3).contiguous()
    conf = NoiseModel(p01=0.05, p10=0.1)
    exp = (1 - 0.15) * z + (0.1 - 0.05)
    assert torch.allclose(conf.apply_readout(z, None, 0), exp)
    shots = NoiseModel(p01=0.05, p10=0.1, shots=200)
    zh = shots.apply_readout(z, _keys(1, "shots"), 0)
    mean, var = zh[0].mean(0), zh[0].var(0)
    ez = exp[0, 0]
    assert torch.all((mean - ez).abs() < 4 * torch.sqrt((1 - ez ** 2) / 200 / 4000) + 1e-6)
    assert torch.allclose(var, (1 - ez ** 2) / 200, rtol=0.15, atol=1e-4)
    k = (1 - zh) * 100                                           # 1 - 2k/S grid: k integer
    assert torch.all((k - k.round()).abs() < 1e-3)


def test_noise_degrades_accuracy():
    from tests.test_fl import small_cfg
    from qfedx_amd.api import run_experiment
    ideal = run_experiment(small_cfg(num_rounds=6))
    noisy = run_experiment(small_cfg(num_rounds=6, **{"noise.kind": "depolarizing", "noise.p": 0.25,
                                                       "noise.readout_p01": 0.1, "noise.readout_p10": 0.1}))
    assert noisy["accuracies"][-1] < ideal["accuracies"][-1] - 0.05


def test_batched_param_shift_matches_adjoint_and_general_path():
    spec = VQCSpec(4, 2, 3, readout_scale=2.0)
    eng = VQCEngine(spec, "cpu", "torch")
    g = torch.Generator().manual_seed(5)
    K, B = 3, 5
    xang = torch.rand(K, B, 4, generator=g) * 3
    y = torch.randint(0, 3, (K, B), generator=g)
    w = torch.full((K, B), 1.0 / B)
    params = spec.init_params(1)[None].repeat(K, 1) + 0.3 * torch.randn(K, spec.n_params, generator=g)
    adj = eng.loss_and_grads(xang, y, w, params, "adjoint")["grad"]
    ps = eng.loss_and_grads(xang, y, w, params, "param_shift")["grad"]
    assert eng._simple_shift_slots()
    assert torch.allclose(adj, ps, atol=1e-5)
    eng._budget = 8 * 16 * B * 3          # force many small chunks
    ps2 = eng.loss_and_grads(xang, y, w, params, "param_shift")["grad"]
    assert torch.allclose(ps, ps2, atol=1e-6)
    th = spec.split(params)[0]
    _, wr, _, _, _ = __import__("qfedx_amd.ops.engine", fromlist=["ce_readout"]).ce_readout(
        eng.expz(xang, th), y, w, *spec.split(params)[1:])
    gen = eng._param_shift(eng._rows(xang, th), wr, K, B)
    assert torch.allclose(gen, ps[:, :spec.n_theta], atol=1e-5)


def test_param_shift_with_shots_is_unbiased():
    spec = VQCSpec(3, 1, 2, readout_scale=2.0)
    nm = NoiseModel(shots=64)
    eng = VQCEngine(spec, "cpu", "torch", noise=nm)
    exact = VQCEngine(spec, "cpu", "torch")
    g = torch.Generator().manual_seed(2)
    K, B = 1, 400
    xang = (torch.rand(1, 1, 3, generator=g) * 3).expand(K, B, 3).contiguous()
    y = torch.zeros(K, B, dtype=torch.long)
    w = torch.full((K, B), 1.0 / B)
    params = spec.init_params(0)[None] + 0.5
    ref = exact.loss_and_grads(xang, y, w, params, "param_shift")["grad"][:, :spec.n_theta]
    keys = nm.client_keys("shots", 0, [0], "cpu")
    est = eng.loss_and_grads(xang, y, w, params, "param_shift", readout_keys=keys)["grad"][:, :spec.n_theta]
    # 400 samples x 64 shots per shifted circuit: the shot estimator is within a few sigma of exact
    assert torch.allclose(est, ref, atol=0.08), (est, ref)
    assert not torch.allclose(est, ref, atol=1e-6)


@pytest.mark.parametrize("kind,p,gamma", [("amplitude", 0.0, 0.25), ("depolarizing", 0.1, 0.0),
                                          ("amplitude_twirl", 0.0, 0.3)])
def test_density_simulator_matches_float64_kraus_oracle(kind, p, gamma):
    """ops/density.py (torch path, the CPU side of csrc/density.hip) == the float64 density-matrix oracle with the
    channel's exact Kraus operators after every gate (ROADMAP.md:66-69)."""
    from qfedx_amd.ops.density import DensityProgram, kraus_ops
    spec = VQCSpec(4, 2, 3, init_std=1.0, entangler="ring")
    ops, coef = spec.program()
    kr = kraus_ops(kind, p, gamma)
    prog = DensityProgram(ops, coef, 4, spec.readout, "cpu", kraus=kr)
    g = torch.Generator().manual_seed(3)
    rows = torch.cat([torch.randn(5, spec.n_theta, generator=g), torch.rand(5, 4, generator=g) * 3], -1).double()
    z = prog.expz(rows)
    for s in range(5):
        ref = density_expz(ops, coef, 4, rows[s].numpy(), spec.readout, (0, 0, 0), kraus=kr)
        assert np.allclose(z[s].numpy(), ref, atol=2e-6), (z[s], ref)


def test_exact_amplitude_damping_differs_from_twirl_and_decays():
    """Exact amplitude damping is not its Pauli twirl: |1> relaxes toward |0> (<Z> -> +1), which the twirl cannot
    do (its fixed point is the maximally mixed state)."""
    from qfedx_amd.ops.density import DensityProgram, kraus_ops
    from qfedx_amd.quantum.circuit import Circuit
    qc = Circuit(1)
    qc.x(0)                                      # |1>, then 12 gates that leave populations alone
    for _ in range(12):
        qc.z(0)
    ops, coef = qc.to_program({})
    rows = torch.zeros(1, 1, dtype=torch.float64)
    ex = DensityProgram(ops, coef, 1, [0], "cpu", kraus=kraus_ops("amplitude", gamma=0.3)).expz(rows)[0, 0]
    tw = DensityProgram(ops, coef, 1, [0], "cpu", kraus=kraus_ops("amplitude_twirl", gamma=0.3)).expz(rows)[0, 0]
    assert abs(float(ex) - (1 - 2 * 0.7 ** 13)) < 1e-6 and abs(float(tw) + 0.7 ** 13) < 1e-6


def test_amplitude_noise_config_uses_density_simulator_and_trains():
    """noise.kind=amplitude selects the exact density-matrix simulator (parameter-shift gradients) and a short
    federated run trains; the twirl keeps the statevector trajectories."""
    from qfedx_amd.api import run_experiment
    from qfedx_amd.fl.adapters import make_adapter
    from tests.test_fl import small_cfg
    cfg = small_cfg(num_rounds=2, kind="vqc", n_qubits=3, n_layers=1, num_clients=2, samples_per_client=24,
                    batch_size=12, grad_method="param_shift", optimizer="sgd")
    cfg.noise.kind, cfg.noise.gamma = "amplitude", 0.05
    ad = make_adapter(cfg, torch.device("cpu"), "torch")
    assert ad.simulator == "density" and ad.engine.backend == "density" and not ad.spec.noisy
    out = run_experiment(cfg)
    assert len(out["accuracies"]) == 3 and all(np.isfinite(out["accuracies"]))
    cfg.noise.kind = "amplitude_twirl"
    ad2 = make_adapter(cfg, torch.device("cpu"), "torch")
    assert ad2.simulator == "statevector" and ad2.spec.noisy
