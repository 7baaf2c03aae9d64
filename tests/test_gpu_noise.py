"""GPU numerics of the noise model + batched parameter shift: HIP kernels vs the torch path."""
import pytest
import torch

from qfedx_amd.models.vqc import VQCSpec
from qfedx_amd.ops.engine import VQCEngine
from qfedx_amd.quantum.noise import NoiseModel, pauli_probs
from qfedx_amd.utils.seeding import philox_key, philox_uniform_rows

pytestmark = pytest.mark.gpu


def _keys(K, purpose, dev=None):
    k = torch.tensor([philox_key(11, purpose, 2, c) for c in range(K)], dtype=torch.int64)
    return k if dev is None else k.to(dev)


def test_philox_uniform_kernel_bitwise(cuda):
    from qfedx_amd.ops._ext import ext
    k = _keys(5, "noise_traj")
    out = torch.empty(5, 1001, device=cuda)
    ext().philox_uniform(k.to(cuda), 1001, 7, out)
    assert torch.equal(out.cpu(), philox_uniform_rows(k, 1001, 7))


def _noisy_setup(n, L, K, B, kind="depolarizing", p=0.2, gamma=0.2, readout=(0.0, 0.0), shots=0, seed=0):
    kind = "amplitude_twirl" if kind == "amplitude" else kind
    px, py, pz = pauli_probs(kind, p, gamma)
    nm = NoiseModel(px, py, pz, readout[0], readout[1], shots)
    spec = VQCSpec(n, L, 3, readout_scale=2.0, init_std=1.0, noisy=nm.gate_noise)
    g = torch.Generator().manual_seed(seed)
    x = torch.rand(K, B, n, generator=g) * 3
    y = torch.randint(0, 3, (K, B), generator=g)
    w = torch.full((K, B), 1.0 / B)
    params = torch.stack([spec.init_params(seed + k) for k in range(K)])
    return nm, spec, x, y, w, params


@pytest.mark.parametrize("n,L,jit", [(4, 2, "1"), (7, 2, "1"), (12, 2, "1"), (7, 2, "0")])
def test_pauli_trajectories_forward_and_adjoint_match_torch(cuda, n, L, jit, monkeypatch):
    monkeypatch.setenv("QFEDX_JIT", jit)
    nm, spec, x, y, w, params = _noisy_setup(n, L, 3, 4)
    hip = VQCEngine(spec, cuda, "hip", noise=nm)
    ref = VQCEngine(spec, "cpu", "torch", noise=nm)
    keys = _keys(3, "noise_traj")
    xa_c = ref.augment(x, keys, 1)
    xa_g = hip.augment(x.to(cuda), keys.to(cuda), 1)
    assert torch.equal(xa_g.cpu(), xa_c)
    th = spec.split(params)[0]
    assert torch.allclose(hip.expz(xa_g, th.to(cuda)).cpu(), ref.expz(xa_c, th), atol=2e-5)
    rg = hip.loss_and_grads(xa_g, y.to(cuda), w.to(cuda), params.to(cuda), "adjoint")
    rc = ref.loss_and_grads(xa_c, y, w, params, "adjoint")
    assert torch.allclose(rg["loss"].cpu(), rc["loss"], atol=2e-5)
    assert torch.allclose(rg["grad"].cpu(), rc["grad"], atol=5e-5)


def test_noisy_readout_and_shots_match_torch(cuda):
    nm, spec, x, y, w, params = _noisy_setup(6, 2, 3, 8, kind="none", readout=(0.05, 0.1), shots=96)
    hip = VQCEngine(spec, cuda, "hip", noise=nm)
    ref = VQCEngine(spec, "cpu", "torch", noise=nm)
    keys = _keys(3, "shots")
    th = spec.split(params)[0]
    zg = hip.expz(x.to(cuda), th.to(cuda), keys.to(cuda), 3).cpu()
    zc = ref.expz(x, th, keys, 3)
    # identical keyed uniforms -> identical shot counts (up to fp ties at p1 exactly): k/S grid equal
    assert (zg - zc).abs().max() <= 2.0 / 96 + 1e-6 and (zg == zc).float().mean() > 0.98
    rg = hip.loss_and_grads(x.to(cuda), y.to(cuda), w.to(cuda), params.to(cuda), "adjoint", readout_keys=keys.to(cuda), step=3)
    rc = ref.loss_and_grads(x, y, w, params, "adjoint", readout_keys=keys, step=3)
    assert torch.allclose(rg["expz"].cpu(), rc["expz"], atol=2.0 / 96 + 1e-6)
    assert torch.allclose(rg["grad"].cpu(), rc["grad"], atol=0.05)


@pytest.mark.parametrize("n", [5, 13])
def test_batched_param_shift_hip_matches_adjoint(cuda, n):
    spec = VQCSpec(n, 2, 3, readout_scale=2.0, init_std=1.0)
    eng = VQCEngine(spec, cuda, "hip")
    g = torch.Generator().manual_seed(1)
    K, B = 2, 3
    x = (torch.rand(K, B, n, generator=g) * 3).to(cuda)
    y = torch.randint(0, 3, (K, B), generator=g).to(cuda)
    w = torch.full((K, B), 1.0 / B, device=cuda)
    params = torch.stack([spec.init_params(k) for k in range(K)]).to(cuda)
    adj = eng.loss_and_grads(x, y, w, params, "adjoint")["grad"]
    eng._budget = (1 << n) * 8 * B * 5       # several chunks
    ps = eng.loss_and_grads(x, y, w, params, "param_shift")["grad"]
    assert torch.allclose(adj, ps, atol=3e-5)


@pytest.mark.parametrize("n,kind,p,gamma", [(4, "amplitude", 0.0, 0.2), (6, "amplitude", 0.0, 0.1),
                                            (7, "depolarizing", 0.05, 0.0), (8, "amplitude", 0.0, 0.05)])
def test_density_kernel_matches_float64_kraus_oracle(cuda, n, kind, p, gamma):
    """csrc/density.hip (rho in LDS up to 6 qubits, in a global slab beyond) == the float64 density-matrix oracle
    with the exact Kraus channel after every gate (ROADMAP.md:66-73 amplitude damping)."""
    import numpy as np
    from qfedx_amd.ops.density import DensityProgram, kraus_ops
    from qfedx_amd.quantum.noise import density_expz
    spec = VQCSpec(n, 2, 3, init_std=1.0)
    ops, coef = spec.program()
    kr = kraus_ops(kind, p, gamma)
    g = torch.Generator().manual_seed(n)
    S = 3
    rows = torch.cat([torch.randn(S, spec.n_theta, generator=g), torch.rand(S, n, generator=g) * 3], -1)
    z = DensityProgram(ops, coef, n, spec.readout, cuda, kraus=kr).expz(rows.to(cuda)).cpu()
    for s in range(S):
        ref = density_expz(ops, coef, n, rows[s].double().numpy(), spec.readout, (0, 0, 0), kraus=kr)
        assert np.allclose(z[s].numpy(), ref, atol=3e-5), (n, z[s], ref)


def test_density_engine_param_shift_on_gpu_matches_cpu(cuda):
    """Exact amplitude-damping VQC step on the HIP density kernel == the torch density path (parameter shift)."""
    from qfedx_amd.quantum.noise import NoiseModel
    nm = NoiseModel(kind="amplitude", gamma=0.1)
    spec = VQCSpec(4, 2, 3, readout_scale=2.0, init_std=1.0)
    g = torch.Generator().manual_seed(1)
    x = spec.encode_features(torch.rand(2, 5, 4, generator=g))
    y = torch.randint(0, 3, (2, 5), generator=g)
    w = torch.full((2, 5), 0.2)
    params = torch.stack([spec.init_params(k) for k in range(2)])
    rg = VQCEngine(spec, cuda, "density", noise=nm).loss_and_grads(x.to(cuda), y.to(cuda), w.to(cuda),
                                                                     params.to(cuda), "param_shift")
    rc = VQCEngine(spec, "cpu", "density", noise=nm).loss_and_grads(x, y, w, params, "param_shift")
    assert torch.allclose(rg["loss"].cpu(), rc["loss"], atol=2e-5)
    assert torch.allclose(rg["grad"].cpu(), rc["grad"], atol=5e-5)
