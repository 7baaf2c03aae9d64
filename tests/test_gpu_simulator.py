"""GPU numerics of the public simulator on random generic circuits: HIP kernels vs the torch executor."""
import numpy as np
import pytest
import torch

from qfedx_amd.quantum.simulator import Simulator
from tests.test_simulator import _random_circuit

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("n,seed,jit", [(5, 0, "1"), (9, 1, "1"), (13, 2, "1"), (9, 3, "0")])
def test_random_circuits_hip_vs_torch(cuda, n, seed, jit, monkeypatch):
    monkeypatch.setenv("QFEDX_JIT", jit)
    qc = _random_circuit(n, 8, seed, gates=70)
    rng = np.random.default_rng(seed)
    vals = torch.tensor(rng.normal(size=(5, 8)), dtype=torch.float32)
    w = torch.tensor(rng.normal(size=(5, 2)), dtype=torch.float32)
    hip = Simulator(qc, readout=[0, n - 1], device=cuda)
    ref = Simulator(qc, readout=[0, n - 1], device="cpu")
    psi_g, z_g = hip.run(vals.to(cuda))
    psi_c, z_c = ref.run(vals)
    assert (psi_g.cpu() - psi_c).abs().max().item() < 2e-5
    assert torch.allclose(z_g.cpu(), z_c, atol=2e-5)
    zg, gg = hip.vjp(vals.to(cuda), w.to(cuda))
    zc, gc = ref.vjp(vals, w)
    assert torch.allclose(gg.cpu(), gc, atol=5e-5)


def test_initial_state_load_hip(cuda):
    from qfedx_amd.quantum.encoders import amplitude_states
    n = 10
    qc = _random_circuit(n, 6, 11, gates=50)
    x = torch.rand(4, 1 << n)
    init = amplitude_states(x)
    vals = torch.randn(4, 6)
    hip = Simulator(qc, readout=[0, 5], device=cuda)
    ref = Simulator(qc, readout=[0, 5], device="cpu")
    psi_g, z_g = hip.run(vals.to(cuda), initial_state=init.to(cuda))
    psi_c, z_c = ref.run(vals, initial_state=init)
    assert (psi_g.cpu() - psi_c).abs().max().item() < 2e-5
    zg, gg = hip.vjp(vals.to(cuda), torch.ones(4, 2, device=cuda), initial_state=init.to(cuda))
    zc, gc = ref.vjp(vals, torch.ones(4, 2), initial_state=init)
    assert torch.allclose(gg.cpu(), gc, atol=5e-5)
