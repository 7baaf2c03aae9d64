"""VQCLayer on the HIP engine: forward and autograd gradients (weights + inputs) match the CPU layer."""
import pytest
import torch

from qfedx_amd.models.qlayer import VQCLayer

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("n,L,fm", [(4, 2, "ry"), (12, 2, "rx"), (16, 3, "ry"), (10, 2, "amplitude")])
def test_vqc_layer_hip_matches_cpu(cuda, n, L, fm):
    torch.manual_seed(n)
    cpu = VQCLayer(n, L, readout=[0, 1, n - 1], feature_map=fm, init_std=1.0)
    gpu = VQCLayer(n, L, readout=[0, 1, n - 1], feature_map=fm, init_std=1.0).to(cuda)
    gpu.load_state_dict(cpu.state_dict())
    F = cpu.n_features
    x = torch.rand(6, F, requires_grad=True)
    xg = x.detach().to(cuda).requires_grad_(True)
    w = torch.randn(6, 3)
    (cpu(x) * w).sum().backward()
    zg = gpu(xg)
    (zg * w.to(cuda)).sum().backward()
    assert torch.allclose(zg.detach().cpu(), cpu(x).detach(), atol=3e-5)
    assert torch.allclose(gpu.theta.grad.cpu(), cpu.theta.grad, atol=3e-4)
    if fm != "amplitude":
        assert torch.allclose(xg.grad.cpu(), x.grad, atol=3e-4)
