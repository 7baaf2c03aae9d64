"""Hybrid quantum layer (models/qlayer.py): autograd gradients (weights and inputs) vs finite differences,
and a classical->quantum->classical model that trains."""
import pytest
import torch
from torch import nn

from qfedx_amd.models.qlayer import VQCLayer


@pytest.mark.parametrize("fm,ent", [("ry", "chain"), ("rx", "ring")])
def test_vqc_layer_grads_match_finite_differences(fm, ent):
    torch.manual_seed(0)
    layer = VQCLayer(4, 2, readout=[0, 2, 3], feature_map=fm, entangler=ent, init_std=1.0).double()
    x = torch.rand(5, 4, dtype=torch.float64, requires_grad=True)
    w = torch.randn(5, 3, dtype=torch.float64)
    (layer(x) * w).sum().backward()
    gx, gt = x.grad.clone(), layer.theta.grad.clone()
    eps = 1e-3

    def f():
        with torch.no_grad():
            return float((layer(x) * w).sum())
    for j in range(0, layer.theta.numel(), 3):
        with torch.no_grad():
            layer.theta[j] += eps
        fp = f()
        with torch.no_grad():
            layer.theta[j] -= 2 * eps
        fm_ = f()
        with torch.no_grad():
            layer.theta[j] += eps
        assert abs((fp - fm_) / (2 * eps) - float(gt[j])) < 2e-3
    for i, q in [(0, 0), (3, 2), (4, 3)]:
        with torch.no_grad():
            x[i, q] += eps
        fp = f()
        with torch.no_grad():
            x[i, q] -= 2 * eps
        fm_ = f()
        with torch.no_grad():
            x[i, q] += eps
        assert abs((fp - fm_) / (2 * eps) - float(gx[i, q])) < 2e-3


def test_hybrid_model_trains():
    torch.manual_seed(1)
    X = torch.randn(64, 6)
    y = (X[:, 0] + 0.5 * X[:, 1] > 0).long()
    model = nn.Sequential(nn.Linear(6, 3), nn.Tanh(), VQCLayer(3, 2, readout=[0, 1], init_std=0.5),
                          nn.Linear(2, 2))
    opt = torch.optim.Adam(model.parameters(), lr=0.05)
    losses = []
    for _ in range(60):
        opt.zero_grad()
        loss = nn.functional.cross_entropy(model(X), y)
        loss.backward()
        opt.step()
        losses.append(float(loss.detach()))
    assert losses[-1] < 0.6 * losses[0]
    assert model[0].weight.grad is not None and model[0].weight.grad.abs().sum() > 0   # flows into Linear


def test_amplitude_layer_forward():
    from qfedx_amd.quantum.statevector import Statevector
    import numpy as np
    layer = VQCLayer(3, 1, readout=[0, 1], feature_map="amplitude", init_std=1.0)
    x = torch.rand(2, 8)
    z = layer(x)
    z.sum().backward()
    assert layer.theta.grad is not None
    spec = layer.spec
    for s in range(2):
        st = spec.initial_states(x[s:s + 1])[0].numpy().astype(complex)
        ref = Statevector(st).evolve(spec.circuit(), {"theta": layer.theta.detach().double().numpy(),
                                                      "x": np.zeros(3)})
        assert np.allclose(z[s].detach().numpy(), [ref.expectation_z(0), ref.expectation_z(1)], atol=1e-5)
