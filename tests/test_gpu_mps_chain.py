"""HIP column contraction of the CNOT-chain VQC (csrc/mps_chain.hip) against its float64 oracle
(quantum/mps_chain.py, itself checked against the dense statevector on the CPU) and against the generic torch MPS
backend at 48 qubits; the engine routes training steps through it."""
import numpy as np
import pytest
import torch

from qfedx_amd.models.vqc import VQCSpec
from qfedx_amd.quantum.mps_chain import chain_columns

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def cuda():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch.device("cuda", 0)


@pytest.mark.parametrize("n,L,C,feat,ro", [(6, 3, 3, "ry", None), (5, 1, 2, "rx", None), (7, 2, 4, "rz", [1, 3, 4, 6]),
                                           (9, 3, 3, "ry", [8, 0, 4])])
def test_kernel_matches_oracle(cuda, n, L, C, feat, ro):
    from qfedx_amd.ops.mps_hip import MpsChainProgram
    spec = VQCSpec(n, L, C, feature_map=feat, readout=ro)
    g = np.random.default_rng(n + L)
    K, B = 3, 4
    x = g.uniform(0, 3, (K, B, n))
    th = g.normal(size=(K, spec.n_theta))
    w = g.normal(size=(K, B, C))
    prog = MpsChainProgram(spec, cuda)
    z = prog.expz(torch.from_numpy(x).float().to(cuda), torch.from_numpy(th).float().to(cuda))
    gr = prog.grads(torch.from_numpy(x).float().to(cuda), torch.from_numpy(th).float().to(cuda),
                    torch.from_numpy(w).float().to(cuda))
    torch.cuda.synchronize()
    zo, go = chain_columns(x.reshape(K * B, n), np.repeat(th, B, 0), n, L, spec.readout, feat, w.reshape(K * B, C))
    np.testing.assert_allclose(z.cpu().numpy().reshape(K * B, C), zo, atol=2e-5)
    np.testing.assert_allclose(gr.cpu().numpy(), go.reshape(K, B, -1).sum(1), atol=1e-4)


def test_48_qubits_match_torch_mps_and_train(cuda):
    """The BASELINE MPS shape (48 qubits, 3 layers): the kernel's <Z> and gradients match the float64 oracle, and the
    engine's loss / gradients on the HIP kernel equal the generic torch MPS backend (reverse-mode AD through its
    complex64 einsum network) to fp32 accumulation over 48 sites."""
    from qfedx_amd.ops.engine import VQCEngine
    spec = VQCSpec(48, 3, 3, readout_scale=3.0)
    g = torch.Generator().manual_seed(3)
    K, B = 2, 4
    xang = spec.encode_features(torch.rand(K, B, 48, generator=g)).to(cuda)
    params = torch.stack([spec.init_params(k) for k in range(K)])
    params = (params + 0.2 * torch.randn(params.shape, generator=g)).to(cuda)
    y = torch.randint(0, 3, (K, B), generator=g).to(cuda)
    wm = torch.full((K, B), 1.0 / B, device=cuda)
    eng = VQCEngine(spec, cuda, "mps")
    assert eng.mps_hip is not None
    fast = eng.loss_and_grads(xang, y, wm, params)
    ez = eng.expz(xang, spec.split(params)[0])
    eng.mps_hip = None                                  # generic torch einsum network
    ref = eng.loss_and_grads(xang, y, wm, params)
    ez_ref = eng.expz(xang, spec.split(params)[0])
    torch.cuda.synchronize()
    np.testing.assert_allclose(ez.cpu().numpy(), ez_ref.cpu().numpy(), atol=1e-4)
    np.testing.assert_allclose(fast["loss"].cpu().numpy(), ref["loss"].cpu().numpy(), rtol=1e-4, atol=1e-5)
    np.testing.assert_allclose(fast["grad"].cpu().numpy(), ref["grad"].cpu().numpy(), atol=1e-4)
    assert torch.equal(fast["correct"], ref["correct"])
    # two samples against the float64 oracle (the kernel's own error, not the difference of two fp32 paths)
    th = spec.split(params)[0]
    w = torch.randn(1, 2, 3, generator=g).to(cuda)
    from qfedx_amd.ops.mps_hip import MpsChainProgram
    kp = MpsChainProgram(spec, cuda)
    z1 = kp.expz(xang[:1, :2].contiguous(), th[:1].contiguous())
    g1 = kp.grads(xang[:1, :2].contiguous(), th[:1].contiguous(), w)
    zo, go = chain_columns(xang[0, :2].double().cpu().numpy(), th[:1].double().cpu().numpy().repeat(2, 0), 48, 3,
                           spec.readout, "ry", w[0].double().cpu().numpy())
    np.testing.assert_allclose(z1[0].cpu().numpy(), zo, atol=2e-5)
    np.testing.assert_allclose(g1[0].cpu().numpy(), go.sum(0), atol=5e-5)


def test_fused_readout_train_matches_two_launch_step(cuda):
    """The one-launch training step (readout cross entropy and dL/d<Z> in the kernel) against the <Z> launch + torch
    readout + gradient launch: same loss, gradients (readout a / b included), hits and <Z>, at fp32 rounding."""
    from qfedx_amd.ops.engine import VQCEngine
    spec = VQCSpec(24, 3, 3, readout_scale=3.0)
    g = torch.Generator().manual_seed(5)
    K, B = 3, 8
    xang = spec.encode_features(torch.rand(K, B, 24, generator=g)).to(cuda)
    params = (torch.stack([spec.init_params(k) for k in range(K)]) + 0.2 * torch.randn(K, spec.n_params,
                                                                                      generator=g)).to(cuda)
    y = torch.randint(0, 3, (K, B), generator=g).to(cuda)
    wm = torch.rand(K, B, generator=g).to(cuda)
    eng = VQCEngine(spec, cuda, "mps")
    assert eng.mps_hip is not None and eng.fused_mps_readout
    calls = [0]
    real = eng.mps_hip.train

    def spy(*a, **k):
        calls[0] += 1
        return real(*a, **k)
    eng.mps_hip.train = spy
    fused = eng.loss_and_grads(xang, y, wm, params)
    eng.fused_mps_readout = False
    ref = eng.loss_and_grads(xang, y, wm, params)
    torch.cuda.synchronize()
    assert calls[0] == 1
    np.testing.assert_allclose(fused["loss"].cpu().numpy(), ref["loss"].cpu().numpy(), rtol=1e-5, atol=1e-6)
    np.testing.assert_allclose(fused["grad"].cpu().numpy(), ref["grad"].cpu().numpy(), atol=1e-5)
    np.testing.assert_allclose(fused["expz"].cpu().numpy(), ref["expz"].cpu().numpy(), atol=1e-6)
    assert torch.equal(fused["correct"].cpu(), ref["correct"].cpu())
