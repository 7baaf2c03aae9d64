"""Amplitude-encoded VQC on the HIP engine (load-from-state forward plan + adjoint) vs the torch executor,
and federated rounds (hipGraph and eager) vs the CPU run."""
import pytest
import torch

from qfedx_amd.ops.engine import VQCEngine
from tests.test_amplitude import _amp_setup

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("n,L,K,B,ent", [(3, 1, 3, 5, "chain"), (5, 2, 2, 7, "ring"), (10, 2, 3, 3, "chain"),
                                         (13, 2, 2, 2, "ring"), (16, 2, 2, 2, "chain")])
@pytest.mark.parametrize("jit", ["1", "0"])
def test_amplitude_hip_matches_torch(cuda, n, L, K, B, ent, jit, monkeypatch):
    monkeypatch.setenv("QFEDX_JIT", jit)
    spec, x, y, w, params = _amp_setup(n, L, 3, K, B, seed=n, ent=ent)
    ref = VQCEngine(spec, "cpu", "torch").loss_and_grads(spec.encode_features(x), y, w, params, "adjoint",
                                                         init=spec.initial_states(x))
    hip = VQCEngine(spec, cuda, "hip")
    xc = x.to(cuda)
    out = hip.loss_and_grads(spec.encode_features(xc), y.to(cuda), w.to(cuda), params.to(cuda), "adjoint",
                             init=spec.initial_states(xc))
    assert torch.allclose(out["loss"].cpu(), ref["loss"], atol=2e-5)
    assert torch.allclose(out["expz"].cpu(), ref["expz"], atol=2e-5)
    assert torch.allclose(out["grad"].cpu(), ref["grad"], atol=3e-4), (out["grad"].cpu() - ref["grad"]).abs().max()
    z = hip.expz(spec.encode_features(xc), spec.split(params.to(cuda))[0], init=spec.initial_states(xc))
    assert torch.allclose(z.cpu(), ref["expz"], atol=2e-5)


def test_amplitude_federated_hip_matches_cpu(cuda):
    from tests.test_fl import small_cfg
    from qfedx_amd.api import run_experiment
    from qfedx_amd.parallel.dist import init_distributed
    kw = dict(num_rounds=2, optimizer="sgd", feature_map="amplitude", n_qubits=5)
    cpu = run_experiment(small_cfg(**kw))
    dev = torch.device("cuda", 0)
    outs = []
    import qfedx_amd.fl.trainer as tr
    old = tr.VQCClientTrainer.use_graph
    for graphs in (True, False):
        tr.VQCClientTrainer.use_graph = property(lambda self, g=graphs: g)
        try:
            outs.append(run_experiment(small_cfg(device="cuda", backend="hip", **kw),
                                       world=init_distributed(dev), device=dev, backend="hip"))
        finally:
            tr.VQCClientTrainer.use_graph = old
    assert torch.equal(outs[0]["params"], outs[1]["params"])
    assert torch.allclose(outs[0]["params"].cpu(), cpu["params"], atol=1e-4)


@pytest.mark.parametrize("n,F", [(4, 16), (4, 11), (13, 8192), (14, 5000), (20, 1 << 20)])
def test_amp_init_kernel_matches_torch(cuda, n, F):
    """K9: device amplitude encoding (float64 norm, zero-pad, zero row -> uniform) == torch reference,
    written straight into complex64 and packed-bf16 pass storage."""
    from qfedx_amd.ops._ext import ext
    from qfedx_amd.quantum.encoders import amplitude_states
    S = 3
    g = torch.Generator().manual_seed(n)
    x = torch.randn(S, F, generator=g)
    x[1] = 0.0                                                  # zero row -> uniform state
    N = 1 << n
    ref = amplitude_states(torch.cat([x, x.new_zeros(S, N - F)], 1))
    xc = x.to(cuda)
    part = torch.empty(S * ext().amp_scratch(F), dtype=torch.float64, device=cuda)
    psi = torch.empty(S * N, dtype=torch.complex64, device=cuda)
    ext().amp_init(xc, n, part, psi)
    assert torch.allclose(psi.view(S, N).cpu(), ref, atol=1e-7, rtol=1e-6)
    packed = torch.empty(S * N, dtype=torch.int32, device=cuda)
    ext().amp_init(xc, n, part, packed)
    re = (packed.view(S, N) << 16).view(torch.float32).cpu()
    assert torch.allclose(re, ref.real, atol=1e-6, rtol=1e-2)
    assert torch.equal(re, ref.real.to(torch.bfloat16).float())   # RNE rounding like torch


def test_amplitude_raw_features_bf16_storage(cuda):
    spec, x, y, w, params = _amp_setup(12, 2, 3, 2, 4, seed=7)
    xc = x.to(cuda)
    f32 = VQCEngine(spec, cuda, "hip", "fp32").expz(spec.encode_features(xc), spec.split(params.to(cuda))[0],
                                                     init=xc)
    b16 = VQCEngine(spec, cuda, "hip", "bf16").expz(spec.encode_features(xc), spec.split(params.to(cuda))[0],
                                                     init=xc)
    ref = VQCEngine(spec, "cpu", "torch").expz(spec.encode_features(x), spec.split(params)[0], init=x)
    assert torch.allclose(f32.cpu(), ref, atol=2e-5)
    assert (b16.cpu() - ref).abs().max() < 2e-2
