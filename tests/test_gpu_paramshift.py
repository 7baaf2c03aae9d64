"""Parameter shift with prefix reuse on the MFMA engine (``HeaMfmaProgram.shifted_expz`` / ``param_shift``) vs
the float64 dense oracle: the shifted expectations f(theta +- pi/2) themselves, the exact-expectation gradient
vs the adjoint, the shot-sampled estimator vs the naive shifted-row path, and chunking invariance."""
import numpy as np
import pytest
import torch

from qfedx_amd.models.vqc import VQCSpec
from qfedx_amd.ops.engine import VQCEngine
from qfedx_amd.ops.hea_mfma import HeaMfmaProgram
from qfedx_amd.ops.statevec_torch import TorchProgram
from qfedx_amd.quantum.noise import NoiseModel

from tests.test_gpu_hea import _dense, _inputs

pytestmark = pytest.mark.gpu


def _dense_shifted(spec, x, params, dev):
    """f(theta +- pi/2 e_j) [K, P, 2, B, C] in complex128 on the GPU."""
    ops, coef = spec.program()
    prog = TorchProgram(ops, coef, spec.n_qubits, dev, dtype=torch.complex128)
    K, B, _ = x.shape
    P = spec.n_theta
    th = params[:, :P].double().to(dev)
    sh = th[:, None, None, :].repeat(1, P, 2, 1)                  # [K, P, 2, P]
    idx = torch.arange(P, device=dev)
    sh[:, idx, 0, idx] += np.pi / 2
    sh[:, idx, 1, idx] -= np.pi / 2
    rows = torch.cat([sh[:, :, :, None, :].expand(K, P, 2, B, P),
                      x.double().to(dev)[:, None, None].expand(K, P, 2, B, x.shape[-1])], -1).reshape(-1, P + x.shape[-1])
    out = []
    for r0 in range(0, rows.shape[0], 256):
        psi = prog.run(rows[r0:r0 + 256])
        out.append(prog.expz(psi, spec.readout))
    return torch.cat(out).reshape(K, P, 2, B, -1)


@pytest.mark.parametrize("n,L,tile", [(12, 3, 14), (14, 3, 10), (16, 3, 14)])
def test_shifted_expz_matches_dense(cuda, n, L, tile):
    """m +- f' (pi identity, +pi branches from the stored prefix of their pass) = f(theta +- pi/2) exactly."""
    spec = VQCSpec(n, L, 3)
    prog = HeaMfmaProgram(spec, cuda, tile_bits=tile)
    K, B = 2, 2
    x, params, _ = _inputs(spec, K, B, seed=5)
    zz = prog.shifted_expz(x.to(cuda), params[:, :spec.n_theta].to(cuda))
    ref = _dense_shifted(spec, x, params, cuda)
    torch.cuda.synchronize()
    np.testing.assert_allclose(zz.cpu().numpy(), ref.cpu().numpy(), atol=4e-3)


@pytest.mark.parametrize("n,L,tile", [(12, 3, 14), (16, 3, 14)])
def test_param_shift_exact_matches_adjoint_oracle(cuda, n, L, tile):
    spec = VQCSpec(n, L, 3)
    prog = HeaMfmaProgram(spec, cuda, tile_bits=tile)
    K, B = 2, 3
    x, params, wr = _inputs(spec, K, B, seed=1)
    _, g_ref = _dense(spec, x.double(), params.double(), wr.double())
    g = prog.param_shift(x.to(cuda), params[:, :spec.n_theta].to(cuda), wr.to(cuda), exact_only=True)
    torch.cuda.synchronize()
    scale = max(1.0, float(g_ref.abs().max()))
    np.testing.assert_allclose(g.cpu().numpy(), g_ref.numpy(), atol=4e-3 * scale)


def test_param_shift_chunking_is_bitwise(cuda, monkeypatch):
    """A 1 MiB budget splits the work into one client per chunk and two parameter rows per +pi chunk."""
    spec = VQCSpec(14, 3, 2)
    x, params, _ = _inputs(spec, 3, 2, seed=2)
    big = HeaMfmaProgram(spec, cuda, tile_bits=10).shifted_expz(x.to(cuda), params[:, :spec.n_theta].to(cuda))
    monkeypatch.setenv("QFEDX_PS_BUDGET_MB", "1")
    small = HeaMfmaProgram(spec, cuda, tile_bits=10).shifted_expz(x.to(cuda), params[:, :spec.n_theta].to(cuda))
    torch.cuda.synchronize()
    assert torch.equal(big, small)


def test_param_shift_shots_matches_naive_rows(cuda, monkeypatch):
    """Shot-sampled estimator: the reuse path samples the same Philox streams per (client, slot, sign) row as
    the naive shifted-row path; only shots whose uniform falls within the fp16 rounding of p differ."""
    spec = VQCSpec(12, 3, 2, readout_scale=2.0)
    K, B, shots = 3, 4, 256
    g = torch.Generator().manual_seed(7)
    x = spec.encode_features(torch.rand(K, B, 12, generator=g)).to(cuda)
    y = torch.randint(0, 2, (K, B), generator=g).to(cuda)
    wm = torch.full((K, B), 1.0 / B, device=cuda)
    params = torch.stack([spec.init_params(k) for k in range(K)]).to(cuda)
    keys = torch.randint(0, 2 ** 31, (K, 2), generator=g).long().to(cuda)
    nz = NoiseModel(shots=shots)
    eng = VQCEngine(spec, cuda, "hip", "mfma", noise=nz)
    eng.ps_reuse = True
    a = eng.loss_and_grads(x, y, wm, params, "param_shift", readout_keys=keys, step=3)
    eng.ps_reuse = False
    b = eng.loss_and_grads(x, y, wm, params, "param_shift", readout_keys=keys, step=3)
    torch.cuda.synchronize()
    ga, gb = a["grad"].cpu(), b["grad"].cpu()
    assert torch.equal(a["loss"].cpu(), b["loss"].cpu())
    d = (ga - gb).abs()
    wmax = float(a["grad"].new_tensor(1.0))
    # a flipped shot moves one estimate by 2 / shots, weighted by |w| <= readout_scale / B per sample
    assert float(d.max()) <= 4 * (2.0 / shots) * 2.0 * wmax
    assert float((d > 1e-6).float().mean()) < 0.5
