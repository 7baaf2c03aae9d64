"""MPS backend on the GPU (batched contractions on hipBLASLt/rocBLAS, QR/SVD on rocSOLVER) vs the float64
CPU MPS: a 32-qubit 3-layer VQC training step (exact at bond 8) and a truncating random circuit."""
import numpy as np
import pytest
import torch

from qfedx_amd.models.vqc import VQCSpec
from qfedx_amd.ops.engine import VQCEngine
from qfedx_amd.quantum.mps import MPSProgram

pytestmark = pytest.mark.gpu


def test_mps_vqc_32q_step_matches_cpu_float64(cuda):
    spec = VQCSpec(32, 3, 3, readout_scale=2.0)
    K, B = 2, 8
    g = torch.Generator().manual_seed(0)
    x = spec.encode_features(torch.rand(K, B, 32, generator=g))
    y = torch.randint(0, 3, (K, B), generator=g)
    w = torch.full((K, B), 1.0 / B)
    params = torch.stack([spec.init_params(k) for k in range(K)]) + 0.2 * torch.randn(K, spec.n_params, generator=g)
    cpu = VQCEngine(spec, "cpu", "mps")
    cpu.prog = MPSProgram(cpu.ops, cpu.coef, 32, "cpu", dtype=torch.complex128)
    ref = cpu.loss_and_grads(x.double(), y, w.double(), params.double())
    gpu = VQCEngine(spec, cuda, "mps")
    out = gpu.loss_and_grads(x.to(cuda), y.to(cuda), w.to(cuda), params.to(cuda))
    torch.cuda.synchronize()
    np.testing.assert_allclose(out["loss"].cpu().numpy(), ref["loss"].numpy(), atol=1e-4)
    np.testing.assert_allclose(out["grad"].cpu().numpy(), ref["grad"].numpy(), atol=1e-3)


def test_mps_truncating_circuit_on_gpu(cuda):
    """Truncated (bond 16) GPU readouts stay within the bound their own discarded weight implies, against the
    exact float64 state (fp32 and fp64 SVDs may keep different near-degenerate vectors, so the two
    truncations are not compared with each other)."""
    from tests.test_mps import _random_circuit
    circ, k = _random_circuit(14, 3, 4)
    ops, coef = circ.to_program({"v": 0})
    rows = torch.randn(4, k, generator=torch.Generator().manual_seed(1), dtype=torch.float64)
    exact = MPSProgram(ops, coef, 14, "cpu", dtype=torch.complex128, chi_max=128)
    dev = MPSProgram(ops, coef, 14, cuda, chi_max=16)
    z_ref = exact.expz(exact.run(rows), [0, 7, 13])
    st = dev.run(rows.to(cuda))
    z = dev.expz(st, [0, 7, 13]).cpu().double()
    assert max(st.bonds()) <= 16 and st.n_trunc > 0
    bound = st.error_bound().cpu()[:, None] + 2e-3
    assert float(bound.max()) < 1.0                       # a non-vacuous truncation regime
    assert torch.all((z - z_ref).abs() <= bound), ((z - z_ref).abs(), bound)
