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


def _ring_step(engine, spec, K, B, seed=3):
    g = torch.Generator().manual_seed(seed)
    x = spec.encode_features(torch.rand(K, B, spec.n_qubits, generator=g))
    y = torch.randint(0, spec.n_classes, (K, B), generator=g)
    w = torch.full((K, B), 1.0 / B)
    params = torch.stack([spec.init_params(k) for k in range(K)]) + 0.2 * torch.randn(K, spec.n_params, generator=g)
    d = engine.device
    return engine.loss_and_grads(x.to(d), y.to(d), w.to(d), params.to(d))


def test_mps_mpo_kernel_32q_ring_step_matches_einsum_network(cuda):
    """A non-chain circuit (ring entangler: chain + wrap-around CX per layer, bond 16 at 2 layers) on the generic HIP
    kernel (csrc/mps_mpo.hip) vs the torch einsum network on the same GPU, and vs the float64 CPU MPS."""
    spec = VQCSpec(32, 2, 3, readout_scale=2.0, entangler="ring")
    K, B = 2, 8
    eng = VQCEngine(spec, cuda, "mps")
    hip = eng.prog.hip_program()
    assert hip is not None and eng.mps_hip is None
    out = _ring_step(eng, spec, K, B)
    ref_eng = VQCEngine(spec, cuda, "mps")
    ref_eng.prog._hip = None                              # the einsum network
    ref = _ring_step(ref_eng, spec, K, B)
    torch.cuda.synchronize()
    assert hip.launches == 2                               # <Z> launch + gradient launch
    np.testing.assert_allclose(out["loss"].cpu().numpy(), ref["loss"].cpu().numpy(), atol=1e-4)
    np.testing.assert_allclose(out["grad"].cpu().numpy(), ref["grad"].cpu().numpy(), atol=1e-4)
    cpu = VQCEngine(spec, "cpu", "mps")
    cpu.prog = MPSProgram(cpu.ops, cpu.coef, 32, "cpu", dtype=torch.complex128)
    g = torch.Generator().manual_seed(3)
    x = spec.encode_features(torch.rand(K, B, 32, generator=g))
    y = torch.randint(0, 3, (K, B), generator=g)
    params = torch.stack([spec.init_params(k) for k in range(K)]) + 0.2 * torch.randn(K, spec.n_params, generator=g)
    r64 = cpu.loss_and_grads(x.double(), y, torch.full((K, B), 1.0 / B).double(), params.double())
    np.testing.assert_allclose(out["grad"].cpu().numpy(), r64["grad"].numpy(), atol=1e-4)


def test_mps_mpo_kernel_random_circuits_match_dense(cuda):
    """Long-range CX / CZ in both directions and every 1-qubit kind: <Z> and the adjoint VJP of the HIP kernel
    (through ``Simulator(backend="mps")``) against the float64 dense statevector."""
    from qfedx_amd.quantum.simulator import Simulator
    from tests.test_mps_mpo import _wide_circuit
    n, ro = 9, [0, 4, 8]
    for seed in range(3):
        circ, k = _wide_circuit(n, seed)
        sim = Simulator(circ, ro, backend="mps", device=cuda)
        if sim.prog.hip_program() is None:
            continue                                       # a draw wider than bond 16
        dense = Simulator(circ, ro)
        g = torch.Generator().manual_seed(seed)
        v = torch.randn(5, k, generator=g) * 2
        w = torch.randn(5, len(ro), generator=g)
        z, gr = sim.vjp(v.to(cuda), w.to(cuda))
        z_ref, g_ref = dense.vjp(v, w)
        torch.cuda.synchronize()
        np.testing.assert_allclose(z.cpu().numpy(), z_ref.numpy(), atol=2e-5)
        np.testing.assert_allclose(gr.cpu().numpy(), g_ref.numpy(), atol=5e-5)
        assert sim.prog.hip_program().launches == 2
