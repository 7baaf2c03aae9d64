"""Column-environment contraction of the CNOT-chain VQC (quantum/mps_chain.py, the oracle of csrc/mps_chain.hip)
against the dense statevector engine: <Z_c> and the adjoint gradient of sum_c w_c <Z_c>."""
import numpy as np
import pytest
import torch

from qfedx_amd.models.vqc import VQCSpec
from qfedx_amd.ops.statevec_torch import TorchProgram, slot_grads
from qfedx_amd.quantum.mps_chain import chain_columns, eligible


@pytest.mark.parametrize("n,L,C,feat", [(5, 1, 2, "ry"), (6, 2, 3, "rx"), (6, 3, 3, "ry"), (7, 3, 4, "rz"),
                                        (4, 3, 2, "ry")])
def test_columns_match_dense_statevector(n, L, C, feat):
    spec = VQCSpec(n, L, C, feature_map=feat, readout=list(range(C)) if C != 4 else [1, 3, 4, 6])
    assert eligible(spec)
    g = np.random.default_rng(n * 10 + L)
    S = 3
    x = g.uniform(0, 3, (S, n))
    th = g.normal(size=(S, spec.n_theta))
    w = g.normal(size=(S, C))
    z, gr = chain_columns(x, th, n, L, spec.readout, feat, w)
    ops, coef = spec.program()
    prog = TorchProgram(ops, coef, n, "cpu", dtype=torch.complex128)
    rows = torch.cat([torch.from_numpy(th), torch.from_numpy(x)], 1)
    psi = prog.run(rows)
    zt = prog.expz(psi, spec.readout)
    gg = prog.adjoint_grads(rows, psi, torch.from_numpy(w), spec.readout)
    gt = slot_grads(gg, torch.from_numpy(ops), torch.from_numpy(coef), spec.n_theta + spec.x_width)[:, : spec.n_theta]
    np.testing.assert_allclose(z, zt.numpy(), atol=1e-10)
    np.testing.assert_allclose(gr, gt.numpy(), atol=1e-10)
