"""Native pass planner: the register-level emulator of the plan (same semantics as the gfx950 kernel,
including the precomputed remap / address tables) must reproduce the float64 oracle for forward,
readout and adjoint gradients, on VQCs and on random generic circuits."""
import numpy as np
import pytest
import torch

from qfedx_amd.models.vqc import VQCSpec
from qfedx_amd.ops.plan_tools import emulate_adjoint, emulate_forward, parse_blob
from qfedx_amd.ops.statevec_torch import TorchProgram
from qfedx_amd.quantum.circuit import Circuit, ParameterVector
from qfedx_amd.quantum.statevector import Statevector

C = pytest.importorskip("qfedx_amd._qfedx_C", reason="native extension not built")


def _plan(ops, coef, n, R, kmax, readout, n_theta, mode, fin):
    return parse_blob(C.plan(torch.from_numpy(ops), torch.from_numpy(coef), n, R, kmax, readout, n_theta, mode, fin))


def _check(ops, coef, n, R, kmax, readout, n_theta, vals_theta, vals_x, circ, values, tol=1e-12):
    info = _plan(ops, coef, n, R, kmax, readout, n_theta, 0, 3)
    psi, out = emulate_forward(info, vals_theta, vals_x)
    sv = Statevector.from_instruction(circ, values)
    assert np.abs(psi - sv.data).max() < tol
    assert np.allclose(out, [sv.expectation_z(q) for q in readout], atol=tol)
    binfo = _plan(ops, coef, n, R, kmax, readout, n_theta, 2, 0)
    w = np.random.default_rng(1).normal(size=len(readout))
    g = emulate_adjoint(binfo, sv.data, vals_theta, vals_x, w)
    prog = TorchProgram(ops, coef, n, dtype=torch.complex128)
    rows = torch.from_numpy(np.concatenate([vals_theta, vals_x]))[None]
    gt = prog.adjoint_grads(rows, prog.run(rows), torch.from_numpy(w)[None], readout)[0].numpy()
    mask = np.array([0 <= s < n_theta and k <= 3 for k, s in zip(ops[:, 0], ops[:, 3])])
    assert np.abs(g[mask] - gt[mask]).max() < tol
    return info, binfo


@pytest.mark.parametrize("n,L,R,kmax,ent", [(2, 1, 4, 12, "chain"), (4, 2, 16, 12, "chain"), (8, 2, 4, 6, "ring"),
                                            (9, 3, 16, 7, "chain"), (10, 2, 4, 5, "chain"), (14, 2, 16, 12, "ring"),
                                            (16, 3, 16, 12, "chain")])
def test_vqc_plans_exact(n, L, R, kmax, ent):
    spec = VQCSpec(n_qubits=n, n_layers=L, n_classes=2 if n < 3 else 3, entangler=ent)
    ops, coef = spec.program()
    rng = np.random.default_rng(n)
    th, x = rng.normal(size=spec.n_theta), rng.uniform(0, 3, n)
    info, _ = _check(ops, coef, n, R, kmax, spec.readout, spec.n_theta, th, x, spec.circuit(), {"theta": th, "x": x})
    if n == 16:   # fusion quality: 3-layer 16-qubit VQC forward in 2 passes
        assert info["npass"] == 2


@pytest.mark.parametrize("seed", range(6))
def test_random_generic_circuits(seed):
    rng = np.random.default_rng(seed)
    n = int(rng.integers(6, 11))
    th = ParameterVector("theta", 40)
    qc = Circuit(n)
    k = 0
    for _ in range(60):
        r = rng.random()
        q = int(rng.integers(n))
        if r < 0.35:
            g = ["rx", "ry", "rz", "p"][int(rng.integers(4))]
            getattr(qc, g)(float(rng.uniform(0.5, 1.5)) * th[k % 40] + float(rng.normal()), q)
            k += 1
        elif r < 0.55:
            getattr(qc, ["h", "x", "y", "z", "s", "sdg", "t", "tdg", "sx"][int(rng.integers(9))])(q)
        elif r < 0.85:
            a, b = rng.choice(n, 2, replace=False)
            qc.cx(int(a), int(b))
        else:
            a, b = rng.choice(n, 2, replace=False)
            qc.cz(int(a), int(b))
    ops, coef = qc.to_program({"theta": 0, "x": 40})
    vals = rng.normal(size=40)
    readout = [0, n - 1]
    # gate scale/offset are stored as float32 in the program table -> ~1e-8 vs the float64 oracle
    _check(ops, coef, n, 4, 5, readout, 40, vals, np.zeros(1), qc, {"theta": vals}, tol=1e-6)
    _check(ops, coef, n, 16, 7, readout, 40, vals, np.zeros(1), qc, {"theta": vals}, tol=1e-6)


def test_jit_codegen_emits_straight_line_kernel():
    spec = VQCSpec(n_qubits=12, n_layers=2, n_classes=3)
    ops, coef = spec.program()
    blob = C.plan(torch.from_numpy(ops), torch.from_numpy(coef), 12, 16, 12, spec.readout, spec.n_theta, 2, 0)
    src = C.jit_source(blob, 0, True)
    assert "qfx_jit_pass" in src and "adj_step<R," in src and "switch" not in src


def _jit_worker(cache, n_layers, q):
    import torch as _t
    from qfedx_amd.ops._ext import ext as _ext
    from qfedx_amd.ops.statevec_hip import ARCH, CSRC
    spec = VQCSpec(n_qubits=8, n_layers=n_layers, n_classes=2)
    ops, coef = spec.program()
    Cx = _ext()
    blob = Cx.plan(_t.from_numpy(ops), _t.from_numpy(coef), 8, 16, 8, spec.readout, spec.n_theta, 2, 0)
    q.put(Cx.jit_prepare(blob, 0, False, cache, CSRC, ARCH, False)[1])


def test_jit_cache_concurrent_writers(tmp_path):
    """Ranks of a node share the code-object cache: several processes compiling the same pass at once leave one
    complete entry (per-process temp files renamed into place), byte-identical to a single process's compile."""
    import multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    shared, alone = str(tmp_path / "shared"), str(tmp_path / "alone")
    procs = [ctx.Process(target=_jit_worker, args=(shared, 1, q)) for _ in range(4)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(300)
        assert p.exitcode == 0
    keys = {q.get(timeout=10) for _ in procs}
    p = ctx.Process(target=_jit_worker, args=(alone, 1, q))
    p.start()
    p.join(300)
    assert p.exitcode == 0 and q.get(timeout=10) in keys and len(keys) == 1
    import os
    names = sorted(os.listdir(shared))
    assert not [f for f in names if f.endswith(".tmp")], names
    key = keys.pop()
    a = open(os.path.join(shared, key + ".co"), "rb").read()
    b = open(os.path.join(alone, key + ".co"), "rb").read()
    assert len(a) > 0 and a == b


def test_prologue_gather_packing_and_upload_fold_gate():
    """The round prologue gathers short rows (the VQC's n features) 256 / tps to a block, tps = the next power of two
    >= n lanes (csrc/train_kernels.hip qfx_prologue_gather_lanes); rows past 64 floats keep one block each.  The
    trainer's upload-fold gate counts those blocks (64 clients x 32 samples of 16 features: 128 blocks, folded; the
    CNN's 4,096 784-pixel rows: 4,096 blocks, not folded)."""
    from qfedx_amd.fl.trainer import FOLD_UPLOAD_MAX_BLOCKS, VQCClientTrainer
    assert [C.prologue_gather_lanes(f) for f in (1, 8, 9, 16, 20, 64, 65, 784)] == [8, 8, 16, 16, 32, 64, 0, 0]
    assert VQCClientTrainer._gather_blocks(2048, 16) == 128 <= FOLD_UPLOAD_MAX_BLOCKS
    assert VQCClientTrainer._gather_blocks(256, 16) == 16
    assert VQCClientTrainer._gather_blocks(2049, 20) == 257
    assert VQCClientTrainer._gather_blocks(4096, 784) == 4096 > FOLD_UPLOAD_MAX_BLOCKS
