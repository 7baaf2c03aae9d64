"""CPU tests of the MFMA-engine pass planner: tile-exact emulation with the kernel's addressing tables
vs a dense float64 simulation (expectations and adjoint gradients), plan structure, table invariants."""
import numpy as np
import pytest
import torch

from qfedx_amd.models.vqc import VQCSpec
from qfedx_amd.ops import hea_plan as hp
from qfedx_amd.ops.statevec_torch import TorchProgram, slot_grads


def _dense(spec, xang, params, wread):
    ops, coef = spec.program()
    prog = TorchProgram(ops, coef, spec.n_qubits, dtype=torch.complex128)
    K, B, n = xang.shape
    P = spec.n_theta
    rows = torch.cat([params[:, None, :P].expand(K, B, P), xang], -1).reshape(K * B, -1)
    psi = prog.run(rows)
    ez = prog.expz(psi, spec.readout).reshape(K, B, -1)
    g = prog.adjoint_grads(rows, psi, wread.reshape(K * B, -1), spec.readout)
    return ez.numpy(), slot_grads(g, prog.ops, prog.coef, rows.shape[1])[:, :P].reshape(K, B, P).sum(1).numpy()


@pytest.mark.parametrize("n,L,t,chain,feat", [(8, 2, 8, True, "ry"), (10, 3, 8, True, "ry"), (10, 3, 14, True, "rx"),
                                              (11, 2, 8, False, "ry"), (12, 4, 9, True, "ry"), (9, 1, 8, True, "rz"),
                                              # trimmed plans (ragged layer tails deferred to a later pass)
                                              (11, 2, 10, True, "ry"), (13, 3, 9, True, "ry"),
                                              # per-layer trimming of the first pass (10q: 7 -> 6 ops)
                                              (12, 3, 10, True, "ry"), (9, 4, 8, True, "rz")])
def test_emulated_plan_matches_dense(n, L, t, chain, feat):
    spec = VQCSpec(n, L, 3, feature_map=feat, entangler="chain" if chain else "none")
    plan = hp.build_plan(n, L, spec.readout, chain, feat, tile_bits=t)
    g = torch.Generator().manual_seed(n * 10 + L)
    x = torch.rand(2, 2, n, generator=g, dtype=torch.float64) * 3
    params = torch.randn(2, spec.n_params, generator=g, dtype=torch.float64)
    wr = torch.randn(2, 2, 3, generator=g, dtype=torch.float64)
    ez, gr = _dense(spec, x, params, wr)
    ez2, gr2 = hp.emulate(plan, x.numpy(), params.numpy(), wr.numpy())
    np.testing.assert_allclose(ez2, ez, atol=1e-12)
    np.testing.assert_allclose(gr2, gr, atol=1e-12)
    ez3, gr3 = hp.emulate(plan, x.numpy(), params.numpy(), wr.numpy(), fp16=True)   # kernel storage format
    np.testing.assert_allclose(ez3, ez, atol=2e-3)
    np.testing.assert_allclose(gr3, gr, atol=3e-3 * max(1.0, np.abs(gr).max()))


def test_bf16_rounding_matches_hardware_conversion():
    """_bf16 is round-to-nearest-even on the fp32 bits (v_cvt_pk_bf16_f32): ties go to the even significand."""
    x = np.array([1.0, 1.0 + 2 ** -8, 1.0 + 3 * 2 ** -8, 1.0 + 2 ** -9, -1.5 - 2 ** -9, 3.0e38, 1e-40], np.float64)
    got = hp._bf16(x)
    assert got[0] == 1.0
    assert got[1] == 1.0                       # 1 + 2^-8 is a tie between 1 and 1 + 2^-7: to even (1)
    assert got[2] == 1.0 + 2 ** -6             # 1 + 3 2^-8 tie: to even (1 + 2^-6)
    assert got[3] == 1.0 and got[4] == -1.5
    assert np.isfinite(got[5]) and abs(got[6]) < 1e-38


@pytest.mark.parametrize("n,L,t", [(10, 3, 8), (12, 3, 9), (11, 2, 10)])
def test_emulated_bf16_storage_error_band(n, L, t):
    """bf16 state storage (BASELINE config 2) on the tile-exact emulator: errors vs the float64 dense oracle are
    above fp16's (8 vs 11 significand bits) and inside the band the bf16 GPU tests use (tests/test_gpu_hea.py)."""
    spec = VQCSpec(n, L, 3)
    plan = hp.build_plan(n, L, spec.readout, True, "ry", tile_bits=t)
    g = torch.Generator().manual_seed(n + L)
    x = torch.rand(2, 2, n, generator=g, dtype=torch.float64) * 3
    params = torch.randn(2, spec.n_params, generator=g, dtype=torch.float64)
    wr = torch.randn(2, 2, 3, generator=g, dtype=torch.float64)
    ez, gr = _dense(spec, x, params, wr)
    e16, g16 = hp.emulate(plan, x.numpy(), params.numpy(), wr.numpy(), storage="fp16")
    eb, gb = hp.emulate(plan, x.numpy(), params.numpy(), wr.numpy(), storage="bf16")
    sc = max(1.0, np.abs(gr).max())
    assert np.abs(eb - ez).max() < 2.5e-2 and np.abs(gb - gr).max() < 3e-2 * sc
    assert np.abs(eb - ez).max() > np.abs(e16 - ez).max()


@pytest.mark.parametrize("n,L,passes", [(16, 3, 2), (16, 2, 2), (20, 2, 2), (20, 3, 2), (24, 2, 3), (12, 3, 1)])
def test_plan_shapes(n, L, passes):
    plan = hp.build_plan(n, L, [0, 1, 2])
    assert len(plan.passes) == passes
    # every rotation (layer >= 2, qubit) lands in exactly one group, every qubit's layer-1 gradient once
    seen = sorted((g.layer, q) for p in plan.passes for g in p.groups for q in g.qubits)
    assert seen == sorted((layer, q) for layer in range(2, L + 1) for q in range(n))
    l1 = sorted(q for p in plan.passes for g in p.l1 for q in g.qubits)
    assert l1 == list(range(n))
    for p in plan.passes:
        assert p.t <= hp.TILE_BITS and p.c >= 2
        for g in p.groups:
            assert g.support(n) & ~p.mask() == 0


def test_group_tables_cover_tile_once():
    """(column, m) -> y'(col) ^ OFF[m ^ b] is a bijection onto the tile for every op and tile."""
    plan = hp.build_plan(16, 3, [0, 1, 2])
    for p in plan.passes:
        for g in p.groups + p.l1:
            w = hp.group_table(plan, p, g, hp.OP_APPLY)
            for tid in (0, (1 << (16 - p.t)) - 1):
                a = hp._addr(w, p.t, p.fixed(tid, 16))
                assert np.array_equal(np.sort(a.ravel()), np.arange(1 << p.t))


def test_frame_algebra():
    n = 12
    for k in range(4):
        R = hp.frame_rows(k, n)
        for q in range(n):
            v = hp.frame_vec(q, k, n)
            assert [hp.parity(v & R[j]) for j in range(n)] == [int(j == q) for j in range(n)]


def test_eligibility():
    assert hp.eligible(VQCSpec(16, 3, 3))
    assert not hp.eligible(VQCSpec(16, 3, 3, entangler="ring"))
    assert not hp.eligible(VQCSpec(4, 2, 3))
    assert not hp.eligible(VQCSpec(8, 2, 3, feature_map="amplitude"))


def test_trimmed_plan_full_groups():
    """16q x 3L: deferring layer tails gives 8 full group ops (greedy: 10) in the same 2 passes, and the
    LDS swizzle search still reaches the conflict-free score for every group of every pass."""
    greedy = hp.build_plan(16, 3, [0, 1, 2], trim=False)
    plan = hp.build_plan(16, 3, [0, 1, 2])
    assert len(plan.passes) == len(greedy.passes) == 2
    assert sum(len(p.groups) for p in plan.passes) == 8 < sum(len(p.groups) for p in greedy.passes)
    assert all(len(g.qubits) == hp.GROUP for p in plan.passes for g in p.groups)
    p20 = hp.build_plan(20, 2, [0, 1, 2], swizzle=False)       # the 20q DP suite config: 6 -> 5 ops
    assert len(p20.passes) == 2 and sum(len(p.groups) for p in p20.passes) == 5
    for n, L, t in [(11, 2, 10), (13, 3, 9), (10, 3, 8), (12, 3, 10)]:
        a = hp.build_plan(n, L, [0, 1, 2], tile_bits=t, trim=False)
        b = hp.build_plan(n, L, [0, 1, 2], tile_bits=t)
        assert len(b.passes) == len(a.passes)
        assert sum(len(p.groups) for p in b.passes) < sum(len(p.groups) for p in a.passes)
    for p in plan.passes:
        # every group that runs as a single op under the default pair mask is conflict free (paired groups are
        # scored as pairs: profiles/r5 stall tables)
        solo = hp.single_op_groups(plan, p, 7)
        groups = [g for g in p.groups + p.l1 if (g.layer, tuple(g.qubits)) in solo]
        total = 0
        for g in groups:
            allv, dirs = hp._group_geom(plan, p, g)[0], hp._group_geom(plan, p, g)[6]
            total += hp._best_cols(p.H, allv, dirs, g in p.groups)[0]
        assert total == hp.FULL_SCORE * len(groups)


@pytest.mark.parametrize("n,L,tile,min_ratio", [(24, 3, 14, 2.0), (16, 3, 14, 2.0), (14, 3, 10, 2.0),
                                                (12, 3, 14, 1.5)])
def test_param_shift_owners_and_pass_savings(n, L, tile, min_ratio):
    """Every parameter is applied by exactly one forward pass (layer 1 in the generating pass 0), and the
    prefix-reuse + pi-identity estimator launches >= 2x fewer passes than 2 n_theta naive shifted circuits
    (adjoint passes weighted 2x)."""
    from qfedx_amd.models.vqc import VQCSpec
    from qfedx_amd.ops.hea_mfma import HeaMfmaProgram
    prog = HeaMfmaProgram(VQCSpec(n, L, 2), "cpu", tile_bits=tile)
    own = prog.shift_owners()
    assert sorted(i for o in own for i in o) == list(range(prog.n_theta))
    assert all(prog.plan.theta_slot(1, q) in own[0] for q in range(n))
    c = prog.shift_pass_counts()
    assert c["naive_fwd_passes"] / (c["reuse_fwd_passes"] + 2 * c["reuse_adj_passes"]) >= min_ratio


def test_pi_identity_of_shifted_expectations():
    """f(theta +- pi/2) = (f(theta) + f(theta + pi)) / 2 +- f'(theta) for every rotation parameter of the HEA
    (float64 dense oracle; the identity HeaMfmaProgram.shifted_expz builds on)."""
    import torch
    from qfedx_amd.models.vqc import VQCSpec
    from qfedx_amd.ops.statevec_torch import TorchProgram, slot_grads
    spec = VQCSpec(5, 3, 2)
    ops, coef = spec.program()
    prog = TorchProgram(ops, coef, 5, dtype=torch.complex128)
    g = torch.Generator().manual_seed(0)
    P = spec.n_theta
    th = torch.randn(P, generator=g, dtype=torch.float64)
    x = torch.rand(5, generator=g, dtype=torch.float64) * 3
    rows = []
    for d in (0.0, np.pi, np.pi / 2, -np.pi / 2):
        for j in range(P):
            t = th.clone()
            t[j] += d
            rows.append(torch.cat([t, x]))
    z = prog.expz(prog.run(torch.stack(rows)), spec.readout).reshape(4, P, -1)
    base = torch.cat([th, x])[None]
    psi = prog.run(base)
    for c in range(2):
        w = torch.zeros(1, 2, dtype=torch.float64)
        w[0, c] = 1
        gg = slot_grads(prog.adjoint_grads(base, psi, w, spec.readout), prog.ops, prog.coef, base.shape[1])[0, :P]
        m = 0.5 * (z[0, :, c] + z[1, :, c])
        np.testing.assert_allclose(z[2, :, c].numpy(), (m + gg).numpy(), atol=1e-10)
        np.testing.assert_allclose(z[3, :, c].numpy(), (m - gg).numpy(), atol=1e-10)


@pytest.mark.parametrize("n,L,t", [(12, 3, 11), (14, 2, 12), (16, 3, 14), (16, 3, 13), (13, 4, 11)])
def test_pair_ops_emulated_match_dense_and_unpaired(n, L, t):
    """Chained pair ops (APPLY2 / BACK2 / GRAD2, hea_plan.pair_table): emulated tile by tile with the pair records'
    coset addressing they give the dense float64 results, and in the fp16 storage format they round at exactly the
    points the unpaired program rounds (bitwise the same expectations and gradients)."""
    spec = VQCSpec(n, L, 3)
    plan = hp.build_plan(n, L, spec.readout, True, "ry", tile_bits=t)
    progs = hp.pass_programs(plan, pair=True)
    codes = {int(w[hp.W_CODE]) for _, f, a in progs for w in list(f) + list(a)}
    assert hp.OP_APPLY2 in codes and hp.OP_BACK2 in codes
    g = torch.Generator().manual_seed(n * 7 + L)
    x = torch.rand(2, 2, n, generator=g, dtype=torch.float64) * 3
    params = torch.randn(2, spec.n_params, generator=g, dtype=torch.float64)
    wr = torch.randn(2, 2, 3, generator=g, dtype=torch.float64)
    ez, gr = _dense(spec, x, params, wr)
    ez2, gr2 = hp.emulate(plan, x.numpy(), params.numpy(), wr.numpy())
    np.testing.assert_allclose(ez2, ez, atol=1e-12)
    np.testing.assert_allclose(gr2, gr, atol=1e-12)
    import os
    ez3, gr3 = hp.emulate(plan, x.numpy(), params.numpy(), wr.numpy(), fp16=True)
    os.environ["QFEDX_HEA_PAIR"] = "0"
    try:
        assert not {int(w[hp.W_CODE]) for _, f, a in hp.pass_programs(plan) for w in list(f) + list(a)} & set(hp.PAIR_CODES)
        ez4, gr4 = hp.emulate(plan, x.numpy(), params.numpy(), wr.numpy(), fp16=True)
    finally:
        del os.environ["QFEDX_HEA_PAIR"]
    np.testing.assert_array_equal(ez3, ez4)
    np.testing.assert_allclose(gr3, gr4, atol=1e-12)


def test_pair_gradient_records_keep_unpaired_order():
    """A pair op carries two gradient records in the unpaired program's order (the slab layout and hea_grad_reduce
    are unchanged): same gmeta rows with and without pairing."""
    spec = VQCSpec(16, 3, 3)
    plan = hp.build_plan(16, 3, spec.readout, True, "ry", tile_bits=13)
    m1, m0 = [], []
    hp.pass_programs(plan, m1, pair=True)
    hp.pass_programs(plan, m0, pair=False)
    assert m1 == m0 and len(m1) > 0


def test_pair_only_pass_counts_as_applying():
    """A forward pass whose only group ops are chained pairs still applies unitaries: the forward reads out at the
    last such pass (20q x 2L: pass 1 is [APPLY2, READOUT]; counting single APPLY ops only stopped the forward one
    pass early, which <Z> of the low readout qubits could not see)."""
    import torch
    from qfedx_amd.ops.hea_mfma import HeaMfmaProgram
    spec = VQCSpec(20, 2, 3)
    plan = hp.build_plan(20, 2, spec.readout, True, "ry", tile_bits=14)
    progs = hp.pass_programs(plan)
    assert [int(w[hp.W_CODE]) for w in progs[-1][1]] == [hp.OP_APPLY2, hp.OP_READOUT]
    prog = HeaMfmaProgram(spec, torch.device("cpu"))
    assert prog.fwd_last == len(prog.passes) - 1


@pytest.mark.parametrize("n,L,t", [(16, 3, 14), (16, 3, 13), (20, 2, 13), (12, 3, 10)])
def test_fo_table_matches_per_tile_op_bases(n, L, t):
    """The host table of per-(tile, op) OFF bases the pass kernels read in their prologue equals the kernels' former
    in-kernel computation (parities of the tile's fixed bits with each op's frame row masks; pair records XOR both
    groups' entries; OBS / READOUT 0) for every tile of every pass program."""
    from qfedx_amd.models.vqc import VQCSpec
    spec = VQCSpec(n, L, 3)
    plan = hp.build_plan(n, L, spec.readout, True, "ry", tile_bits=t)
    for p, fwd, adj in hp.pass_programs(plan, []):
        for ops in (fwd, adj):
            tab = hp.fo_table(ops, p, n).view(np.uint32)
            for tile, fixed in enumerate(hp.tile_fixed(p, n)):
                for o, w in enumerate(ops):
                    code = int(w[hp.W_CODE])
                    want = 0
                    if code not in (hp.OP_OBS, hp.OP_READOUT):
                        fp = sum(hp.parity(int(fixed) & int(w[hp.W_RFULL + j])) << j for j in range(int(w[hp.W_NREAL])))
                        want = int(w[hp.W_OFF + fp])
                        if code in hp.PAIR_CODES:
                            fy = sum(hp.parity(int(fixed) & int(w[hp.W_RFULL2 + j])) << j for j in range(4))
                            want ^= int(w[hp.W_OFF2 + fy])
                    assert int(tab[tile, o]) == want
