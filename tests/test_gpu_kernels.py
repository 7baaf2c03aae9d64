"""GPU numerics tests: every gfx950 kernel vs a plain PyTorch / float64 reference of the same op."""
import math

import numpy as np
import pytest
import torch

from qfedx_amd.models.vqc import VQCSpec
from qfedx_amd.ops.engine import VQCEngine
from qfedx_amd.quantum.statevector import Statevector

pytestmark = pytest.mark.gpu


def _setup(n, L, C, K, B, seed=0, ent="chain"):
    spec = VQCSpec(n_qubits=n, n_layers=L, n_classes=C, init_std=1.0, entangler=ent, readout_scale=2.0)
    g = torch.Generator().manual_seed(seed)
    x = torch.rand(K, B, n, generator=g)
    y = torch.randint(0, C, (K, B), generator=g)
    w = torch.full((K, B), 1.0 / B)
    params = torch.stack([spec.init_params(seed + k) for k in range(K)])
    params[:, : spec.n_theta] += torch.randn(K, spec.n_theta, generator=g)
    return spec, x, y, w, params


@pytest.mark.parametrize("n,L,K,B,ent", [(2, 1, 3, 5, "chain"), (4, 2, 4, 7, "chain"), (6, 2, 2, 9, "ring"),
                                         (8, 3, 3, 4, "chain"), (10, 2, 3, 3, "chain"), (11, 2, 3, 3, "ring"),
                                         (12, 2, 2, 3, "ring"), (14, 2, 2, 2, "chain"),
                                         (16, 3, 2, 2, "chain")])
@pytest.mark.parametrize("jit", ["1", "0"])
def test_forward_expz_matches_torch(cuda, n, L, K, B, ent, jit, monkeypatch):
    monkeypatch.setenv("QFEDX_JIT", jit)
    C = 2 if n < 3 else 3
    spec, x, y, w, params = _setup(n, L, C, K, B, ent=ent)
    ref = VQCEngine(spec, "cpu", "torch")
    hip = VQCEngine(spec, cuda, "hip")
    xang = spec.encode_features(x)
    th = params[:, : spec.n_theta]
    z_ref = ref.expz(xang, th)
    z_hip = hip.expz(xang.to(cuda), th.to(cuda)).cpu()
    assert torch.allclose(z_hip, z_ref, atol=2e-5), (z_hip - z_ref).abs().max()


def test_forward_matches_float64_oracle(cuda):
    spec, x, y, w, params = _setup(10, 2, 3, 1, 1, seed=3)
    hip = VQCEngine(spec, cuda, "hip")
    xang = spec.encode_features(x)
    z = hip.expz(xang.to(cuda), params[:, : spec.n_theta].to(cuda)).cpu()[0, 0]
    sv = Statevector.from_instruction(spec.circuit(), {"theta": params[0, : spec.n_theta].double().numpy(),
                                                        "x": xang[0, 0].double().numpy()})
    ref = torch.tensor([sv.expectation_z(c) for c in spec.readout], dtype=torch.float32)
    assert torch.allclose(z, ref, atol=2e-5)


@pytest.mark.parametrize("n,L,K,B", [(3, 2, 2, 4), (4, 2, 3, 6), (8, 2, 2, 5), (10, 2, 2, 3), (11, 2, 3, 3), (13, 2, 2, 2), (16, 2, 2, 2)])
@pytest.mark.parametrize("jit", ["1", "0"])
def test_adjoint_grads_match_torch(cuda, n, L, K, B, jit, monkeypatch):
    monkeypatch.setenv("QFEDX_JIT", jit)
    spec, x, y, w, params = _setup(n, L, 3 if n >= 3 else 2, K, B, seed=n)
    ref = VQCEngine(spec, "cpu", "torch")
    hip = VQCEngine(spec, cuda, "hip")
    xang = spec.encode_features(x)
    r_ref = ref.loss_and_grads(xang, y, w, params, "adjoint")
    r_hip = hip.loss_and_grads(xang.to(cuda), y.to(cuda), w.to(cuda), params.to(cuda), "adjoint")
    assert torch.allclose(r_hip["loss"].cpu(), r_ref["loss"], atol=2e-5)
    assert torch.allclose(r_hip["grad"].cpu(), r_ref["grad"], atol=5e-5), (r_hip["grad"].cpu() - r_ref["grad"]).abs().max()
    assert torch.equal(r_hip["correct"].cpu(), r_ref["correct"])


def test_adjoint_matches_param_shift_on_gpu(cuda):
    spec, x, y, w, params = _setup(6, 2, 3, 2, 3, seed=11)
    hip = VQCEngine(spec, cuda, "hip")
    xang = spec.encode_features(x).to(cuda)
    a = hip.loss_and_grads(xang, y.to(cuda), w.to(cuda), params.to(cuda), "adjoint")["grad"]
    ps = VQCEngine(spec, "cpu", "torch").loss_and_grads(xang.cpu(), y, w, params, "param_shift")["grad"]
    assert torch.allclose(a.cpu(), ps, atol=5e-5)


def test_fused_adam_matches_torch(cuda):
    from qfedx_amd.fl.optim import BatchedOptimizer
    K, P = 5, 37
    g = torch.Generator().manual_seed(0)
    p0 = torch.randn(K, P, generator=g)
    grads = [torch.randn(K, P, generator=g) for _ in range(3)]
    active = torch.tensor([1, 1, 0, 1, 1], dtype=torch.float32)
    for kind in ("adam", "sgd"):
        pc, pg = p0.clone(), p0.clone().to(cuda)
        oc = BatchedOptimizer(kind, (K, P), "cpu", 0.05, backend="torch")
        og = BatchedOptimizer(kind, (K, P), cuda, 0.05, backend="hip")
        for gr in grads:
            oc.step(pc, gr, active)
            og.step(pg, gr.to(cuda), active.to(cuda))
        assert torch.allclose(pg.cpu(), pc, atol=1e-6), kind


@pytest.mark.parametrize("dp", [False, True])
def test_fused_fedavg_reduce_matches_torch(cuda, dp):
    from qfedx_amd.fl.aggregator import Aggregator
    K, P = 6, 50
    g = torch.Generator().manual_seed(1)
    tk = torch.randn(K, P, generator=g) * 3
    tg = torch.randn(P, generator=g)
    mask = torch.zeros(P)
    mask[:40] = 1
    w = torch.rand(K, generator=g).double() + 0.5
    ids = [3, 7, 8, 11, 20, 21]
    cpu = Aggregator(P, mask, "cpu", "torch", dp=dp, clip_norm=0.7, noise_multiplier=1.3, seed=5)
    gpu = Aggregator(P, mask, cuda, "hip", dp=dp, clip_norm=0.7, noise_multiplier=1.3, seed=5)
    a = cpu.finalize(cpu.local_reduce(tk, tg, w, 4, ids))[0]
    b = gpu.finalize(gpu.local_reduce(tk.to(cuda), tg.to(cuda), w.to(cuda), 4, ids).cpu())[0]
    assert torch.allclose(a, b, atol=1e-6, rtol=1e-6), (a - b).abs().max()


@pytest.mark.parametrize("K,P", [(150, 20000), (150, 20003), (37, 16385), (64, 300), (130, 113859), (20, 9001)])
def test_fedavg_fixed_point_sum_exact(cuda, K, P):
    """The FedAvg reduce's int64 sums equal the host's exact fixed-point sums bitwise, over client counts that take
    every client-batch path (4 rows in flight per thread, single rows) and the CFed TinyCNN's vector length."""
    import numpy as np
    from qfedx_amd.ops import fedavg_hip
    g = torch.Generator().manual_seed(K + P)
    tk = torch.randn(K, P, generator=g) * 0.2
    tg = torch.randn(P, generator=g)
    w = torch.rand(K, generator=g).double() * 30 + 0.5
    mask = torch.zeros(P, dtype=torch.uint8, device=cuda)
    out, _, sat = fedavg_hip.fused_local_reduce(tk.to(cuda), tg.to(cuda), w.to(cuda), mask, list(range(K)), 0, 0,
                                                False, False, 1.0, 0.0)
    d = tk.double().numpy() - tg.double().numpy()[None, :]
    terms = np.rint(w.numpy()[:, None] * d * 4294967296.0).astype(np.int64)
    ref = np.concatenate([terms.sum(0), [np.rint(w.numpy() * 4294967296.0).astype(np.int64).sum()]])
    assert np.array_equal(out.cpu().numpy(), ref) and int(sat.item()) == 0


@pytest.mark.parametrize("fraction,sampling,dp", [(1.0, "fixed", False), (0.5, "fixed", False),
                                                  (0.5, "poisson", False), (0.5, "poisson", True)])
def test_graph_round_matches_eager(cuda, fraction, sampling, dp):
    """hipGraph-replayed local rounds produce the same global model as eager launches (with client
    sampling the set changes every round while the captured shape is reused; under Poisson sampling the
    client count changes too and the graph runs padded to its bucket, trainer.graph_bucket)."""
    from tests.test_fl import small_cfg
    from qfedx_amd.api import run_experiment
    from qfedx_amd.parallel.dist import init_distributed
    outs = []
    for graphs in (True, False):
        cfg = small_cfg(num_rounds=6, n_qubits=6, device="cuda", backend="hip", client_fraction=fraction,
                        sampling=sampling, num_clients=7, dp=dp, deterministic_noise=dp, noise_multiplier=0.3)
        dev = torch.device("cuda", 0)
        world = init_distributed(dev)
        import qfedx_amd.fl.trainer as tr
        old = tr.VQCClientTrainer.use_graph
        tr.VQCClientTrainer.use_graph = property(lambda self, g=graphs: g)
        try:
            outs.append(run_experiment(cfg, world=world, device=dev, backend="hip"))
        finally:
            tr.VQCClientTrainer.use_graph = old
    assert torch.equal(outs[0]["params"], outs[1]["params"])


def test_upfront_and_per_step_gathers_give_the_same_run(cuda, monkeypatch):
    """Rounds whose minibatches are gathered by the prologue launch == rounds gathering per step (the path taken
    past UPFRONT_GATHER_BYTES), bitwise, with several local steps per round."""
    from tests.test_fl import small_cfg
    from qfedx_amd.api import run_experiment
    from qfedx_amd.parallel.dist import init_distributed
    import qfedx_amd.fl.trainer as tr
    outs = []
    for cap in (tr.UPFRONT_GATHER_BYTES, 0):
        monkeypatch.setattr(tr, "UPFRONT_GATHER_BYTES", cap)
        cfg = small_cfg(num_rounds=3, n_qubits=8, device="cuda", backend="hip", num_clients=5, local_epochs=2)
        dev = torch.device("cuda", 0)
        outs.append(run_experiment(cfg, world=init_distributed(dev), device=dev, backend="hip"))
    assert torch.equal(outs[0]["params"], outs[1]["params"])


def test_hip_federated_run_matches_cpu(cuda):
    from tests.test_fl import small_cfg
    from qfedx_amd.api import run_experiment
    from qfedx_amd.parallel.dist import init_distributed
    # SGD: Adam would blow fp32 noise on the zero-gradient angles (last-layer RZ, unmeasured
    # qubits) up to lr-sized steps of random sign, so those would not be comparable
    cpu = run_experiment(small_cfg(num_rounds=2, optimizer="sgd"))
    dev = torch.device("cuda", 0)
    gpu = run_experiment(small_cfg(num_rounds=2, optimizer="sgd", device="cuda", backend="hip"),
                         world=init_distributed(dev), device=dev, backend="hip")
    assert torch.allclose(gpu["params"].cpu(), cpu["params"], atol=1e-4)
    for hg, hc in zip(gpu["history"], cpu["history"]):
        assert abs(hg["train_loss"] - hc["train_loss"]) < 1e-4


@pytest.mark.parametrize("n,L", [(6, 2), (13, 2), (16, 3)])
def test_bf16_state_storage_close_to_fp32(cuda, n, L):
    """state_dtype=bf16: packed bf16 amplitudes between passes (fp32 compute) stay close to fp32."""
    spec, x, y, w, params = _setup(n, L, 3, 2, 8, seed=4)
    f32 = VQCEngine(spec, cuda, "hip", "fp32")
    b16 = VQCEngine(spec, cuda, "hip", "bf16")
    xa = spec.encode_features(x).to(cuda)
    th = spec.split(params)[0].to(cuda)
    z32, z16 = f32.expz(xa, th), b16.expz(xa, th)
    assert (z32 - z16).abs().max().item() < 2e-2
    r32 = f32.loss_and_grads(xa, y.to(cuda), w.to(cuda), params.to(cuda), "adjoint")
    r16 = b16.loss_and_grads(xa, y.to(cuda), w.to(cuda), params.to(cuda), "adjoint")
    assert torch.allclose(r32["loss"], r16["loss"], atol=2e-2, rtol=2e-2)
    g32, g16 = r32["grad"], r16["grad"]
    rel = (g32 - g16).norm() / g32.norm()
    assert rel.item() < 0.05, rel.item()
    assert b16.hip._ws["psi"].dtype == torch.int32          # 4 bytes per amplitude


@pytest.mark.parametrize("mode,F", [(0, 16), (1, 16), (1, 300), (2, 784)])
def test_batch_gather_matches_torch(cuda, mode, F):
    """Fused per-step minibatch gather + encoding == torch indexing + angle_scale (bitwise)."""
    from qfedx_amd.data.features import angle_scale
    from qfedx_amd.ops._ext import ext
    g = torch.Generator().manual_seed(F)
    Nc, nmax, K, B = 7, 40, 4, 9
    X = torch.randn(Nc, nmax, F, generator=g)
    X[2, 3] = 0.5                                   # constant row -> minmax gives zeros
    Y = torch.randint(0, 5, (Nc, nmax), generator=g)
    lid = torch.tensor([5, 2, 0, 6])
    idx = torch.randint(0, nmax, (K, B), generator=g)
    idx[1, 0] = 3
    xo = torch.empty(K, B, F, device=cuda)
    yo = torch.empty(K * B, dtype=torch.int64, device=cuda)
    ext().batch_gather(X.to(cuda), Y.to(cuda), lid.to(cuda), idx.to(cuda), mode, 2.5, xo, yo)
    xb = X[lid[:, None], idx]
    ref = {0: lambda: angle_scale(xb, "scale", 2.5), 1: lambda: angle_scale(xb, "minmax"), 2: lambda: xb}[mode]()
    assert torch.equal(xo.cpu(), ref)
    assert torch.equal(yo.cpu().view(K, B), Y[lid[:, None], idx])


@pytest.mark.parametrize("mode,F", [(0, 16), (1, 16), (1, 300), (2, 784)])
def test_round_prologue_matches_init_and_per_step_gathers(cuda, mode, F):
    """One prologue launch (client rows + Adam state init, every step's minibatch gathered) == round_init +
    one batch_gather per step (bitwise)."""
    from qfedx_amd.ops._ext import ext
    g = torch.Generator().manual_seed(F + 1)
    Nc, nmax, K, B, S, P = 7, 40, 4, 9, 3, 3000
    X = torch.randn(Nc, nmax, F, generator=g).to(cuda)
    Y = torch.randint(0, 5, (Nc, nmax), generator=g).to(cuda)
    lid = torch.tensor([5, 2, 0, 6]).to(cuda)
    idx = torch.randint(0, nmax, (S, K, B), generator=g).to(cuda)
    theta = torch.randn(P, generator=g).to(cuda)
    xo = torch.full((S, K, B, F), 7.0, device=cuda)
    yo = torch.full((S * K * B,), -1, dtype=torch.int64, device=cuda)
    p, m, v, t = (torch.full((K, P), 9.0, device=cuda), torch.ones(K, P, device=cuda),
                  torch.ones(K, P, device=cuda), torch.ones(2, K, device=cuda))
    ext().round_prologue(theta, p, m, v, t, X, Y, lid, idx, mode, 2.5, xo, yo)
    p2, m2, v2, t2 = (torch.full((K, P), 9.0, device=cuda), torch.ones(K, P, device=cuda),
                      torch.ones(K, P, device=cuda), torch.ones(2, K, device=cuda))
    ext().round_init(theta, p2, m2, v2, t2)
    for s in range(S):
        xr = torch.empty(K, B, F, device=cuda)
        yr = torch.empty(K * B, dtype=torch.int64, device=cuda)
        ext().batch_gather(X, Y, lid, idx[s].contiguous(), mode, 2.5, xr, yr)
        assert torch.equal(xo[s], xr) and torch.equal(yo.view(S, K * B)[s], yr)
    for a, b in ((p, p2), (m, m2), (v, v2), (t, t2)):
        assert torch.equal(a, b)
    assert torch.equal(p, theta[None].expand(K, P)) and not m.any() and not t.any()


@pytest.mark.parametrize("dp", [False, True])
def test_fedavg_launch_packs_round_metrics(cuda, dp):
    """The FedAvg reduce with the metric pack fused into its last block == reduce + round_pack (bitwise)."""
    from qfedx_amd.ops import fedavg_hip
    from qfedx_amd.ops._ext import ext
    K, P, n = 5, 300, 24
    g = torch.Generator().manual_seed(2)
    tk = (torch.randn(K, P, generator=g) * 2).to(cuda)
    tg = torch.randn(P, generator=g).to(cuda)
    w = (torch.rand(K, generator=g).double() + 0.5).to(cuda)
    mask = (torch.arange(P) < 200).to(torch.uint8).to(cuda)
    mets = [torch.rand(n, generator=g).to(cuda) for _ in range(4)]
    keys = torch.randint(0, 2 ** 31 - 1, (K, 2), generator=g, dtype=torch.int64).to(torch.int32).to(cuda)
    bufs = []
    for fused in (True, False):
        buf = torch.full((P + 6,), 123, dtype=torch.int64, device=cuda)
        buf[P + 5] = 0
        fedavg_hip.fused_local_reduce(tk, tg, w, mask, list(range(K)), 3, 9, True, dp, 0.8, 1.1, out=buf[: P + 1],
                                      keys=keys, pack=(buf, *mets) if fused else None)
        if not fused:
            ext().round_pack(buf, P, *mets)
        bufs.append(buf.cpu())
    assert torch.equal(bufs[0][: P + 5], bufs[1][: P + 5])
    assert bufs[0][P + 5] == 0


@pytest.mark.parametrize("dp,P", [(False, 300), (True, 300), (False, 5000)])
def test_fedavg_fused_apply_matches_round_apply(cuda, dp, P):
    """Single-rank rounds: the FedAvg reduce whose last arriving block applies the round == reduce + round_apply
    (bitwise params, metrics, saturation count, weight sum and CC6 norm slots), twice in a row (the arrival counter
    resets itself)."""
    from qfedx_amd.ops import fedavg_hip
    from qfedx_amd.ops._ext import ext
    K, n, NN = 6, 24, 9 if dp else 0
    g = torch.Generator().manual_seed(P + dp)
    mask = (torch.arange(P) < P // 2).to(torch.uint8).to(cuda)
    cid = torch.tensor([0, 2, 3, 5, 7, 8], dtype=torch.int32).to(cuda) if dp else None
    keys = torch.randint(0, 2 ** 31 - 1, (K, 2), generator=g, dtype=torch.int64).to(torch.int32).to(cuda)
    theta0 = torch.randn(P, generator=g).to(cuda)
    thetas, outs = {}, {}
    cnt = torch.zeros(1, dtype=torch.int32, device=cuda)
    for fused in (True, False):
        gg = torch.Generator().manual_seed(7)
        theta = theta0.clone()
        buf = torch.zeros(P + 6 + NN, dtype=torch.int64, device=cuda)
        res = []
        for r in range(2):
            tk = (theta[None] + torch.randn(K, P, generator=gg).to(cuda) * 0.1).contiguous()
            w = (torch.rand(K, generator=gg).double() + 0.5).to(cuda)
            mets = [torch.rand(n, generator=gg).to(cuda) for _ in range(4)]
            out = torch.full((6 + NN,), -1.0, dtype=torch.float64, device=cuda)
            fedavg_hip.fused_local_reduce(tk, theta, w, mask, list(range(K)), r, 9, True, dp, 0.8, 1.1,
                                          out=buf[: P + 1], keys=keys, pack=(buf, *mets), norm_cid=cid,
                                          apply=(theta, out, cnt, 0, 1.0, NN) if fused else None)
            if not fused:
                ext().round_apply(buf, P, theta, 1.0, out, 0, 1.0, NN)
            res.append(out.cpu())
        thetas[fused], outs[fused] = theta.cpu(), res
    assert torch.equal(thetas[True], thetas[False]) and not torch.equal(thetas[True], theta0.cpu())
    for a, b in zip(outs[True], outs[False]):
        assert torch.equal(a, b)
    assert int(cnt.item()) == 0


def test_fedavg_saturation_is_counted_not_wrapped(cuda):
    """A fixed-point term past 2^53 (w * Delta > 2^21) is clamped and counted; round_apply reports the count
    and zeroes the counter for the next round."""
    from qfedx_amd.ops import fedavg_hip
    from qfedx_amd.ops._ext import ext
    K, P = 3, 70
    tg = torch.zeros(P, device=cuda)
    tk = torch.zeros(K, P, device=cuda)
    tk[1, 5] = 1.0e4
    tk[2, 6] = float("nan")
    w = torch.tensor([1.0, 1.0e3, 1.0], dtype=torch.float64, device=cuda)   # 1e3 * 1e4 = 1e7 > 2^21
    mask = torch.zeros(P, dtype=torch.uint8, device=cuda)
    buf = torch.zeros(P + 6, dtype=torch.int64, device=cuda)
    mets = [torch.zeros(4, device=cuda) for _ in range(4)]
    fedavg_hip.fused_local_reduce(tk, tg, w, mask, [0, 1, 2], 0, 0, False, False, 1.0, 0.0, out=buf[: P + 1],
                                  pack=(buf, *mets))
    assert int(buf[P + 5]) == 2 and int(buf[5]) == 2 ** 53 and int(buf[6]) == 0
    out = torch.zeros(6, dtype=torch.float64, device=cuda)
    theta = torch.zeros(P, device=cuda)
    ext().round_apply(buf, P, theta, 1.0, out, 0, 1.0, 0)
    torch.cuda.synchronize()
    assert out[4].item() == 2.0 and int(buf[P + 5]) == 0


def test_round_init_and_counter_pingpong(cuda):
    from qfedx_amd.fl.optim import BatchedOptimizer
    K, P = 5, 37
    theta = torch.randn(P)
    act = [torch.tensor([1., 1., 0., 1., 1.]), torch.tensor([1., 0., 0., 1., 1.]), torch.tensor([1., 0., 0., 0., 1.])]
    g = [torch.randn(K, P) for _ in range(3)]
    outs = []
    for dev, backend in (("cpu", "torch"), (cuda, "hip")):
        p = torch.empty(K, P, device=dev)
        opt = BatchedOptimizer("adam", (K, P), dev, 0.05, backend=backend)
        opt.init_round(p, theta.to(dev))
        for s in range(3):
            opt.step(p, g[s].to(dev), act[s].to(dev))
        outs.append((p.cpu(), opt.t.cpu()))
    assert torch.allclose(outs[0][0], outs[1][0], atol=1e-6)
    assert torch.equal(outs[0][1], outs[1][1]) and outs[1][1].tolist() == [3, 1, 0, 2, 3]


def test_host_upload_ring_roundtrip(cuda):
    """h2d / PackedUpload go through the pinned ring + copy kernel: exact bytes, also across slot reuse while
    earlier uploads may still be queued behind device work."""
    from qfedx_amd.utils.device import PackedUpload, h2d
    g = torch.Generator().manual_seed(3)
    a = torch.randn(512, 512, device=cuda)
    outs = []
    for it in range(40):                       # > ring slots: every slot is reused at least twice
        a = a @ a * 1e-3                       # keep the stream busy so uploads queue behind work
        t = torch.randint(-2 ** 40, 2 ** 40, (it + 3,), generator=g)
        w = torch.rand(it % 5 + 1, 3, generator=g)
        up = PackedUpload({"t": t, "w": w, "b": torch.tensor([it], dtype=torch.int32)})
        dv = up.to_device(cuda)
        outs.append((t, w, it, h2d(w * 2, cuda), dv))
    torch.cuda.synchronize()
    for t, w, it, w2, dv in outs:
        assert torch.equal(dv["t"].cpu(), t) and torch.equal(dv["w"].cpu(), w) and int(dv["b"].item()) == it
        assert torch.equal(w2.cpu(), w * 2)


def test_padded_inactive_client_rows_mfma(cuda):
    """MFMA engine, several local steps with clients that stop early (non-IID shard sizes) and a graph padded from
    3 to 4 client rows (trainer.graph_bucket): the active rows are bitwise the eager, unpadded run's, and the
    padding row is never touched (its params stay theta, its loss / hit columns stay zero)."""
    from tests.test_fl import small_cfg
    from qfedx_amd.data.datasets import build_federated_data
    from qfedx_amd.fl.adapters import make_adapter
    from qfedx_amd.fl.trainer import ShardStore, graph_bucket
    dev = torch.device("cuda", 0)
    cfg = small_cfg(n_qubits=10, n_layers=2, num_clients=7, samples_per_client=40, batch_size=8, local_epochs=2,
                    device="cuda", backend="hip", partition_type="non_iid", alpha=0.3)
    data = build_federated_data(cfg, clients=list(range(7)))
    ad = make_adapter(cfg, dev, "hip")
    assert ad.state_dtype == "mfma"
    sizes = [40, 23, 9, 40, 17, 30, 40]               # unequal shards: clients run 10, 6 and 8 steps
    store = ShardStore([(X[:n], y[:n]) for (X, y), n in zip(data.clients, sizes)], data.client_ids, dev)
    theta = ad.init_params(cfg.train.seed).to(dev)
    tr = ad.trainer
    local = [0, 1, 5]
    assert graph_bucket(len(local), len(store)) == 4
    steps = sorted({int(store.counts[i]) for i in local})
    assert len(steps) > 1                           # clients finish at different steps
    outs = {}
    for graphs in (True, False):
        tr.graphs = graphs
        outs[graphs] = []
        for r in range(3):                            # the graph is replayed twice; its outputs are static buffers
            rec = tr.run_round(store, local, theta, r)
            outs[graphs].append((rec["params"][: len(local)].clone(), rec["loss"][:, : len(local)].clone(),
                                 rec["correct"][:, : len(local)].clone()))
    for (pg, lg, cg), (pe, le, ce) in zip(outs[True], outs[False]):
        assert lg.shape[0] >= 3                       # several local steps
        assert torch.equal(pg, pe) and torch.equal(lg, le) and torch.equal(cg, ce)
    ent = next(reversed(tr._graph_cache.values()))
    p_pad, loss_pad, corr_pad = ent["out"][0][:3]        # graph variant 0's static outputs
    assert p_pad.shape[0] == 4
    assert torch.equal(p_pad[3], theta.float())
    assert not loss_pad[:, 3].any() and not corr_pad[:, 3].any()


def test_secagg_sparse_graph_in_fused_reduce_match_host_protocol(cuda):
    """SecAgg+ neighbour graph on the device: the mask kernel walks each client's compact neighbour table (width
    secagg_degree(N)) and the masked local sum is bitwise the host protocol's, dropped neighbours included."""
    from qfedx_amd.fl.aggregator import Aggregator
    from qfedx_amd.privacy.secure_agg import SecureAggregator
    K, P, N = 6, 257, 64
    g = torch.Generator().manual_seed(9)
    tk = torch.randn(K, P, generator=g) * 0.3
    tg = torch.randn(P, generator=g)
    w = torch.rand(K, generator=g).double() * 40 + 1
    ids = [3, 8, 11, 20, 29, 40]
    participants = sorted(set(ids) | {1, 2, 7, 9, 14, 25, 33, 38, 41, 47, 50, 52, 55, 58, 60, 63})
    dropped = [7, 25, 50]
    sa = SecureAggregator(123, graph="sparse")
    assert len(sa.neighbors(3, participants, 4)) < len(participants) - 1
    kw = dict(dp=False, seed=5, secure_agg=True, secagg=sa, num_clients=N)
    cpu = Aggregator(P, torch.zeros(P), "cpu", "torch", wrap=False, **kw)
    gpu = Aggregator(P, torch.zeros(P), cuda, "hip", wrap=False, **kw)
    a = cpu.local_reduce(tk, tg, w, 4, ids, participants=participants, dropped=dropped)
    b = gpu.local_reduce(tk.to(cuda), tg.to(cuda), w.to(cuda), 4, ids, participants=participants, dropped=dropped)
    m = (1 << sa.bits) - 1
    assert torch.equal(b.cpu() & m, a & m)


@pytest.mark.parametrize("K,bits,P", [(6, 48, 301), (7, 32, 301), (128, 48, 1037), (127, 32, 515)])
def test_secagg_pair_symmetric_masks_are_bitwise(cuda, K, bits, P):
    """Square full-graph table (one rank holds every client, row k = client k): the pair-symmetric mask kernel
    generates each pair's stream once for both clients.  Its masked local sum is bitwise the per-client kernel's and
    (small K) the host protocol's, with non-participants and dropped clients in the table, odd K (the round-robin
    bye) and P + 1 not a multiple of a workgroup's 8 Philox blocks."""
    from qfedx_amd.fl.aggregator import Aggregator
    from qfedx_amd.ops import fedavg_hip
    from qfedx_amd.privacy.secure_agg import SecureAggregator
    from qfedx_amd.utils.device import h2d
    g = torch.Generator().manual_seed(K)
    tk = torch.randn(K, P, generator=g) * 0.3
    tg = torch.randn(P, generator=g)
    w = torch.rand(K, generator=g).double() * 40 + 1
    ids = list(range(K))
    participants = [c for c in ids if c % 5 != 4]        # clients 4, 9, ... sit the round out
    dropped = [1, K - 2]
    sa = SecureAggregator(321, bits=bits, scale=2.0 ** 24 if bits > 32 else 2.0 ** 16)
    kw = dict(dp=False, seed=5, secure_agg=True, secagg=sa, num_clients=K)
    gpu = Aggregator(P, torch.zeros(P), cuda, "hip", wrap=False, **kw)
    seeds, sign = sa.round_tables(ids, participants, dropped, K, 3)
    tabs = (h2d(seeds, cuda), h2d(sign, cuda), h2d(torch.tensor([3], dtype=torch.int32), cuda))
    outs = []
    for pairsym in (False, True):
        out, _, _ = fedavg_hip.fused_local_reduce(
            tk.to(cuda), tg.to(cuda), w.to(cuda), torch.zeros(P, dtype=torch.uint8, device=cuda), ids, 3, 5,
            wrap=False, dp=False, clip_norm=1.0, noise_multiplier=0.0, secagg=(*tabs, sa.scale, sa.bits, pairsym))
        outs.append(out.cpu())
    m = (1 << sa.bits) - 1
    assert torch.equal(outs[0], outs[1])
    b = gpu.local_reduce(tk.to(cuda), tg.to(cuda), w.to(cuda), 3, ids, participants=participants, dropped=dropped)
    assert torch.equal(b.cpu(), outs[1])                 # the aggregator takes the pair-symmetric path itself
    if K <= 8:                                           # every client participates and survives: host protocol
        cpu = Aggregator(P, torch.zeros(P), "cpu", "torch", wrap=False, **kw)
        a = cpu.local_reduce(tk, tg, w, 3, ids, participants=ids, dropped=[])
        b = gpu.local_reduce(tk.to(cuda), tg.to(cuda), w.to(cuda), 3, ids, participants=ids, dropped=[])
        assert torch.equal(b.cpu() & m, a & m)


@pytest.mark.parametrize("dp,bits", [(False, 48), (True, 48), (False, 32), (True, 32)])
def test_secagg_masks_in_fused_reduce_match_host_protocol(cuda, dp, bits):
    """SecAgg on the device (K18): the fused FedAvg kernel masks every local client's ring element with the pairwise
    Philox masks itself.  Without DP the masked local sum is bitwise the host SecureAggregator's (mod 2^48),
    including the orphan-mask correction of dropped peers on and off this rank; with DP (and angle wrap) the decoded
    update matches to fixed-point resolution.  The round-apply kernel decodes the ring sum like finalize + apply.
    At bits <= 32 the device mask uses prg_mask's one-word-per-element layout (4 elements per Philox block)."""
    from qfedx_amd.fl.aggregator import Aggregator
    from qfedx_amd.ops._ext import ext
    from qfedx_amd.privacy.secure_agg import SecureAggregator
    K, P, N = 5, 301, 30
    g = torch.Generator().manual_seed(7)
    tk = torch.randn(K, P, generator=g) * 0.3
    tg = torch.randn(P, generator=g)
    w = torch.rand(K, generator=g).double() * 40 + 1
    mask = torch.zeros(P)
    if dp:
        mask[:100] = 1
    ids = [3, 8, 11, 20, 29]                      # this rank's surviving clients
    participants = [1, 2, 3, 7, 8, 11, 20, 25, 29]
    dropped = [7, 25]                             # 7 was local, 25 on another rank
    sa = SecureAggregator(123, bits=bits, scale=2.0 ** 24 if bits > 32 else 2.0 ** 16)
    kw = dict(dp=dp, clip_norm=0.9, noise_multiplier=0.7, seed=5, secure_agg=True, secagg=sa, num_clients=N)
    cpu = Aggregator(P, mask, "cpu", "torch", wrap=dp, **kw)
    gpu = Aggregator(P, mask, cuda, "hip", wrap=dp, **kw)
    a = cpu.local_reduce(tk, tg, w, 4, ids, participants=participants, dropped=dropped)
    b = gpu.local_reduce(tk.to(cuda), tg.to(cuda), w.to(cuda), 4, ids, participants=participants, dropped=dropped)
    m = (1 << sa.bits) - 1
    if not dp:
        assert torch.equal(b.cpu() & m, a & m)
    ma, wa = cpu.finalize(a)
    mb, wb = gpu.finalize(b.cpu())
    assert abs(float(wa) - float(wb)) < 1e-6
    assert torch.allclose(ma, mb, atol=4 / sa.scale)
    # the round-apply decode (SecAgg ring) == finalize + apply
    buf = torch.zeros(P + 6, dtype=torch.int64, device=cuda)
    buf[: P + 1] = b
    theta = tg.to(cuda).clone()
    out = torch.zeros(6, dtype=torch.float64, device=cuda)
    ext().round_apply(buf, P, theta, 1.0, out, sa.bits, sa.scale, 0)
    ref = gpu.apply(tg.to(cuda), mb.to(cuda), wsum=wb)
    assert torch.equal(theta, ref) and abs(out[5].item() - float(wb)) < 1e-12
    # single rank: the same reduce launch applies the ring sum itself (its last block, FusedApply) == round_apply
    buf2 = torch.zeros(P + 6, dtype=torch.int64, device=cuda)
    theta2 = tg.to(cuda).clone()
    out2 = torch.zeros(6, dtype=torch.float64, device=cuda)
    mets = [torch.zeros(4, device=cuda) for _ in range(4)]
    cnt = torch.zeros(1, dtype=torch.int32, device=cuda)
    gpu.local_reduce(tk.to(cuda), theta2, w.to(cuda), 4, ids, participants=participants, dropped=dropped,
                     out=buf2[: P + 1], pack=(buf2, *mets), apply=(theta2, out2, cnt, sa.bits, sa.scale, 0))
    assert torch.equal(theta2, theta) and out2[5].item() == out[5].item() and int(cnt.item()) == 0


def test_dp_client_norms_ride_in_round_buffer(cuda):
    """CC6 on the HIP fast path: the fused reduce's pack block scatters each client's pre-clip norm into the round
    all-reduce buffer and round_apply reads them back; round 1's norm quantiles match the CPU path's."""
    from tests.test_fl import small_cfg
    from qfedx_amd.api import run_experiment
    from qfedx_amd.parallel.dist import init_distributed
    kw = dict(num_rounds=2, dp=True, clip_norm=0.05, noise_multiplier=0.5, num_clients=5, deterministic_noise=True,
              optimizer="sgd", log_client_norms=True)
    cpu = run_experiment(small_cfg(**kw))
    dev = torch.device("cuda", 0)
    gpu = run_experiment(small_cfg(device="cuda", backend="hip", **kw), world=init_distributed(dev), device=dev,
                         backend="hip")
    hc, hg = cpu["history"][0], gpu["history"][0]
    for key in ("norm_p10", "norm_p50", "norm_p90"):
        assert abs(hc[key] - hg[key]) < 1e-3 * max(1.0, hc[key]), (key, hc[key], hg[key])
    assert all(0.0 <= h["clip_frac"] <= 1.0 for h in gpu["history"])


def test_fused_adam_in_grad_reduce_bitwise(cuda):
    """MFMA engine: the Adam step fused into hea_grad_reduce (the client's last block updates its row) gives bitwise
    the parameters, moments and step counters of the separate qfx_adam launch, over several steps with clients that
    drop out (active 0: row untouched, counter unchanged)."""
    from qfedx_amd.fl.optim import BatchedOptimizer
    from qfedx_amd.models.vqc import VQCSpec
    from qfedx_amd.ops.engine import VQCEngine
    spec = VQCSpec(n_qubits=12, n_layers=2, n_classes=3)
    eng = VQCEngine(spec, cuda, "hip", "mfma")
    assert getattr(eng.hip, "fuses_optimizer", False)
    K, B = 5, 8
    g = torch.Generator().manual_seed(7)
    xs = [spec.encode_features(torch.rand(K, B, 12, generator=g)).to(cuda) for _ in range(3)]
    ys = [torch.randint(0, 3, (K, B), generator=g).to(cuda) for _ in range(3)]
    w = torch.full((K, B), 1.0 / B, device=cuda)
    acts = [torch.tensor(a, dtype=torch.float32, device=cuda) for a in ([1, 1, 1, 1, 1], [1, 0, 1, 1, 0], [0, 0, 1, 1, 0])]
    p0 = torch.stack([spec.init_params(k) for k in range(K)]).to(cuda)
    outs = []
    for fused in (False, True):
        p = p0.clone()
        opt = BatchedOptimizer("adam", p.shape, cuda, 0.05, backend="hip")
        grads = []
        for s in range(3):
            res = eng.loss_and_grads(xs[s], ys[s], w, p, "adjoint", fused_opt=(opt, acts[s]) if fused else None)
            assert res.get("opt_done", False) == fused
            if not fused:
                opt.step(p, res["grad"], acts[s])
            grads.append(res["grad"].clone())
        torch.cuda.synchronize()
        outs.append((p, opt.m, opt.v, opt.t, grads))
    (pa, ma, va, ta, ga), (pb, mb, vb, tb, gb) = outs
    for a, b in zip(ga, gb):
        assert torch.equal(a, b)
    assert torch.equal(pa, pb) and torch.equal(ma, mb) and torch.equal(va, vb) and torch.equal(ta, tb)
    assert ta.tolist() == [2, 1, 3, 3, 1]
    assert not torch.equal(pa[0], p0[0]) and torch.equal(pa[1], pb[1])


def test_secagg_sparse_federated_hip_run_matches_plain(cuda):
    """the end-to-end sparse (SecAgg+) path on the HIP round graph - server round_tables -> device mask
    kernel -> fused reduce with the single-rank FusedApply - with 20 clients (a true circulant graph: degree 10 < 19)
    and dropouts decodes to the plain HIP aggregate; a round whose dropouts would isolate a survivor is aborted."""
    from tests.test_fl import small_cfg
    from qfedx_amd.api import run_experiment
    from qfedx_amd.parallel.dist import init_distributed
    from qfedx_amd.privacy.secure_agg import SecureAggregator
    assert len(SecureAggregator(0, graph="sparse").neighbors(0, range(20), 0)) < 19
    dev = torch.device("cuda", 0)
    kw = dict(num_rounds=1, n_qubits=6, num_clients=20, samples_per_client=16, dropout_prob=0.2, device="cuda",
              backend="hip")
    plain = run_experiment(small_cfg(**kw), world=init_distributed(dev), device=dev, backend="hip")
    sec = run_experiment(small_cfg(secure_agg=True, secagg_graph="sparse", **kw), world=init_distributed(dev),
                         device=dev, backend="hip")
    assert sec["history"][0]["dropped"] > 0 and not sec["history"][0]["secagg_aborted"]
    assert torch.allclose(plain["params"].cpu(), sec["params"].cpu(), atol=1e-5)


@pytest.mark.parametrize("scale", [None, 0.25])
def test_fused_reduce_dp_noise_scale_matches_host(cuda, scale):
    """Distributed DP on the device: the fused reduce multiplies each client's noise std by its dp_scale entry
    (uploaded per round); the decoded update matches the torch reference clip_and_noise(scale_k) to fixed point."""
    from qfedx_amd.fl.aggregator import Aggregator
    K, P = 6, 513
    g = torch.Generator().manual_seed(3)
    tk = torch.randn(K, P, generator=g) * 0.3
    tg = torch.randn(P, generator=g)
    w = torch.ones(K, dtype=torch.float64)
    ids = [0, 3, 4, 7, 9, 12]
    kw = dict(dp=True, clip_norm=0.8, noise_multiplier=1.3, seed=21)
    cpu = Aggregator(P, torch.zeros(P), "cpu", "torch", wrap=False, **kw)
    gpu = Aggregator(P, torch.zeros(P), cuda, "hip", wrap=False, **kw)
    a = cpu.local_reduce(tk, tg, w, 2, ids, dp_scale=scale)
    tab = None if scale is None else torch.full((K,), scale, dtype=torch.float32, device=cuda)
    b = gpu.local_reduce(tk.to(cuda), tg.to(cuda), w.to(cuda), 2, ids, dp_scale=tab)
    ma, _ = cpu.finalize(a)
    mb, _ = gpu.finalize(b.cpu())
    assert torch.allclose(ma, mb, atol=1e-6)
    if scale is not None:                       # and it is not the unscaled noise
        full = gpu.finalize(gpu.local_reduce(tk.to(cuda), tg.to(cuda), w.to(cuda), 2, ids).cpu())[0]
        assert not torch.allclose(full, mb, atol=1e-3)


def test_prologue_fragments_match_per_client_fragments(cuda, monkeypatch):
    """The MFMA engine's first local step reads ONE fragment set built from theta by the round prologue launch
    (hea_frag.h; every client row starts as theta) instead of the per-client fragment launch: the federated run is
    bitwise the run with the prologue job disabled, over rounds of several local steps (later steps build
    per-client fragments from the updated rows), graph-captured and eager."""
    from tests.test_fl import small_cfg
    from qfedx_amd.api import run_experiment
    from qfedx_amd.ops.engine import VQCEngine
    from qfedx_amd.parallel.dist import init_distributed
    outs = []
    for on in (True, False):
        if not on:
            monkeypatch.setattr(VQCEngine, "prologue_frag_job", lambda self: None)
        cfg = small_cfg(num_rounds=3, n_qubits=12, n_layers=3, device="cuda", backend="hip", num_clients=5,
                        local_epochs=2, state_dtype="mfma")
        dev = torch.device("cuda", 0)
        outs.append(run_experiment(cfg, world=init_distributed(dev), device=dev, backend="hip"))
    assert torch.equal(outs[0]["params"], outs[1]["params"])
    assert torch.equal(torch.tensor(outs[0]["accuracies"]), torch.tensor(outs[1]["accuracies"]))


@pytest.mark.parametrize("kw", [dict(local_epochs=2), dict(local_steps=1, weighting="uniform")])
def test_fedavg_tail_in_adam_epilogue_is_bitwise(cuda, monkeypatch, kw):
    """Plain FedAvg folded into the MFMA engine's fused Adam epilogue of the round's last local step (QfxFedTail:
    the same fixed-point terms added with int64 atomics into the buffer head the prologue zeroed, metrics packed and
    the single-rank round applied by the last client) gives bitwise the run with the separate FedAvg launch: global
    parameters, accuracies and the round losses, eager and graph-captured rounds alike."""
    from tests.test_fl import small_cfg
    from qfedx_amd.api import run_experiment
    from qfedx_amd.parallel.dist import init_distributed
    from qfedx_amd.ops.hea_mfma import HeaMfmaProgram
    orig = HeaMfmaProgram.loss_and_grads
    fused = {"1": 0, "0": 0}
    mode = ["1"]

    def spy(self, *a, **k):          # the knob-on run must actually take the fused path
        res = orig(self, *a, **k)
        fused[mode[0]] += int(bool(res.get("fed_done")))
        return res
    monkeypatch.setattr(HeaMfmaProgram, "loss_and_grads", spy)
    outs = []
    for on in ("1", "0"):
        mode[0] = on
        monkeypatch.setenv("QFEDX_FED_TAIL", on)
        cfg = small_cfg(num_rounds=4, n_qubits=12, n_layers=3, device="cuda", backend="hip", num_clients=6,
                        state_dtype="mfma", **kw)
        dev = torch.device("cuda", 0)
        outs.append(run_experiment(cfg, world=init_distributed(dev), device=dev, backend="hip"))
    assert fused["1"] >= 1 and fused["0"] == 0, fused      # the fused FedAvg tail ran (graph replays skip Python)
    assert torch.equal(outs[0]["params"], outs[1]["params"])
    assert torch.equal(torch.tensor(outs[0]["accuracies"]), torch.tensor(outs[1]["accuracies"]))
    l0 = [h.get("train_loss") for h in outs[0]["history"]]
    l1 = [h.get("train_loss") for h in outs[1]["history"]]
    assert l0 == l1
