"""Federated runtime: FedAvg parity, aggregation, training progress, checkpoint/resume, config."""
import copy
import os

import numpy as np
import pytest
import torch

from qfedx_amd.api import run_experiment
from qfedx_amd.config import ExperimentConfig, apply_overrides, load_config, save_config
from qfedx_amd.fl.aggregator import Aggregator, federated_averaging, wrap_angles
from qfedx_amd.fl.server import sample_dropouts, sample_participants
from qfedx_amd.fl.trainer import BatchPlan


def small_cfg(**kw) -> ExperimentConfig:
    cfg = ExperimentConfig()
    cfg.data.num_clients = 4
    cfg.data.samples_per_client = 48
    cfg.data.test_samples = 128
    cfg.data.partition_type = "non_iid"
    cfg.model.n_qubits = 4
    cfg.model.n_layers = 2
    cfg.model.readout_scale = 3.0
    cfg.train.num_rounds = 4
    cfg.train.batch_size = 16
    cfg.train.learning_rate = 0.1
    cfg.runtime.device = "cpu"
    cfg.runtime.log_every = 100
    apply_overrides(cfg, [f"{k}={v}" for k, v in kw.items()])
    return cfg


def test_federated_averaging_reference_formula():
    a = {"w": torch.tensor([1.0, 2.0]), "n": torch.tensor(3)}
    b = {"w": torch.tensor([3.0, 6.0]), "n": torch.tensor(5)}
    out = federated_averaging([(a, 1), (b, 3)])
    assert torch.allclose(out["w"], torch.tensor([2.5, 5.0]))
    assert out["n"].item() == 3          # integer buffers no longer break


def test_aggregator_reconstructs_weighted_mean_update():
    """ROADMAP.md:42 - the aggregator reconstructs the (weighted) mean update."""
    P = 12
    tg = torch.randn(P)
    tk = tg + torch.randn(3, P) * 0.1
    w = torch.tensor([1.0, 2.0, 3.0], dtype=torch.float64)
    agg = Aggregator(P, torch.ones(P), "cpu", wrap=True)
    red = agg.local_reduce(tk, tg, w, 0, [0, 1, 2])
    mean, ws = agg.finalize(red)
    ref = ((tk - tg).double() * w[:, None]).sum(0) / w.sum()
    assert torch.allclose(mean, ref, atol=1e-9) and ws == 6.0


def test_angle_wrap():
    d = torch.tensor([3.5, -3.5, 0.1, 6.2])
    wr = wrap_angles(d)
    assert torch.all(wr >= -np.pi) and torch.all(wr < np.pi)
    assert torch.allclose(torch.cos(wr), torch.cos(d), atol=1e-6)


def test_sampling_and_dropouts_deterministic():
    a = sample_participants(100, 0.3, seed=1, round_num=5)
    assert a == sample_participants(100, 0.3, seed=1, round_num=5) and len(a) == 30
    assert sample_participants(10, 1.0, 0, 0) == list(range(10))
    d = sample_dropouts(list(range(200)), 0.25, seed=2, round_num=1)
    assert 20 < len(d) < 80


def test_batch_plan_epoch_semantics():
    counts = torch.tensor([10, 33])
    plan = BatchPlan(counts, [0, 1], batch_size=8, round_num=0, seed=0, local_epochs=2)
    assert plan.steps_per_client == [4, 10]          # epochs * ceil(n / B), like len(dataloader)
    seen = plan.idx[: plan.steps_per_client[1] // 2, 1][plan.wts[: plan.steps_per_client[1] // 2, 1] > 0]
    assert sorted(seen.tolist()) == list(range(33))  # one epoch covers each sample exactly once
    assert float(plan.wts[3, 0].sum()) == pytest.approx(1.0)   # partial batch re-normalised


def test_global_model_beats_round0():
    """ROADMAP.md:43 - the global model improves on held-out data vs round 0."""
    out = run_experiment(small_cfg(num_rounds=6))
    assert out["accuracies"][-1] > out["accuracies"][0] + 0.1


def test_dp_secagg_dropout_run_and_epsilon():
    cfg = small_cfg(dp=True, secure_agg=True, clip_norm=0.5, noise_multiplier=0.5, dropout_prob=0.25,
                    client_fraction=0.75)
    out = run_experiment(cfg)
    assert out["epsilon"] is not None and out["epsilon"] > 0
    eps = [h["epsilon"] for h in out["history"]]
    assert all(a <= b for a, b in zip(eps, eps[1:]))


def test_secagg_equals_plain_aggregation():
    # one round: local training is identical; SecAgg's 2^-24 ring rounding differs from the exact
    # 2^-32 path by ~1e-8 (over several rounds Adam amplifies such noise on zero-gradient angles)
    plain = run_experiment(small_cfg(num_rounds=1))
    sec = run_experiment(small_cfg(num_rounds=1, secure_agg=True))
    assert torch.allclose(plain["params"], sec["params"], atol=1e-5)


@pytest.mark.parametrize("method,opt", [("param_shift", "adam"), ("adjoint", "sgd"), ("adjoint", "spsa")])
def test_gradient_methods_train(method, opt):
    out = run_experiment(small_cfg(num_rounds=2, grad_method=method, optimizer=opt))
    assert np.isfinite(out["accuracies"][-1])


@pytest.mark.parametrize("server", [{}, {"server_optimizer": "momentum", "server_lr": 0.5},
                                    {"server_optimizer": "adam", "server_lr": 0.3}])
def test_checkpoint_resume_matches_uninterrupted(tmp_path, server):
    """Resume reproduces the uninterrupted run, including the server optimizer's moments."""
    full = run_experiment(small_cfg(num_rounds=4, **server))
    cfg = small_cfg(num_rounds=2, checkpoint_every=1, checkpoint_dir=str(tmp_path / "ck"), **server)
    run_experiment(cfg)
    cfg2 = small_cfg(num_rounds=4, checkpoint_every=1, checkpoint_dir=str(tmp_path / "ck"), resume=True, **server)
    resumed = run_experiment(cfg2)
    assert torch.equal(full["params"], resumed["params"])
    ck = torch.load(sorted((tmp_path / "ck").glob("round_*.pt"))[-1], weights_only=True)
    assert set(ck["global_state"]) == {"theta", "readout.a", "readout.b"}
    if server:
        st = ck["server_state"]
        assert st["kind"] == server["server_optimizer"] and int(st["t"]) == 4
        assert st["m"].shape == (full["params"].numel(),) and st["m"].abs().sum() > 0
    else:
        assert "server_state" not in ck


def test_resume_refuses_checkpoint_without_server_state(tmp_path):
    run_experiment(small_cfg(num_rounds=1, checkpoint_every=1, checkpoint_dir=str(tmp_path / "ck")))
    with pytest.raises(ValueError, match="server_state"):
        run_experiment(small_cfg(num_rounds=2, checkpoint_every=1, checkpoint_dir=str(tmp_path / "ck"),
                                 resume=True, server_optimizer="adam"))


def test_dp_noise_is_keyed_by_a_run_secret(tmp_path):
    """DP noise is not reproducible from the public config/checkpoint: two runs with the same
    train.seed differ, and nothing written to disk holds the key; deterministic_noise=True restores
    reproducibility for tests."""
    kw = dict(num_rounds=2, dp=True, noise_multiplier=0.5)
    a = run_experiment(small_cfg(**kw, checkpoint_every=1, checkpoint_dir=str(tmp_path / "a"),
                                 metrics_path=str(tmp_path / "m.jsonl")))
    b = run_experiment(small_cfg(**kw))
    assert not torch.equal(a["params"], b["params"])
    c = run_experiment(small_cfg(**kw, deterministic_noise=True))
    d = run_experiment(small_cfg(**kw, deterministic_noise=True))
    assert torch.equal(c["params"], d["params"])
    ck = torch.load(sorted((tmp_path / "a").glob("round_*.pt"))[-1], weights_only=True)
    assert not any("noise" in k for k in ck) and "noise_seed" not in open(tmp_path / "m.jsonl").read()


def test_poisson_sampling_under_dp():
    sizes = [len(sample_participants(200, 0.1, 7, r, poisson=True)) for r in range(200)]
    assert 17 < float(np.mean(sizes)) < 23 and len(set(sizes)) > 5        # Bernoulli(q), variable size
    assert sample_participants(200, 0.1, 7, 3, poisson=True) == sample_participants(200, 0.1, 7, 3, poisson=True)
    # DP defaults to Poisson and accounts at q = client_fraction; fixed-size sampling is accounted with q = 1
    pois = run_experiment(small_cfg(num_rounds=2, dp=True, client_fraction=0.5, num_clients=8))
    fixed = run_experiment(small_cfg(num_rounds=2, dp=True, client_fraction=0.5, num_clients=8, sampling="fixed"))
    from qfedx_amd.privacy.accountant import epsilon
    assert pois["epsilon"] == pytest.approx(epsilon(0.5, 1.0, 2, 1e-5), rel=1e-9)
    assert fixed["epsilon"] == pytest.approx(epsilon(1.0, 1.0, 2, 1e-5), rel=1e-9)
    assert fixed["epsilon"] > pois["epsilon"]


def test_config_yaml_and_overrides(tmp_path):
    cfg = small_cfg()
    p = str(tmp_path / "c.yaml")
    save_config(cfg, p)
    back = load_config(p, ["num_rounds=9", "model.n_qubits=6", "digits=[3,5]"])
    assert back.train.num_rounds == 9 and back.model.n_qubits == 6 and back.data.digits == (3, 5)
    flat = tmp_path / "flat.yaml"
    flat.write_text("num_clients: 7\nlearning_rate: 0.2\npartition_type: non_iid\n")
    f = load_config(str(flat))
    assert f.data.num_clients == 7 and f.train.learning_rate == 0.2
    with pytest.raises(KeyError):
        apply_overrides(copy.deepcopy(cfg), ["nonsense=1"])


def test_metrics_jsonl(tmp_path):
    from qfedx_amd.utils.logging import read_jsonl
    path = str(tmp_path / "m.jsonl")
    run_experiment(small_cfg(num_rounds=2, metrics_path=path))
    recs = read_jsonl(path)
    rounds = [r for r in recs if "round" in r]
    assert recs[0]["event"] == "config" and rounds[-1]["round"] == 2 and "test_acc" in rounds[-1]
    assert recs[-1].get("final") and 0.0 <= recs[-1]["test_auc"] <= 1.0


from hypothesis import given, settings, strategies as st  # noqa: E402


@settings(max_examples=30, deadline=None)
@given(st.integers(2, 9), st.integers(0, 2 ** 31 - 1), st.integers(1, 8))
def test_exact_aggregation_permutation_and_split_invariant(K, seed, split):
    """Fixed-point FedAvg: the aggregate is bitwise identical for any client order and any split of
    the clients over ranks (the property that makes results independent of the GPU count)."""
    g = torch.Generator().manual_seed(seed)
    P = 17
    tg = torch.randn(P, generator=g)
    tk = tg + torch.randn(K, P, generator=g) * 0.3
    w = torch.rand(K, generator=g, dtype=torch.float64) * 10 + 0.1
    ids = list(range(K))
    agg = Aggregator(P, torch.ones(P), "cpu", wrap=True)
    full = agg.local_reduce(tk, tg, w, 0, ids)
    perm = torch.randperm(K, generator=g)
    permuted = agg.local_reduce(tk[perm], tg, w[perm], 0, [ids[i] for i in perm.tolist()])
    cut = split % K
    parts = agg.local_reduce(tk[:cut], tg, w[:cut], 0, ids[:cut]) if cut else torch.zeros_like(full)
    parts = parts + agg.local_reduce(tk[cut:], tg, w[cut:], 0, ids[cut:])
    assert torch.equal(full, permuted) and torch.equal(full, parts)


@pytest.mark.parametrize("opt", ["momentum", "adam"])
def test_server_optimizers_train(opt):
    out = run_experiment(small_cfg(num_rounds=5, server_optimizer=opt, server_lr=0.1 if opt == "adam" else 1.0))
    assert max(out["accuracies"][1:]) > out["accuracies"][0] + 0.05


def test_sharded_fedavg_step_equals_plain_path():
    from qfedx_amd.parallel.dist import ShardedServerState, World
    # local SGD: Adam would amplify the 1e-12 lr offset on the zero-gradient angles
    plain = run_experiment(small_cfg(num_rounds=3, optimizer="sgd"))
    # a FedAvg "server optimizer" with lr 1 through the sharded reduce-scatter/all-gather path
    sharded = run_experiment(small_cfg(num_rounds=3, optimizer="sgd", server_optimizer="fedavg",
                                       server_lr=1.0 + 1e-12))
    assert torch.allclose(plain["params"], sharded["params"], atol=1e-6)


@pytest.mark.parametrize("local_epochs,local_steps,shuffle", [(1, 0, True), (3, 0, True), (2, 0, False),
                                                                (1, 7, True), (1, 40, True)])
def test_native_batch_plan_matches_torch_oracle(local_epochs, local_steps, shuffle):
    """csrc/runtime.cpp builds the same keyed plan tables as the torch oracle (bitwise)."""
    pytest.importorskip("qfedx_amd._qfedx_C", reason="native extension not built")
    counts = torch.tensor([0, 1, 5, 33, 64, 17, 100, 31])
    ids = [3, 17, 2, 40, 1 << 33, 9, 11, 5]
    for r in (0, 7):
        a = BatchPlan(counts, ids, 16, r, 1234, local_epochs, local_steps, shuffle, native=True)
        b = BatchPlan(counts, ids, 16, r, 1234, local_epochs, local_steps, shuffle, native=False)
        assert a.steps_per_client == b.steps_per_client and a.max_steps == b.max_steps
        assert torch.equal(a.idx, b.idx) and torch.equal(a.wts, b.wts) and torch.equal(a.active, b.active)


def test_graph_bucket_and_client_padding():
    """Poisson client sampling varies the per-rank client count; the hipGraph path pads to a few buckets
    with inactive weight-0 rows (trainer.graph_bucket / _pad_clients)."""
    from qfedx_amd.fl.trainer import _pad_clients, graph_bucket
    assert [graph_bucket(k, 64) for k in (1, 2, 3, 5, 8, 9, 16, 17, 31)] == [1, 2, 4, 8, 8, 16, 16, 24, 32]
    assert graph_bucket(5, 6) == 6 and graph_bucket(7, 7) == 7 and graph_bucket(0, 4) == 0
    assert len({graph_bucket(k, 64) for k in range(20, 45)}) == 4      # Binomial(64, .5) bulk -> 4 shapes
    S, K, B = 2, 3, 4
    tabs = {"lid": torch.tensor([5, 1, 2]), "idx": torch.randint(0, 9, (S, K, B)), "wts": torch.rand(S, K, B),
            "act": torch.ones(S, K), "nvalid": torch.full((S, K), 4.0), "w": torch.tensor([3.0, 4.0, 5.0]).double()}
    out = _pad_clients(tabs, 8)
    assert out["lid"].tolist() == [5, 1, 2, 5, 5, 5, 5, 5]
    assert out["idx"].shape == (S, 8, B) and torch.equal(out["idx"][:, :K], tabs["idx"])
    for key in ("wts", "act", "nvalid"):
        assert torch.equal(out[key][:, :K], tabs[key]) and not out[key][:, K:].any()
    assert out["w"].tolist() == [3.0, 4.0, 5.0, 0, 0, 0, 0, 0] and out["w"].dtype == torch.float64
    assert _pad_clients(tabs, 3) is tabs


def test_trainer_epilogue_and_extra_tables():
    """The trainer runs a device epilogue right after the local steps on the trained params, with the round's
    tables (plus caller-provided per-client ``extra`` tables); the server's fused FedAvg uses this hook."""
    from qfedx_amd.api import setup
    from qfedx_amd.data.datasets import build_federated_data
    from qfedx_amd.fl.adapters import make_adapter
    from qfedx_amd.fl.trainer import ShardStore
    cfg = small_cfg(num_clients=3)
    device, backend, world = setup(cfg)
    data = build_federated_data(cfg)
    adapter = make_adapter(cfg, device, backend)
    store = ShardStore(data.clients, data.client_ids, device)
    theta = adapter.init_params(0)
    seen = {}

    def epi(params, tabs, th):
        seen.update(params=params.clone(), keys=tabs["dpkeys"].clone(), loss=tabs["loss"].clone(), theta=th)

    keys = torch.arange(4, dtype=torch.int32).reshape(2, 2)
    res = adapter.trainer.run_round(store, [0, 2], theta, 0, epilogue=epi, extra={"dpkeys": keys})
    assert torch.equal(seen["params"], res["params"]) and torch.equal(seen["keys"], keys)
    assert torch.equal(seen["loss"], res["loss"]) and torch.equal(seen["theta"], theta)
    with pytest.raises(ValueError):
        adapter.trainer.run_round(store, [0, 2], theta, 0, extra={"w": torch.ones(2)})


def test_dp_rounds_log_client_norms_and_clip_fraction():
    """CC6 (opt-in, non-private diagnostic): under DP with runtime.log_client_norms every round record carries the clip
    fraction and norm quantiles of the participating clients' pre-clip update norms (gathered through the round's
    all-reduce buffer), flagged norms_private=False; off by default."""
    cfg = small_cfg(num_rounds=3, dp=True, clip_norm=0.05, noise_multiplier=0.5, num_clients=5, client_fraction=1.0,
                    deterministic_noise=True, log_client_norms=True)
    out = run_experiment(cfg)
    for h in out["history"]:
        assert 0.0 <= h["clip_frac"] <= 1.0 and h["norm_p10"] <= h["norm_p50"] <= h["norm_p90"]
    assert out["history"][0]["norm_p50"] > 0
    assert all(h["norms_private"] is False for h in out["history"])
    cfg2 = small_cfg(num_rounds=1, dp=True, num_clients=3)
    assert "clip_frac" not in run_experiment(cfg2)["history"][0]
