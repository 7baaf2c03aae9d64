"""Configs, CLI, experiment grid + report (ROADMAP.md:102-121)."""
import glob
import json
import os

import pytest

from qfedx_amd.cli import main as cli_main
from qfedx_amd.config import load_config
from qfedx_amd.experiments import aggregate, expand_grid, run_grid, write_report

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.parametrize("path", sorted(glob.glob(os.path.join(ROOT, "configs", "*.yaml"))))
def test_every_config_file_loads(path):
    if os.path.basename(path).startswith("grid_"):
        import yaml
        spec = yaml.safe_load(open(path))
        assert expand_grid(spec)
    else:
        cfg = load_config(path)
        assert cfg.name and cfg.model.kind in ("vqc", "tinycnn")


def test_expand_grid_cartesian_times_seeds():
    runs = expand_grid({"grid": {"a.b": [1, 2], "c.d": ["x", "y", "z"]}, "seeds": [0, 1], "fixed": {"e.f": 3}})
    assert len(runs) == 12 and all(r["overrides"]["e.f"] == 3 for r in runs)


def test_grid_run_resume_and_report(tmp_path):
    spec = {"base": {"data.dataset": "iris", "data.num_clients": 2, "model.n_qubits": 4, "model.n_layers": 1,
                     "train.num_rounds": 2, "train.batch_size": 16, "runtime.device": "cpu", "runtime.log_every": 100},
            "seeds": [0, 1], "grid": {"privacy.dp": [False, True]}}
    out = str(tmp_path / "g")
    res = run_grid(spec, out)
    assert len(res) == 4
    again = run_grid(spec, out)                  # resumes: nothing left to run
    assert again == []
    rows = aggregate([json.loads(x) for x in open(os.path.join(out, "results.jsonl"))])
    assert len(rows) == 2 and all(r["n_seeds"] == 2 for r in rows)
    dp_row = [r for r in rows if r["overrides"]["privacy.dp"]][0]
    assert dp_row["epsilon_mean"] > 0 and dp_row["comm_mb_per_round_mean"] > 0
    rep = write_report(os.path.join(out, "results.jsonl"))
    assert "acc (mean±std)" in rep["markdown"] and os.path.exists(os.path.join(out, "report.md"))


def test_cli_run_prints_summary(capsys):
    rc = cli_main(["run", "data.dataset=iris", "data.num_clients=2", "train.num_rounds=1", "runtime.device=cpu",
                   "runtime.log_every=100"])
    assert rc == 0
    line = [l for l in capsys.readouterr().out.splitlines() if l.startswith("{")][-1]
    out = json.loads(line)
    assert len(out["accuracies"]) == 2 and out["backend"] == "torch"


def test_mlflow_file_store_tracking(tmp_path):
    """ROADMAP.md:92-93: per-experiment config, metrics, checkpoints and artifacts in the MLflow file-store
    layout (written without the mlflow package)."""
    import glob
    import os
    import yaml
    from qfedx_amd.api import run_experiment
    from qfedx_amd.utils.tracking import FINISHED, read_metric
    from tests.test_fl import small_cfg
    root = tmp_path / "mlruns"
    run_experiment(small_cfg(num_rounds=3, tracking_dir=str(root), experiment="unit", checkpoint_every=1,
                             checkpoint_dir=str(tmp_path / "ck")))
    exp = glob.glob(str(root / "*" / "meta.yaml"))
    assert len(exp) == 1 and yaml.safe_load(open(exp[0]))["name"] == "unit"
    runs = [d for d in glob.glob(str(root / "*" / "*")) if os.path.isdir(d)]
    assert len(runs) == 1
    run = runs[0]
    meta = yaml.safe_load(open(os.path.join(run, "meta.yaml")))
    assert meta["status"] == FINISHED and meta["end_time"] >= meta["start_time"]
    assert open(os.path.join(run, "params", "train.num_rounds")).read() == "3"
    acc = read_metric(run, "test_acc")
    assert [s for _, _, s in acc] == [0, 1, 2, 3] and all(0.0 <= v <= 1.0 for _, v, _ in acc)
    assert len(glob.glob(os.path.join(run, "artifacts", "checkpoints", "round_*.pt"))) == 3
    assert yaml.safe_load(open(os.path.join(run, "artifacts", "config.yaml")))["train"]["num_rounds"] == 3


def test_roadmap_digits_grid_has_baselines_and_alpha_axis(tmp_path):
    """Reduced ROADMAP.md:102-116 model-comparison grid: VQC on PCA features across the Dirichlet alpha axis, the
    classical FL TinyCNN under the same DP, and the centralized-VQC baseline, all in one report table."""
    import yaml
    spec = yaml.safe_load(open(os.path.join(ROOT, "configs", "grid_roadmap_digits.yaml")))
    spec["seeds"] = [0]
    spec["fixed"] = {"train.num_rounds": 1, "runtime.device": "cpu", "runtime.log_every": 100}
    spec["grid"] = {"model.n_qubits": [4], "privacy.dp": [True], "data.alpha": [0.1, 1.0]}
    spec["extra"] = [e for e in spec["extra"] if e.get("privacy.dp")]
    out = str(tmp_path / "g")
    res = run_grid(spec, out)
    kinds = {(r["config"]["model"]["kind"], r["config"]["train"]["mode"]) for r in res}
    assert kinds == {("vqc", "federated"), ("tinycnn", "federated"), ("vqc", "centralized")}
    assert {r["config"]["data"]["alpha"] for r in res if r["config"]["model"]["kind"] == "vqc"} >= {0.1, 1.0}
    assert all(r["epsilon"] and r["epsilon"] > 0 for r in res)
    rep = write_report(os.path.join(out, "results.jsonl"))
    assert "tinycnn" in rep["markdown"] and "centralized" in rep["markdown"] and "alpha" in rep["markdown"]


def test_centralized_mode_pools_every_shard_into_one_client():
    from qfedx_amd.config import ExperimentConfig, apply_overrides
    from qfedx_amd.data.datasets import build_federated_data
    cfg = ExperimentConfig()
    apply_overrides(cfg, ["data.dataset=iris", "data.num_clients=3", "model.n_qubits=4"])
    fed = build_federated_data(cfg)
    cfg.train.mode = "centralized"
    cen = build_federated_data(cfg, clients=[0])
    assert cen.num_clients == 1 and cen.client_ids == [0] and len(cen.clients) == 1
    assert cen.clients[0][1].shape[0] == sum(fed.sizes())
    assert build_federated_data(cfg, clients=[]).clients == []


def test_noise_grid_runs_exact_amplitude_damping(tmp_path):
    """configs/grid_noise.yaml: noise.kind=amplitude runs EXACT amplitude damping on the density-matrix simulator,
    amplitude_twirl its Pauli twirl on statevector trajectories (ROADMAP.md:66-73)."""
    import yaml
    spec = yaml.safe_load(open(os.path.join(ROOT, "configs", "grid_noise.yaml")))
    spec["base"] = os.path.join(ROOT, "configs", spec["base"])
    spec["seeds"] = [0]
    spec["fixed"] = {"train.num_rounds": 1, "runtime.device": "cpu", "runtime.log_every": 100}
    res = run_grid(spec, str(tmp_path / "g"))
    sim = {r["config"]["noise"]["kind"]: r["simulator"] for r in res}
    assert sim["amplitude"] == "density" and sim["amplitude_twirl"] == "statevector"
    assert sim["none"] == "statevector" and sim["depolarizing"] == "statevector"
    assert all(r["final_loss"] == r["final_loss"] for r in res)       # finite
