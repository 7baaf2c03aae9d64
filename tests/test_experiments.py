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
