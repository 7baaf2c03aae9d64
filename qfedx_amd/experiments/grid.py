"""Grid runner (ROADMAP.md:102-109).

A grid spec (YAML)::

    base: configs/iris_4q.yaml        # or an inline mapping of config keys
    seeds: [0, 1, 2]
    grid:                             # cartesian product of override lists
      model.n_qubits: [2, 4, 8]
      privacy.noise_multiplier: [0.5, 1.0, 2.0]
    fixed: {privacy.dp: true}         # overrides applied to every run
    extra:                            # single runs beside the product (baselines), with ``fixed`` and seeds
      - {train.mode: centralized}

Every run is one ``run_experiment`` in this process (or under ``torchrun`` - all ranks execute the
grid in lockstep); rank 0 appends one summary line per run to ``<out>/results.jsonl`` and the
report is built from that file, so an interrupted grid resumes where it stopped.
"""
from __future__ import annotations

import copy
import itertools
import json
import os
from typing import Optional

import yaml

from ..config import ExperimentConfig, apply_overrides, load_config


def expand_grid(spec: dict) -> list[dict]:
    """-> list of {"overrides": {key: value}, "seed": s} in a stable order."""
    grid = spec.get("grid", {}) or {}
    keys = list(grid)
    combos = list(itertools.product(*[grid[k] for k in keys])) if keys else [()]
    seeds = spec.get("seeds", [spec.get("seed", 42)])
    fixed = spec.get("fixed", {}) or {}
    runs = []
    for combo in combos:
        ov = dict(fixed)
        ov.update(dict(zip(keys, combo)))
        for s in seeds:
            runs.append({"overrides": ov, "seed": int(s)})
    for extra in spec.get("extra", []) or []:
        ov = dict(fixed)
        ov.update(extra)
        for s in seeds:
            runs.append({"overrides": ov, "seed": int(s)})
    return runs


def _fmt(v) -> str:
    if isinstance(v, (list, tuple)):
        return "[" + ",".join(str(x) for x in v) + "]"
    return str(v)


def build_config(spec: dict, run: dict, base_dir: str = ".") -> ExperimentConfig:
    base = spec.get("base")
    if isinstance(base, str):
        cfg = load_config(base if os.path.isabs(base) else os.path.join(base_dir, base))
    else:
        cfg = ExperimentConfig()
        if isinstance(base, dict):
            apply_overrides(cfg, [f"{k}={_fmt(v)}" for k, v in base.items()])
    apply_overrides(cfg, [f"{k}={_fmt(v)}" for k, v in run["overrides"].items()] + [f"train.seed={run['seed']}"])
    return cfg


def run_key(run: dict) -> str:
    return json.dumps({"overrides": run["overrides"], "seed": run["seed"]}, sort_keys=True)


def summarize_run(cfg: ExperimentConfig, out: dict, run: Optional[dict] = None) -> dict:
    hist = out.get("history", [])
    accs = out.get("accuracies", [])
    P = int(out["params"].numel()) if "params" in out else 0
    parts = [h.get("participants", 0) - h.get("dropped", 0) for h in hist]
    up = sum(p * P * 4 for p in parts)                       # client -> server updates (fp32)
    down = sum(h.get("participants", 0) * P * 4 for h in hist)  # server -> client model broadcast
    n = max(len(hist), 1)
    ws = int(out.get("world_size", 1))
    rec = {
        "name": cfg.name, "final_acc": accs[-1] if accs else float("nan"),
        "best_acc": max(accs) if accs else float("nan"), "round0_acc": accs[0] if accs else float("nan"),
        "final_loss": hist[-1].get("test_loss", float("nan")) if hist else float("nan"),
        "auc": out.get("auc", float("nan")), "epsilon": out.get("epsilon"), "delta": cfg.privacy.delta,
        "rounds": len(hist), "wall_s": out.get("wall_s", 0.0),
        "gpu_hours": out.get("wall_s", 0.0) * ws / 3600.0 if str(out.get("device", "")).startswith("cuda") else 0.0,
        "comm_mb_per_round": (up + down) / n / 2 ** 20, "comm_mb_total": (up + down) / 2 ** 20,
        # bytes each rank actually puts into the round's collective(s) (the all-reduce buffer as sized by the runner)
        "collective_mb_per_round": sum(h.get("comm_bytes_per_rank", 0) for h in hist) / n / 2 ** 20,
        "n_params": P, "world_size": ws, "backend": out.get("backend"), "simulator": out.get("simulator"),
        "config": cfg.to_dict(),
    }
    if run is not None:
        rec["overrides"] = run["overrides"]
        rec["seed"] = run["seed"]
    return rec


def run_grid(spec_or_path, out_dir: str, world=None, device=None, backend=None, limit: int = 0) -> list[dict]:
    from ..api import run_experiment, setup
    if isinstance(spec_or_path, str):
        base_dir = os.path.dirname(os.path.abspath(spec_or_path))
        with open(spec_or_path) as f:
            spec = yaml.safe_load(f)
    else:
        spec, base_dir = copy.deepcopy(spec_or_path), "."
    runs = expand_grid(spec)
    if limit > 0:
        runs = runs[:limit]
    os.makedirs(out_dir, exist_ok=True)
    path = os.path.join(out_dir, "results.jsonl")
    done = set()
    if os.path.exists(path):
        with open(path) as f:
            for line in f:
                if line.strip():
                    r = json.loads(line)
                    done.add(run_key(r))
    results = []
    for run in runs:
        if run_key(run) in done:
            continue
        cfg = build_config(spec, run, base_dir)
        if world is None:
            device, backend, world = setup(cfg)
        out = run_experiment(cfg, world=world, device=device, backend=backend)
        rec = summarize_run(cfg, out, run)
        results.append(rec)
        if world.is_main:
            with open(path, "a") as f:
                f.write(json.dumps(rec, default=float) + "\n")
    return results
