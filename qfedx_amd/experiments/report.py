"""Grid reporting (ROADMAP.md:118-121): mean +/- std over seeds per configuration, a markdown
table, and the acc-vs-epsilon, acc-vs-qubits and speedup-vs-clients plots."""
from __future__ import annotations

import json
import math
import os
from collections import defaultdict

import numpy as np

METRICS = ("final_acc", "best_acc", "auc", "epsilon", "wall_s", "comm_mb_per_round", "comm_mb_total", "gpu_hours")


def load_results(path: str) -> list[dict]:
    with open(path) as f:
        return [json.loads(x) for x in f if x.strip()]


def _num(v):
    try:
        v = float(v)
        return v if math.isfinite(v) else None
    except (TypeError, ValueError):
        return None


def aggregate(results: list[dict]) -> list[dict]:
    """Group runs by their overrides (seeds pooled) -> mean/std/n of every metric."""
    groups = defaultdict(list)
    for r in results:
        groups[json.dumps(r.get("overrides", {}), sort_keys=True)].append(r)
    rows = []
    for key, rs in groups.items():
        row = {"overrides": json.loads(key), "n_seeds": len(rs)}
        for m in METRICS:
            vals = [x for x in (_num(r.get(m)) for r in rs) if x is not None]
            row[m + "_mean"] = float(np.mean(vals)) if vals else None
            row[m + "_std"] = float(np.std(vals)) if len(vals) > 1 else 0.0 if vals else None
        rows.append(row)
    return rows


def _series(rows, x_key, y_metric, group_keys=()):
    by = defaultdict(list)
    for r in rows:
        ov = r["overrides"]
        if x_key not in ov or r.get(y_metric + "_mean") is None:
            continue
        label = ", ".join(f"{k.split('.')[-1]}={ov[k]}" for k in group_keys if k in ov) or y_metric
        by[label].append((ov[x_key], r[y_metric + "_mean"], r[y_metric + "_std"] or 0.0))
    out = {}
    for label, pts in by.items():
        pts.sort(key=lambda t: t[0])
        out[label] = pts
    return out


def _plot(series: dict, xlabel: str, ylabel: str, title: str, path: str) -> bool:
    if not series:
        return False
    from ..data.viz import plot_series
    xs_all = sorted({p[0] for pts in series.values() for p in pts})
    ys, es = {}, {}
    for label, pts in series.items():
        d = {p[0]: p for p in pts}
        ys[label] = [d[x][1] if x in d else float("nan") for x in xs_all]
        es[label] = [d[x][2] if x in d else 0.0 for x in xs_all]
    try:
        plot_series(xs_all, ys, xlabel, ylabel, title, path, es)
        return True
    except Exception:
        return False


def write_report(results_path: str, out_dir: str | None = None) -> dict:
    results = load_results(results_path)
    out_dir = out_dir or os.path.dirname(os.path.abspath(results_path))
    rows = aggregate(results)
    keys = sorted({k for r in rows for k in r["overrides"]})
    lines = ["| " + " | ".join(keys + ["seeds", "acc (mean±std)", "AUC", "ε", "comm MB/round", "wall s"]) + " |",
             "|" + "---|" * (len(keys) + 6)]
    for r in sorted(rows, key=lambda r: json.dumps(r["overrides"], sort_keys=True)):
        def ms(m, nd=4):
            mu, sd = r[m + "_mean"], r[m + "_std"]
            return "-" if mu is None else f"{mu:.{nd}f} ± {sd:.{nd}f}"
        lines.append("| " + " | ".join([str(r["overrides"].get(k, "")) for k in keys] +
                                       [str(r["n_seeds"]), ms("final_acc"), ms("auc", 3), ms("epsilon", 3),
                                        ms("comm_mb_per_round", 4), ms("wall_s", 2)]) + " |")
    md = "\n".join(lines) + "\n"
    with open(os.path.join(out_dir, "report.md"), "w") as f:
        f.write(md)
    with open(os.path.join(out_dir, "summary.json"), "w") as f:
        json.dump(rows, f, indent=1, default=float)
    plots = {}
    # acc vs epsilon: x = epsilon (mean), series by non-privacy overrides
    eps_pts = defaultdict(list)
    for r in rows:
        if r.get("epsilon_mean") is not None and r.get("final_acc_mean") is not None:
            label = ", ".join(f"{k.split('.')[-1]}={v}" for k, v in sorted(r["overrides"].items())
                              if not k.startswith("privacy.")) or "acc"
            eps_pts[label].append((r["epsilon_mean"], r["final_acc_mean"], r["final_acc_std"] or 0.0))
    plots["acc_vs_eps"] = _plot({k: sorted(v) for k, v in eps_pts.items()}, "epsilon (delta=1e-5)", "test accuracy",
                                "Accuracy vs privacy budget", os.path.join(out_dir, "acc_vs_eps.png"))
    plots["acc_vs_qubits"] = _plot(_series(rows, "model.n_qubits", "final_acc", ("model.n_layers",)), "qubits",
                                   "test accuracy", "Accuracy vs qubits", os.path.join(out_dir, "acc_vs_qubits.png"))
    sp = _series(rows, "data.num_clients", "wall_s")
    if sp:
        sp = {k: [(x, pts[0][1] / y if y else float("nan"), 0.0) for x, y, _ in pts] for k, pts in sp.items()}
    plots["speedup_vs_clients"] = _plot(sp, "clients", "speedup vs fewest clients", "Speedup vs clients",
                                        os.path.join(out_dir, "speedup_vs_clients.png"))
    return {"rows": rows, "markdown": md, "plots": plots}
