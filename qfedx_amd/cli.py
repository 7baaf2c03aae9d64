"""Command line (reference entry points ``python Classical_FL.py`` / ``Preprocess.py`` /
``testEncoder.py``, plus the ROADMAP grid and reporting).

    python -m qfedx_amd run --config configs/iris_4q.yaml train.num_rounds=10 privacy.dp=true
    torchrun --nproc-per-node 8 --master-addr 127.0.0.1 -m qfedx_amd run --config configs/baseline3_20q_dp.yaml
    python -m qfedx_amd grid --spec configs/grid_roadmap.yaml --out results/grid
    python -m qfedx_amd report --results results/grid/results.jsonl
    python -m qfedx_amd preprocess --raw ./dataset/raw --processed ./dataset/processed
    python -m qfedx_amd demo-encoder
    python -m qfedx_amd cfed-main                      # reference Classical_FL.main()
    python -m qfedx_amd show-config --config ...       # resolved config as YAML
"""
from __future__ import annotations

import argparse
import json
import sys


def _cmd_run(a) -> int:
    from .api import run_experiment
    from .config import load_config
    cfg = load_config(a.config, a.overrides)
    out = run_experiment(cfg)
    summary = {"final_acc": out["accuracies"][-1] if out["accuracies"] else None, "accuracies": out["accuracies"],
               "auc": out.get("auc"), "epsilon": out.get("epsilon"), "wall_s": out.get("wall_s"),
               "world_size": out.get("world_size"), "backend": out.get("backend"), "device": out.get("device")}
    if out.get("world_size", 1) == 1 or _rank0():
        print(json.dumps(summary, default=float))
    return 0


def _rank0() -> bool:
    import os
    return int(os.environ.get("RANK", "0")) == 0


def _cmd_grid(a) -> int:
    from .experiments import run_grid, write_report
    run_grid(a.spec, a.out, limit=a.limit)
    if _rank0():
        rep = write_report(f"{a.out}/results.jsonl")
        print(rep["markdown"])
    return 0


def _cmd_report(a) -> int:
    from .experiments import write_report
    rep = write_report(a.results, a.out)
    print(rep["markdown"])
    return 0


def _cmd_preprocess(a) -> int:
    from .compat.Preprocess import main
    out = main(a.raw, a.processed, digits=tuple(a.digits), num_clients=a.num_clients, partition_type=a.partition,
               alpha=a.alpha)
    return 0 if out is not None else 1


def _cmd_demo(a) -> int:
    from .compat.testEncoder import main
    img = None
    if a.synthetic:
        import numpy as np
        from .data.synthetic import synthetic_digit_images
        img = synthetic_digit_images(np.array([2]), 0)[0]
    main(a.raw, a.processed, image=img)
    return 0


def _cmd_cfed(a) -> int:
    from .compat.Classical_FL import main
    out = main(a.raw, a.processed)
    if out is None:
        return 1
    print(json.dumps({"accuracies": out["accuracies"]}))
    return 0


def _cmd_show(a) -> int:
    import yaml
    from .config import load_config
    print(yaml.safe_dump(load_config(a.config, a.overrides).to_dict(), sort_keys=False))
    return 0


def main(argv=None) -> int:
    p = argparse.ArgumentParser(prog="qfedx_amd", description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    sub = p.add_subparsers(dest="cmd", required=True)
    r = sub.add_parser("run", help="one federated experiment")
    r.add_argument("--config", default=None)
    r.add_argument("overrides", nargs="*", help="section.key=value overrides")
    r.set_defaults(fn=_cmd_run)
    g = sub.add_parser("grid", help="experiment grid (ROADMAP:102-109)")
    g.add_argument("--spec", required=True)
    g.add_argument("--out", default="results/grid")
    g.add_argument("--limit", type=int, default=0)
    g.set_defaults(fn=_cmd_grid)
    rp = sub.add_parser("report", help="mean±std table + plots from a grid's results.jsonl")
    rp.add_argument("--results", required=True)
    rp.add_argument("--out", default=None)
    rp.set_defaults(fn=_cmd_report)
    pp = sub.add_parser("preprocess", help="MNIST IDX -> {train,val,test}.pt + client shards (Preprocess.py)")
    pp.add_argument("--raw", default="./dataset/raw")
    pp.add_argument("--processed", default="./dataset/processed")
    pp.add_argument("--digits", type=int, nargs="+", default=[0, 1, 2])
    pp.add_argument("--num-clients", type=int, default=4)
    pp.add_argument("--partition", default="iid")
    pp.add_argument("--alpha", type=float, default=0.5)
    pp.set_defaults(fn=_cmd_preprocess)
    d = sub.add_parser("demo-encoder", help="amplitude / angle encoder demo (testEncoder.py)")
    d.add_argument("--raw", default="./dataset/raw")
    d.add_argument("--processed", default="./dataset/processed")
    d.add_argument("--synthetic", action="store_true", help="use a synthetic digit instead of MNIST")
    d.set_defaults(fn=_cmd_demo)
    c = sub.add_parser("cfed-main", help="reference Classical_FL.main() (TinyCNN FedAvg on MNIST)")
    c.add_argument("--raw", default="./dataset/raw")
    c.add_argument("--processed", default="./dataset/processed")
    c.set_defaults(fn=_cmd_cfed)
    s = sub.add_parser("show-config", help="print the resolved config")
    s.add_argument("--config", default=None)
    s.add_argument("overrides", nargs="*")
    s.set_defaults(fn=_cmd_show)
    a = p.parse_args(argv)
    return a.fn(a)


if __name__ == "__main__":
    sys.exit(main())
