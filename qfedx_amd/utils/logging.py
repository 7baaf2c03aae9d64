"""Metrics and logging.

Reference: ``print`` only, accuracy list returned (``Classical_FL.py:116,124,148,157``), progress
every 5 rounds (``:151-152``); MLflow planned (``ROADMAP.md:16,92-93``).  Here: a rank-0 JSONL
metrics writer (one JSON object per round: acc, loss, AUC, epsilon, comm bytes, wall-clock,
rounds/s, local-steps/s) plus a stdlib ``logging`` logger.  With ``tracking_dir`` set, every record
also goes to an MLflow-file-store run (``utils/tracking.py``: params, metrics, config + checkpoint
artifacts), written without the ``mlflow`` package.
"""
from __future__ import annotations

import json
import logging
import os
import sys
import time
from typing import Any, Optional

_LOGGER: Optional[logging.Logger] = None


def get_logger(name: str = "qfedx") -> logging.Logger:
    global _LOGGER
    if _LOGGER is None:
        lg = logging.getLogger(name)
        if not lg.handlers:
            h = logging.StreamHandler(sys.stdout)
            rank = os.environ.get("RANK", "0")
            h.setFormatter(logging.Formatter(f"[%(asctime)s r{rank} %(levelname)s] %(message)s",
                                             "%H:%M:%S"))
            lg.addHandler(h)
        lg.setLevel(os.environ.get("QFEDX_LOGLEVEL", "INFO"))
        lg.propagate = False
        _LOGGER = lg
    return _LOGGER


class MetricsWriter:
    """Append-only JSONL metrics sink; only rank 0 writes."""

    def __init__(self, path: str = "", rank: int = 0, config: Optional[dict] = None, tracking_dir: str = "",
                 experiment: str = "qfedx"):
        from .tracking import FileTracker
        self.path = path
        self.tracker = FileTracker(tracking_dir, experiment, (config or {}).get("name", ""), rank)
        if config is not None:
            self.tracker.log_params(config)
            self.tracker.log_text(yaml_dump(config), "config.yaml")
        self.rank = rank
        self.records: list[dict] = []
        self._f = None
        self._mlflow = None
        if path and rank == 0:
            os.makedirs(os.path.dirname(os.path.abspath(path)), exist_ok=True)
            self._f = open(path, "a", buffering=1)
            if config is not None:
                self._f.write(json.dumps({"event": "config", "time": time.time(), "config": config}) + "\n")
        try:  # optional tracking backend (ROADMAP:92-93)
            import mlflow  # type: ignore
            if rank == 0 and os.environ.get("QFEDX_MLFLOW"):
                self._mlflow = mlflow
        except ImportError:
            pass

    def log(self, record: dict[str, Any]) -> None:
        rec = {"time": time.time(), **record}
        self.records.append(rec)
        if self._f is not None:
            self._f.write(json.dumps(rec, default=float) + "\n")
        self.tracker.log_metrics(record, step=int(rec.get("round", 0)))
        if self._mlflow is not None:
            step = int(rec.get("round", 0))
            self._mlflow.log_metrics({k: float(v) for k, v in rec.items()
                                      if isinstance(v, (int, float))}, step=step)

    def close(self) -> None:
        self.tracker.end()
        if self._f is not None:
            self._f.close()
            self._f = None

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()


def yaml_dump(obj: dict) -> str:
    import yaml
    return yaml.safe_dump(json.loads(json.dumps(obj, default=str)), sort_keys=False)


def read_jsonl(path: str) -> list[dict]:
    with open(path) as f:
        return [json.loads(line) for line in f if line.strip()]
