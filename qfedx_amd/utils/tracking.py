"""Experiment tracking in the MLflow *file store* layout, written without the ``mlflow`` package.

ROADMAP.md:92-93 plans "MLflow per experiment: config, checkpoints, metrics, artifacts".  ``mlflow`` is
not in this image, but its file store is a plain directory format, so a run written here can be browsed
later with ``mlflow ui --backend-store-uri <root>`` on any machine that has it:

    <root>/<experiment_id>/meta.yaml
    <root>/<experiment_id>/<run_id>/meta.yaml
    <root>/<experiment_id>/<run_id>/params/<key>            value text
    <root>/<experiment_id>/<run_id>/metrics/<key>           "<timestamp_ms> <value> <step>" lines
    <root>/<experiment_id>/<run_id>/tags/<key>
    <root>/<experiment_id>/<run_id>/artifacts/...           config.yaml, checkpoints, reports

Only rank 0 writes.  Experiment ids are derived from the experiment name (stable across runs).
"""
from __future__ import annotations

import os
import re
import shutil
import time
import uuid
import zlib
from typing import Any, Optional

import yaml

RUNNING, FINISHED, FAILED = 1, 3, 4


def _flatten(d: dict, prefix: str = "") -> dict:
    out = {}
    for k, v in d.items():
        key = f"{prefix}{k}"
        if isinstance(v, dict):
            out.update(_flatten(v, key + "."))
        else:
            out[key] = v
    return out


def _safe(key: str) -> str:
    """MLflow keys allow alphanumerics, _ - . / and space; map anything else to _."""
    return re.sub(r"[^0-9A-Za-z_\-./ ]", "_", key).strip("/") or "_"


class FileTracker:
    def __init__(self, root: str, experiment: str = "qfedx", run_name: str = "", rank: int = 0):
        self.active = bool(root) and rank == 0
        self.run_id = uuid.uuid4().hex
        if not self.active:
            return
        self.root = os.path.abspath(root)
        self.exp_id = str(zlib.crc32(experiment.encode()) % 10 ** 9 + 1)
        exp_dir = os.path.join(self.root, self.exp_id)
        os.makedirs(exp_dir, exist_ok=True)
        meta = os.path.join(exp_dir, "meta.yaml")
        if not os.path.exists(meta):
            self._yaml(meta, {"artifact_location": "file://" + exp_dir, "experiment_id": self.exp_id,
                              "lifecycle_stage": "active", "name": experiment,
                              "creation_time": int(time.time() * 1000),
                              "last_update_time": int(time.time() * 1000)})
        self.dir = os.path.join(exp_dir, self.run_id)
        for sub in ("params", "metrics", "tags", "artifacts"):
            os.makedirs(os.path.join(self.dir, sub), exist_ok=True)
        self.start = int(time.time() * 1000)
        self.name = run_name or self.run_id[:8]
        self._meta(RUNNING, None)
        self.set_tag("mlflow.runName", self.name)
        self.set_tag("mlflow.source.type", "LOCAL")

    # ------------------------------------------------------------------ writers
    @staticmethod
    def _yaml(path: str, obj: dict) -> None:
        with open(path, "w") as f:
            yaml.safe_dump(obj, f, sort_keys=True)

    def _meta(self, status: int, end: Optional[int]) -> None:
        self._yaml(os.path.join(self.dir, "meta.yaml"), {
            "artifact_uri": "file://" + os.path.join(self.dir, "artifacts"), "end_time": end,
            "entry_point_name": "", "experiment_id": self.exp_id, "lifecycle_stage": "active",
            "run_id": self.run_id, "run_name": self.name, "run_uuid": self.run_id, "source_name": "",
            "source_type": 4, "source_version": "", "start_time": self.start, "status": status,
            "tags": [], "user_id": os.environ.get("USER", "qfedx")})

    def log_params(self, params: dict) -> None:
        if not self.active:
            return
        for k, v in _flatten(params).items():
            with open(os.path.join(self.dir, "params", _safe(k)), "w") as f:
                f.write(str(v))

    def set_tag(self, key: str, value: Any) -> None:
        if self.active:
            with open(os.path.join(self.dir, "tags", _safe(key)), "w") as f:
                f.write(str(value))

    def log_metrics(self, metrics: dict, step: int = 0) -> None:
        if not self.active:
            return
        ts = int(time.time() * 1000)
        for k, v in metrics.items():
            if isinstance(v, bool) or not isinstance(v, (int, float)):
                continue
            path = os.path.join(self.dir, "metrics", _safe(k))
            os.makedirs(os.path.dirname(path), exist_ok=True)
            with open(path, "a") as f:
                f.write(f"{ts} {float(v)!r} {int(step)}\n")

    def log_artifact(self, path: str, subdir: str = "") -> None:
        if not self.active or not os.path.exists(path):
            return
        dst = os.path.join(self.dir, "artifacts", subdir)
        os.makedirs(dst, exist_ok=True)
        if os.path.isdir(path):
            shutil.copytree(path, os.path.join(dst, os.path.basename(path)), dirs_exist_ok=True)
        else:
            shutil.copy2(path, dst)

    def log_text(self, text: str, name: str) -> None:
        if self.active:
            with open(os.path.join(self.dir, "artifacts", name), "w") as f:
                f.write(text)

    def end(self, status: int = FINISHED) -> None:
        if self.active:
            self._meta(status, int(time.time() * 1000))
            self.active = False


def read_metric(run_dir: str, key: str) -> list[tuple[int, float, int]]:
    """(timestamp_ms, value, step) rows of one metric file."""
    with open(os.path.join(run_dir, "metrics", _safe(key))) as f:
        return [(int(a), float(b), int(c)) for a, b, c in (ln.split() for ln in f if ln.strip())]
