"""Checkpoint / resume (ROADMAP.md:90-91 "Checkpoint theta every K rounds").

Reference checkpoint layout: only the data splits, ``torch.save((X float32 [N,1,28,28],
y int64 [N]))`` to ``dataset/processed/{train,val,test}.pt`` (``Preprocess.py:192-199``); the
model lives only in memory (``Classical_FL.py:157``).  Here a model checkpoint is a plain dict of
tensors + JSON-able metadata, loadable with ``torch.load(weights_only=True)``:

``{"round", "global_state" (state_dict with reference key names for TinyCNN / VQC param names),
"server_state" (optimizer/momentum), "accountant" (RDP orders + accumulated rdp),
"rng" (root seed; all streams are keyed so no generator state is needed), "config" (json str),
"metrics" (json str)}``.  Rank 0 writes atomically (tmp + rename); every rank can read.
"""
from __future__ import annotations

import glob
import json
import os
from typing import Any, Optional

import torch


def _to_saveable(obj: Any):
    if isinstance(obj, torch.Tensor):
        return obj.detach().cpu()
    if isinstance(obj, dict):
        return {k: _to_saveable(v) for k, v in obj.items()}
    if isinstance(obj, (list, tuple)):
        return type(obj)(_to_saveable(v) for v in obj)
    return obj


def save_checkpoint(path_dir: str, round_num: int, payload: dict, keep_last: int = 3) -> str:
    os.makedirs(path_dir, exist_ok=True)
    path = os.path.join(path_dir, f"round_{round_num:06d}.pt")
    tmp = path + ".tmp"
    data = _to_saveable(dict(payload))
    data["round"] = int(round_num)
    for k in ("config", "metrics"):
        if k in data and not isinstance(data[k], str):
            data[k] = json.dumps(data[k], default=float)
    torch.save(data, tmp)
    os.replace(tmp, path)
    if keep_last > 0:
        ckpts = sorted(glob.glob(os.path.join(path_dir, "round_*.pt")))
        for old in ckpts[:-keep_last]:
            os.remove(old)
    return path


def latest_checkpoint(path_dir: str) -> Optional[str]:
    if not path_dir or not os.path.isdir(path_dir):
        return None
    ckpts = sorted(glob.glob(os.path.join(path_dir, "round_*.pt")))
    return ckpts[-1] if ckpts else None


def load_checkpoint(path: str, map_location="cpu") -> dict:
    data = torch.load(path, map_location=map_location, weights_only=True)
    for k in ("config", "metrics"):
        if k in data and isinstance(data[k], str):
            data[k] = json.loads(data[k])
    return data
