"""The driver's ``bench.py`` contract, rehearsed on the CPU: one JSON line from rank 0 with the required keys,
the whole-job value, and the same line shape at world_size 2 (gloo, launched by torch.distributed.run exactly
as the driver launches the multi-GPU scaling runs)."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
KEYS = {"metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
        "vs_baseline", "dtype", "data", "config"}
SMALL = ["--steps", "2", "--warmup", "1", "--device", "cpu", "--qubits", "6", "--clients", "4", "--batch", "8"]


def _json_lines(out: str):
    return [json.loads(l) for l in out.splitlines() if l.startswith("{") and '"metric"' in l]


def _run(cmd, port=None):
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", OMP_NUM_THREADS="2")
    r = subprocess.run(cmd, cwd="/tmp", env=env, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-2000:]
    return _json_lines(r.stdout)


def _check(rec, n, steps=2, warmup=1):
    assert KEYS <= rec.keys()
    assert rec["n_gpus"] == n and rec["steps"] == steps and rec["warmup"] == warmup
    assert rec["higher_is_better"] is True and rec["scaling"] == "strong"
    assert rec["value"] > 0 and rec["ms_per_step"] > 0
    # value is the whole-job aggregate: all clients' local steps over the timed rounds
    total = rec["config"]["n_clients"] * rec["config"]["local_steps_per_round"] * steps
    assert rec["value"] == pytest.approx(total / (rec["ms_per_step"] * steps / 1e3), rel=2e-3)
    assert rec["config"]["parallelism"] == f"client-parallel dp{n}"
    # a CPU run must not claim the MFMA engine's dtype
    assert rec["engine"] == "torch" or rec["backend"] != "hip"
    assert rec["dtype"] == "fp32"


def test_bench_single_process_cpu():
    recs = _run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "1"] + SMALL)
    assert len(recs) == 1
    _check(recs[0], 1)


def test_bench_two_ranks_gloo():
    recs = _run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
                 "--master-addr", "127.0.0.1", "--master-port", "29627", os.path.join(ROOT, "bench.py"),
                 "--gpus", "2"] + SMALL)
    assert len(recs) == 1, "only rank 0 prints"
    _check(recs[0], 2)


def test_bench_self_launches_ranks_for_gpus_flag():
    """``python bench.py --gpus 2`` without a launcher spawns torch.distributed.run itself."""
    recs = _run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2"] + SMALL)
    assert len(recs) == 1
    _check(recs[0], 2)


def test_bench_rejects_mismatched_world():
    env = dict(os.environ, WORLD_SIZE="1", RANK="0", LOCAL_RANK="0", MASTER_ADDR="127.0.0.1")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "4"] + SMALL, cwd="/tmp",
                       env=env, capture_output=True, text=True, timeout=120)
    assert r.returncode != 0 and "WORLD_SIZE=1" in r.stderr
