"""The RCCL ("nccl") path on the one GPU of a test box: a single-rank RCCL communicator runs every collective of
a federated round exactly as in an 8-GPU job (the broadcast of theta, the int64 fixed-point all-reduce of the
round buffer, the metric all-reduces of the evaluation, barrier(device_ids) and max_over_ranks on a device
tensor).  Each case runs in a child process so the process group never leaks into other tests."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

_SCRIPT = r"""
import sys, torch
sys.path.insert(0, {root!r})
from tests.test_fl import small_cfg
from qfedx_amd.api import run_experiment
from qfedx_amd.parallel.dist import init_distributed, shutdown, max_over_ranks, barrier
import torch.distributed as dist

def cfg(backend, **kw):
    base = dict(num_rounds=3, n_qubits=10, n_layers=2, num_clients=6, samples_per_client=32, batch_size=8,
                device="cuda", backend="hip", dist_backend=backend)
    return small_cfg(**{{**base, **kw}})

dev = torch.device("cuda", 0)
torch.cuda.set_device(dev)
kw = {kw}
plain = run_experiment(cfg("auto", **kw), world=init_distributed(dev, "auto"), device=dev, backend="hip")
world = init_distributed(dev, "nccl")
assert world.distributed and world.backend == "nccl" and dist.get_backend() == "nccl", world
rccl = run_experiment(cfg("nccl", **kw), world=world, device=dev, backend="hip")
barrier(world)
m = max_over_ranks(1.5, world)
assert m == 1.5, m
same = torch.equal(plain["params"].cpu(), rccl["params"].cpu()) and plain["accuracies"] == rccl["accuracies"]
shutdown(world)
print("RESULT", int(same))
"""


@pytest.mark.parametrize("kw", [{}, dict(dp=True, client_fraction=0.5, deterministic_noise=True),
                                dict(kind="tinycnn", batch_size=32, samples_per_client=64, learning_rate=0.01)])
def test_single_rank_rccl_round_matches_no_group(kw):
    """The HIP round with a one-rank RCCL communicator is bitwise the run without a process group."""
    code = _SCRIPT.format(root=ROOT, kw=repr(kw))
    r = subprocess.run([sys.executable, "-c", code], cwd=ROOT, capture_output=True, text=True, timeout=300,
                       env=dict(os.environ, MASTER_ADDR="127.0.0.1"))
    assert r.returncode == 0, r.stderr[-3000:]
    assert "RESULT 1" in r.stdout, r.stdout[-2000:]


def test_bench_rccl_single_rank():
    """bench.py with --dist-backend nccl at one GPU: the round's all-reduce, barrier and max-over-ranks go
    through RCCL; the JSON line reports it, with the per-phase times and the precision fields."""
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--dist-backend", "nccl", "--qubits", "12",
           "--clients", "8", "--batch", "8", "--steps", "3", "--warmup", "2"]
    r = subprocess.run(cmd, cwd="/tmp", capture_output=True, text=True, timeout=300,
                       env=dict(os.environ, MASTER_ADDR="127.0.0.1"))
    assert r.returncode == 0, r.stderr[-3000:]
    recs = [json.loads(l) for l in r.stdout.splitlines() if l.startswith("{") and '"metric"' in l]
    assert len(recs) == 1
    rec = recs[0]
    assert rec["dist_backend"] == "nccl" and rec["engine"] == "mfma" and rec["value"] > 0
    # the startup self-check (one captured all-reduce replay == an eager one) passed: the round collective runs
    # inside the round hipGraph on the RCCL communicator torch.distributed reports
    assert rec["rccl_world_size"] == 1 and rec["graph_comm"] == "captured", rec
    assert rec["comm_ms"] >= 0 and rec["local_train_ms"] > 0
    assert rec["max_abs_err_expz"] < 5e-3 and rec["max_abs_err_grad"] < 5e-3 * max(1.0, rec["max_abs_grad"])


_SELFCHECK = r"""
import sys, torch
sys.path.insert(0, {root!r})
from qfedx_amd.parallel.dist import init_distributed, shutdown, graph_allreduce_selfcheck, agree_graph_comm
dev = torch.device("cuda", 0)
torch.cuda.set_device(dev)
world = init_distributed(dev, "nccl")
replay = graph_allreduce_selfcheck(world)
ok1 = replay is not None and replay()
ok2 = agree_graph_comm(world, True)
shutdown(world)
print("RESULT", int(ok1), int(ok2))
"""


def test_captured_allreduce_selfcheck_rccl():
    """The startup self-check on a real RCCL communicator: one all-reduce captured in a hipGraph, replayed, equals an
    eager all-reduce bitwise, and the (one-rank) vote agrees on capturing the round collective."""
    r = subprocess.run([sys.executable, "-c", _SELFCHECK.format(root=ROOT)], cwd=ROOT, capture_output=True, text=True,
                       timeout=300, env=dict(os.environ, MASTER_ADDR="127.0.0.1"))
    assert r.returncode == 0, r.stderr[-3000:]
    assert "RESULT 1 1" in r.stdout, r.stdout[-2000:]


_CC4 = r"""
import sys, torch
sys.path.insert(0, {root!r})
from tests.test_fl import small_cfg
from qfedx_amd.api import run_experiment
from qfedx_amd.parallel.dist import init_distributed, shutdown
from qfedx_amd.fl.trainer import VQCClientTrainer
import os

calls = [0]
real = VQCClientTrainer._cc4_gather
def counting(self, *a, **k):
    calls[0] += 1
    return real(self, *a, **k)
VQCClientTrainer._cc4_gather = counting

def cfg(backend, **kw):
    base = dict(num_rounds=4, n_qubits=12, n_layers=3, num_clients=6, samples_per_client=32, batch_size=8,
                device="cuda", backend="hip", dist_backend=backend, state_dtype="mfma")
    return small_cfg(**{{**base, **kw}})

dev = torch.device("cuda", 0)
torch.cuda.set_device(dev)
kw = {kw}
os.environ["QFEDX_CC4"] = "0"
plain = run_experiment(cfg("auto", **kw), world=init_distributed(dev, "auto"), device=dev, backend="hip")
c_off = calls[0]
os.environ["QFEDX_CC4"] = "1"
world = init_distributed(dev, "nccl")
rccl = run_experiment(cfg("nccl", **kw), world=world, device=dev, backend="hip")
same = torch.equal(plain["params"].cpu(), rccl["params"].cpu()) and plain["accuracies"] == rccl["accuracies"]
shutdown(world)
print("RESULT", int(same), c_off, calls[0])
"""


@pytest.mark.parametrize("kw", [{}, dict(local_epochs=2, client_fraction=0.5)])
def test_cc4_side_stream_gather_is_bitwise(kw):
    """Verdict r5 item 4 (CC4): with a one-rank RCCL group and QFEDX_CC4=1 every round's host upload and minibatch
    gather run on a side stream (ahead of the round graph, against the previous round's graph and collective), and
    the run is bitwise the no-group run without the overlap.  (Plain FedAvg on the MFMA engine: with the group, the
    Adam-epilogue FedAvg tail writes the all-reduce buffer and leaves the apply to the collective's post step; without
    it, the tail also applies the round - the multi-rank form of the fused tail)"""
    code = _CC4.format(root=ROOT, kw=repr(kw))
    r = subprocess.run([sys.executable, "-c", code], cwd=ROOT, capture_output=True, text=True, timeout=300,
                       env=dict(os.environ, MASTER_ADDR="127.0.0.1"))
    assert r.returncode == 0, r.stderr[-3000:]
    line = [l for l in r.stdout.splitlines() if l.startswith("RESULT")][-1].split()
    assert line[1] == "1", r.stdout[-2000:]
    assert int(line[2]) == 0 and int(line[3]) >= 4, line      # the side-stream path ran every round (+ warm-ups)
