"""Multi-rank runs of the HIP path on the one GPU of a test box: two ranks share cuda:0 over gloo (RCCL needs one
GPU per rank).  Everything a rank does on the device - hipGraph-replayed local rounds on the MFMA engine, the fused
FedAvg reduce, the device-side round epilogue, the collectives on device tensors - runs exactly as in an 8-GPU
job; only the transport differs.  The driver's 8 x MI355X scaling run uses the same code over RCCL."""
import json
import os
import socket
import subprocess
import sys

import pytest
import torch
import torch.multiprocessing as mp

from tests.test_fl import small_cfg

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _cfg(**kw):
    base = dict(num_rounds=3, n_qubits=10, n_layers=2, num_clients=6, samples_per_client=32, batch_size=8,
                device="cuda", backend="hip", dist_backend="gloo")
    return small_cfg(**{**base, **kw})


def _worker(rank, world, port, kw, out_path):
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK="0", MASTER_ADDR="127.0.0.1",
                      MASTER_PORT=str(port))
    from qfedx_amd.api import run_experiment
    out = run_experiment(_cfg(**kw))
    import torch.distributed as dist
    if rank == 0:
        torch.save({"params": out["params"].cpu(), "acc": torch.tensor(out["accuracies"])}, out_path)
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("kw", [{}, dict(dp=True, client_fraction=0.5, deterministic_noise=True),
                                # CFed: the CNN backward's per-workgroup sample grouping depends on the batch only,
                                # so 6 clients on one rank and 3 + 3 on two ranks sum gradients in the same order
                                dict(kind="tinycnn", batch_size=32, samples_per_client=64, learning_rate=0.01)])
def test_two_ranks_on_gpu_match_single_process(tmp_path, kw):
    """Clients sharded over 2 GPU ranks give the bitwise-same global model as one rank (exact fixed-point
    FedAvg; RNG keyed by client, never by rank)."""
    from qfedx_amd.api import run_experiment
    from qfedx_amd.parallel.dist import init_distributed
    dev = torch.device("cuda", 0)
    single = run_experiment(_cfg(**kw), world=init_distributed(dev), device=dev, backend="hip")
    out_path = str(tmp_path / "two.pt")
    mp.spawn(_worker, args=(2, _free_port(), kw, out_path), nprocs=2, join=True)
    two = torch.load(out_path, weights_only=True)
    assert torch.equal(two["params"], single["params"].cpu())
    assert torch.equal(two["acc"], torch.tensor(single["accuracies"]))


def test_bench_two_ranks_share_gpu():
    """bench.py as the driver launches it for N = 2 (torch.distributed.run, one JSON line from rank 0)."""
    env = dict(os.environ, MASTER_ADDR="127.0.0.1")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2", "--master-addr",
           "127.0.0.1", "--master-port", str(_free_port()), os.path.join(ROOT, "bench.py"), "--gpus", "2",
           "--dist-backend", "gloo", "--qubits", "12", "--clients", "8", "--batch", "8", "--steps", "3",
           "--warmup", "2"]
    r = subprocess.run(cmd, cwd="/tmp", env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    recs = [json.loads(l) for l in r.stdout.splitlines() if l.startswith("{") and '"metric"' in l]
    assert len(recs) == 1
    rec = recs[0]
    assert rec["n_gpus"] == 2 and rec["engine"] == "mfma" and rec["backend"] == "hip" and rec["value"] > 0
    assert rec["config"]["parallelism"] == "client-parallel dp2"
