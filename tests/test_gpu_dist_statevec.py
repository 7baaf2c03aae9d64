"""Distributed statevector with HIP segments: 2 ranks sharing the box's GPU (gloo, host-staged exchange)
vs the single-GPU Simulator on the same random circuit."""
import os

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

from tests.test_dist_statevec import _circuit
from tests.test_distributed import _free_port

pytestmark = pytest.mark.gpu


def _worker(rank, world, port, n, seed, out_path):
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch.distributed as dist
    from qfedx_amd.parallel.dist_statevec import DistributedStatevector
    dist.init_process_group("gloo", rank=rank, world_size=world)
    qc, P = _circuit(n, seed, gates=120)
    dev = torch.device("cuda", 0)
    ds = DistributedStatevector(qc, world, rank, dev)
    vals = torch.tensor(np.random.default_rng(seed).normal(size=(4, P)), dtype=torch.float32)
    psi = ds.run(vals)
    full = ds.gather(psi)
    z = ds.expz_from_shard(psi, [0, n - 1])
    if rank == 0:
        torch.save({"full": full.cpu(), "z": z.cpu(), "vals": vals, "swaps": torch.tensor(ds.n_swaps)}, out_path)
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("n", [12, 15])
def test_distributed_hip_segments_match_simulator(tmp_path, cuda, n):
    from qfedx_amd.quantum.simulator import Simulator
    out = str(tmp_path / "ds.pt")
    port = _free_port()
    mp.start_processes(_worker, args=(2, port, n, n, out), nprocs=2, join=True, start_method="spawn")
    r = torch.load(out, weights_only=True)
    assert int(r["swaps"]) > 0
    qc, P = _circuit(n, n, gates=120)
    psi, z = Simulator(qc, readout=[0, n - 1], device=cuda).run(r["vals"].to(cuda))
    assert (r["full"] - psi.cpu()).abs().max() < 1e-4
    assert torch.allclose(r["z"], z.cpu(), atol=1e-4)
