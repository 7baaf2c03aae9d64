"""Distributed statevector (CC7): states sharded over 2 / 4 gloo ranks by their top qubits, global-qubit
gates via pairwise half-shard exchanges, per-rank phases and relabelled SWAPs; checked against the
float64 single-process oracle (states, <Z>, parameter-shift gradients)."""
import os

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

from tests.test_distributed import _free_port


def _circuit(n, seed, gates=60):
    from qfedx_amd.quantum.circuit import Circuit, ParameterVector
    rng = np.random.default_rng(seed)
    th = ParameterVector("theta", gates)
    qc = Circuit(n)
    k = 0
    for _ in range(gates):
        r = rng.random()
        q = int(rng.integers(n))
        if r < 0.4:
            getattr(qc, ["rx", "ry", "rz", "p"][int(rng.integers(4))])(th[k], q)
            k += 1
        elif r < 0.6:
            getattr(qc, ["h", "x", "y", "z", "s", "sdg", "t", "tdg", "sx"][int(rng.integers(9))])(q)
        else:
            a, b = (int(v) for v in rng.choice(n, 2, replace=False))
            [qc.cx, qc.cz, qc.swap][int(rng.integers(3))](a, b)
    return qc, k


def _worker(rank, world, port, n, seed, out_path):
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.set_num_threads(1)
    import torch.distributed as dist
    from qfedx_amd.parallel.dist_statevec import DistributedStatevector
    dist.init_process_group("gloo", rank=rank, world_size=world)
    qc, P = _circuit(n, seed)
    ds = DistributedStatevector(qc, world, rank)
    vals = torch.tensor(np.random.default_rng(seed + 1).normal(size=(3, P)), dtype=torch.float32)
    psi = ds.run(vals)
    full = ds.gather(psi)
    readout = [0, n - 1, n // 2]
    z = ds.expz_from_shard(psi, readout)
    w = torch.tensor(np.random.default_rng(seed + 2).normal(size=(3, 3)))
    g = ds.param_shift(vals, w, readout)
    if rank == 0:
        torch.save({"full": full, "z": z, "g": g, "vals": vals, "w": w, "swaps": torch.tensor(ds.n_swaps)}, out_path)
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world,n,seed", [(2, 5, 0), (4, 6, 1), (4, 7, 2)])
def test_distributed_statevector_matches_oracle(tmp_path, world, n, seed):
    from qfedx_amd.quantum.statevector import Statevector
    out = str(tmp_path / "ds.pt")
    mp.spawn(_worker, args=(world, _free_port(), n, seed, out), nprocs=world, join=True)
    r = torch.load(out, weights_only=True)
    qc, P = _circuit(n, seed)
    readout = [0, n - 1, n // 2]
    assert int(r["swaps"]) > 0                      # the random circuit does touch global qubits
    for s in range(3):
        ref = Statevector.zero(n).evolve(qc, {"theta": r["vals"][s].double().numpy()})
        assert np.abs(r["full"][s].numpy() - ref.data).max() < 1e-5
        assert np.allclose(r["z"][s].numpy(), [ref.expectation_z(q) for q in readout], atol=1e-5)
    # parameter shift vs central finite differences of the oracle
    eps = 1e-4
    for j in range(0, P, max(1, P // 5)):
        for s in range(3):
            v = r["vals"][s].double().numpy()
            d = np.zeros(P)
            d[j] = eps
            fp = Statevector.zero(n).evolve(qc, {"theta": v + d})
            fm = Statevector.zero(n).evolve(qc, {"theta": v - d})
            num = sum(float(r["w"][s, c]) * (fp.expectation_z(q) - fm.expectation_z(q)) / (2 * eps)
                      for c, q in enumerate(readout))
            assert abs(num - float(r["g"][s, j])) < 2e-3


def test_single_rank_schedule_is_one_segment():
    from qfedx_amd.parallel.dist_statevec import DistributedStatevector
    qc, P = _circuit(5, 3)
    ds = DistributedStatevector(qc, 1, 0)
    assert ds.n_swaps == 0
    from qfedx_amd.quantum.statevector import Statevector
    vals = torch.tensor(np.random.default_rng(0).normal(size=(2, P)), dtype=torch.float32)
    full = ds.gather(ds.run(vals))
    for s in range(2):
        ref = Statevector.zero(5).evolve(qc, {"theta": vals[s].double().numpy()})
        assert np.abs(full[s].numpy() - ref.data).max() < 1e-5
