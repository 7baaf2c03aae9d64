"""Graph vs eager federated runs: bitwise equality over repeated runs (debug helper)."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from tests.test_fl import small_cfg
from qfedx_amd.api import run_experiment
from qfedx_amd.parallel.dist import init_distributed
import qfedx_amd.fl.trainer as tr
dev = torch.device("cuda", 0)
world = init_distributed(dev)
res = {}
for name, graphs in [("g%d" % i, True) for i in range(4)] + [("e%d" % i, False) for i in range(4)]:
    tr.VQCClientTrainer.use_graph = property(lambda self, g=graphs: g)
    out = run_experiment(small_cfg(num_rounds=3, n_qubits=6, device="cuda", backend="hip"), world=world, device=dev, backend="hip")
    res[name] = out["params"].clone()
names = list(res)
for a in names:
    print(a, " ".join(f"{(res[a] - res[b]).abs().max().item():.1e}" for b in names))
