"""Host-side cost of enqueueing one federated round (no device sync) vs the device time per round: tells
whether small per-rank shares are host-bound.  python scripts/host_round_time.py [--clients 8]"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--clients", type=int, default=8)
    ap.add_argument("--rounds", type=int, default=40)
    args = ap.parse_args()
    import torch
    import bench
    from qfedx_amd.api import setup
    from qfedx_amd.parallel.dist import World
    ns = argparse.Namespace(gpus=1, steps=args.rounds, warmup=3, qubits=16, layers=3, clients=args.clients, batch=32,
                            local_steps=1, classes=3, dp=False, backend="auto", device="auto", engine="mfma")
    cfg = bench.make_config(ns)
    device, backend, world = setup(cfg)
    from qfedx_amd.data.datasets import build_federated_data
    from qfedx_amd.fl.adapters import make_adapter
    from qfedx_amd.fl.server import FederatedRunner
    data = build_federated_data(cfg)
    runner = FederatedRunner(cfg, make_adapter(cfg, device, backend), data, world, device, backend)
    for r in range(5):
        runner.run_round(r, sync=False)
    torch.cuda.synchronize()
    host = []
    t0 = time.perf_counter()
    for r in range(5, 5 + args.rounds):
        h0 = time.perf_counter()
        runner.run_round(r, sync=False)
        host.append(time.perf_counter() - h0)
    torch.cuda.synchronize()
    wall = (time.perf_counter() - t0) / args.rounds
    host.sort()
    print(json.dumps({"clients": args.clients, "wall_ms_per_round": round(wall * 1e3, 3),
                      "host_ms_median": round(host[len(host) // 2] * 1e3, 3),
                      "host_ms_p90": round(host[int(0.9 * len(host))] * 1e3, 3)}), flush=True)


if __name__ == "__main__":
    main()
