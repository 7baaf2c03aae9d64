"""Host-side cost of the headline round: per-call time of ``run_round(sync=False)`` (the host's own work,
the GPU runs behind it) vs the wall period of the same rounds.  If the host cost approaches the period,
the GPU idles between rounds waiting for launches.

    python scripts/host_round_time.py [--rounds 30] [--profile]   (--profile: cProfile top functions)
"""
import argparse
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=30)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--profile", action="store_true")
    a = ap.parse_args()
    import torch
    import bench
    from qfedx_amd.api import setup
    from qfedx_amd.data.datasets import build_federated_data
    from qfedx_amd.fl.adapters import make_adapter
    from qfedx_amd.fl.server import FederatedRunner
    from qfedx_amd.parallel.dist import shard_clients

    args = bench.argparse.Namespace(gpus=1, clients=64, batch=32, qubits=16, layers=3, classes=3, local_steps=1,
                                    dp=False, backend="auto", device="auto", dist_backend="auto", engine="mfma")
    cfg = bench.make_config(args)
    device, backend, world = setup(cfg)
    data = build_federated_data(cfg, clients=shard_clients(cfg.data.num_clients, 1, 0))
    runner = FederatedRunner(cfg, make_adapter(cfg, device, backend), data, world, device, backend)
    for r in range(a.warmup):
        runner.run_round(r, sync=False)
    torch.cuda.synchronize()
    host = []
    prof = None
    if a.profile:
        import cProfile
        prof = cProfile.Profile()
        prof.enable()
    t0 = time.perf_counter()
    for r in range(a.warmup, a.warmup + a.rounds):
        h0 = time.perf_counter()
        runner.run_round(r, sync=False)
        host.append(time.perf_counter() - h0)
    t_host = time.perf_counter() - t0
    torch.cuda.synchronize()
    wall = time.perf_counter() - t0
    if prof is not None:
        prof.disable()
    host.sort()
    print(f"rounds {a.rounds}: wall {1e3 * wall / a.rounds:.3f} ms/round, host loop {1e3 * t_host / a.rounds:.3f} "
          f"ms/round, run_round host p50 {1e3 * host[len(host) // 2]:.3f} ms, p90 {1e3 * host[int(0.9 * len(host))]:.3f} ms")
    if prof is not None:
        import pstats
        st = pstats.Stats(prof)
        st.sort_stats("tottime").print_stats(12)


if __name__ == "__main__":
    main()
