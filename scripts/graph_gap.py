"""Inter-graph launch gap on this ROCm stack: replay captured hipGraphs back to back (no host sync) and report the
GPU time per replay vs the kernels inside (scripts: run under rocprofv3 --kernel-trace for the per-gap split).

python scripts/graph_gap.py [--kernels 12] [--reps 200] [--graphs 1|2] [--work 64] [--dirty-mb 0] [--trace]

``--dirty-mb``: the graph's last node writes that many MB (dirty L2 lines at the graph boundary), to tell a
boundary cache writeback from a fixed launch cost.  ``--trace``: also print the inter-graph gaps measured from
the replays' kernel timestamps (run under rocprofv3 --kernel-trace and read the CSV instead when available).
"""
import argparse
import json
import time

import torch


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--kernels", type=int, default=12)
    ap.add_argument("--reps", type=int, default=200)
    ap.add_argument("--graphs", type=int, default=1)
    ap.add_argument("--work", type=int, default=64, help="elements x 1024 per kernel (tiny by default)")
    ap.add_argument("--events", type=int, default=0, help="HIP events recorded around each replay (0 / 2)")
    ap.add_argument("--dirty-mb", type=int, default=0)
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    x = torch.zeros(args.work * 1024, device=dev)
    big = torch.zeros(max(args.dirty_mb, 1) * 262144, device=dev)
    graphs = []
    s = torch.cuda.Stream(device=dev)
    with torch.cuda.stream(s):
        for _ in range(3):
            for _ in range(args.kernels):
                x.add_(1.0)
    torch.cuda.synchronize()
    for _ in range(args.graphs):
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            for _ in range(args.kernels):
                x.add_(1.0)
            if args.dirty_mb:
                big.add_(1.0)
        graphs.append(g)
    for i in range(10):
        graphs[i % args.graphs].replay()
    torch.cuda.synchronize()
    evs = [torch.cuda.Event(enable_timing=True) for _ in range(2 * args.reps)] if args.events else None
    t0 = time.perf_counter()
    for i in range(args.reps):
        if evs:
            evs[2 * i].record()
        graphs[i % args.graphs].replay()
        if evs:
            evs[2 * i + 1].record()
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / args.reps
    # the same kernels launched eagerly (no graph)
    t0 = time.perf_counter()
    for i in range(args.reps):
        for _ in range(args.kernels):
            x.add_(1.0)
    torch.cuda.synchronize()
    de = (time.perf_counter() - t0) / args.reps
    print(json.dumps({"graphs": args.graphs, "kernels": args.kernels, "events": args.events, "dirty_mb": args.dirty_mb,
                      "us_per_replay": round(dt * 1e6, 2),
                      "us_per_eager_round": round(de * 1e6, 2)}))


if __name__ == "__main__":
    main()
