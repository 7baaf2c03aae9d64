"""Does a small pinned->device non_blocking copy (or the pinned allocation) block the host while the GPU
is busy?  Enqueues ~2 ms of GPU work per iteration, then times the host side of each operation."""
import time

import torch


def main():
    dev = torch.device("cuda:0")
    a = torch.randn(2048, 2048, device=dev)
    dst = torch.empty(32768, dtype=torch.uint8, device=dev)
    res = {"alloc": [], "fill": [], "copy": [], "kernel": []}
    for it in range(60):
        t = time.perf_counter()
        for _ in range(8):
            a = a @ a * 1e-3
        res["kernel"].append(time.perf_counter() - t)
        t = time.perf_counter()
        src = torch.empty(32768, dtype=torch.uint8, pin_memory=True)
        res["alloc"].append(time.perf_counter() - t)
        t = time.perf_counter()
        src.fill_(it % 7)
        res["fill"].append(time.perf_counter() - t)
        t = time.perf_counter()
        dst.copy_(src, non_blocking=True)
        res["copy"].append(time.perf_counter() - t)
    torch.cuda.synchronize()
    for k, v in res.items():
        v = sorted(v[10:])
        print(f"{k:7s} p50 {1e3 * v[len(v) // 2]:.3f} ms  p90 {1e3 * v[int(0.9 * len(v))]:.3f} ms  max {1e3 * v[-1]:.3f} ms")


if __name__ == "__main__":
    main()
