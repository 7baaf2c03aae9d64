"""Timing of the CFed conv kernels alone (cnn_forward / cnn_backward) at the cfed128 shape.

    python scripts/cnn_kbench.py [--clients 128] [--batch 32] [--iters 20]
Prints one JSON line: mean ms per call of each kernel (device events, after warm-up).
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.environ.get("QFX_PKG_ROOT") or os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from qfedx_amd.models import tinycnn as tc  # noqa: E402
from qfedx_amd.ops._ext import ext  # noqa: E402
from qfedx_amd.ops.cnn_hip import HipTinyCNN  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--clients", type=int, default=128)
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--iters", type=int, default=20)
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    K, B, C = a.clients, a.batch, 10
    m = HipTinyCNN(C, dev)
    g = torch.Generator(device="cpu").manual_seed(0)
    params = (torch.randn(K, tc.n_params(C), generator=g) * 0.1).to(dev)
    X = torch.rand(K, B, 1, 28, 28, generator=g).to(dev)
    Xf, pool1, am1, pool2, am2 = m.conv_forward(params, X)
    dP2 = (torch.randn(K * B, 1568, generator=g) * 0.01).to(dev)
    E = ext()
    G = E.cnn_bwd_groups(K, B)
    part = torch.empty(K * G, E.cnn_partial_size(), device=dev)
    grad = torch.zeros(K, m.P, device=dev)

    def fwd():
        E.cnn_forward(Xf, params, K, B, m.off_conv, pool1, am1, pool2, am2)

    def bwd():
        E.cnn_backward(Xf, params, K, B, m.off_conv, pool1, am1, pool2, am2, dP2, part, grad)

    out = {"clients": K, "batch": B}
    for name, fn in (("cnn_fwd", fwd), ("cnn_bwd", bwd)):
        for _ in range(3):
            fn()
        torch.cuda.synchronize()
        t0, t1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        t0.record()
        for _ in range(a.iters):
            fn()
        t1.record()
        torch.cuda.synchronize()
        out[name] = round(t0.elapsed_time(t1) / a.iters, 4)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
