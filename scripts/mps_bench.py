"""Throughput of the MPS backend on one device: one VQC local step (loss + gradients) of K clients x B
samples at n qubits.  python scripts/mps_bench.py [--qubits 32 --layers 3 --clients 64 --batch 32]"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--qubits", type=int, default=32)
    ap.add_argument("--layers", type=int, default=3)
    ap.add_argument("--clients", type=int, default=64)
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--iters", type=int, default=3)
    args = ap.parse_args()
    import torch
    from qfedx_amd.models.vqc import VQCSpec
    from qfedx_amd.ops.engine import VQCEngine
    dev = torch.device("cuda", 0) if torch.cuda.is_available() else torch.device("cpu")
    spec = VQCSpec(args.qubits, args.layers, 3)
    eng = VQCEngine(spec, dev, "mps")
    K, B = args.clients, args.batch
    g = torch.Generator().manual_seed(0)
    x = spec.encode_features(torch.rand(K, B, args.qubits, generator=g)).to(dev)
    y = torch.randint(0, 3, (K, B), generator=g).to(dev)
    w = torch.full((K, B), 1.0 / B, device=dev)
    params = torch.stack([spec.init_params(k) for k in range(K)]).to(dev)
    eng.loss_and_grads(x, y, w, params)
    if dev.type == "cuda":
        torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.iters):
        eng.loss_and_grads(x, y, w, params)
    if dev.type == "cuda":
        torch.cuda.synchronize()
    ms = (time.perf_counter() - t0) / args.iters * 1e3
    print(json.dumps({"qubits": args.qubits, "layers": args.layers, "samples": K * B, "step_ms": round(ms, 2),
                      "samples_per_s": round(K * B / ms * 1e3, 1), "exact_bond": eng.prog.exact_bond,
                      "autograd": eng.prog.autograd_ok, "device": str(dev)}), flush=True)


if __name__ == "__main__":
    main()
