"""Non-chain MPS training step: the generic HIP kernel (csrc/mps_mpo.hip) vs the torch einsum network on the same GPU.

python scripts/mps_generic_bench.py [--qubits 32 --layers 2 --clients 16 --batch 32 --iters 3]
A ring-entangler VQC (chain + wrap-around CX per layer: bond 16 at 2 layers, outside the chain kernel) - one
``VQCEngine.loss_and_grads`` (readout, CE, adjoint gradients) per iteration.  Prints one JSON line: ms per step of
both paths, the speedup and the max |d loss| / |d grad| between them.
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--qubits", type=int, default=32)
    ap.add_argument("--layers", type=int, default=2)
    ap.add_argument("--clients", type=int, default=16)
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--iters", type=int, default=3)
    args = ap.parse_args()
    import torch
    from qfedx_amd.models.vqc import VQCSpec
    from qfedx_amd.ops.engine import VQCEngine

    dev = torch.device("cuda", 0)
    spec = VQCSpec(args.qubits, args.layers, 3, readout_scale=2.0, entangler="ring")
    K, B = args.clients, args.batch
    g = torch.Generator().manual_seed(0)
    x = spec.encode_features(torch.rand(K, B, args.qubits, generator=g)).to(dev)
    y = torch.randint(0, 3, (K, B), generator=g).to(dev)
    w = torch.full((K, B), 1.0 / B, device=dev)
    params = (torch.stack([spec.init_params(k) for k in range(K)])
              + 0.2 * torch.randn(K, spec.n_params, generator=g)).to(dev)
    res = {}
    for name in ("hip", "torch"):
        eng = VQCEngine(spec, dev, "mps")
        if name == "torch":
            eng.prog._hip = None
        elif eng.prog.hip_program() is None:
            raise SystemExit("the generic MPS kernel does not cover this program")
        out = eng.loss_and_grads(x, y, w, params)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(args.iters):
            out = eng.loss_and_grads(x, y, w, params)
        torch.cuda.synchronize()
        res[name] = (1e3 * (time.perf_counter() - t0) / args.iters, out)
    (th, oh), (tt, ot) = res["hip"], res["torch"]
    print(json.dumps({"model": f"vqc-{args.qubits}q-{args.layers}L-ring", "samples": K * B, "bond": 1 << (2 * args.layers),
                      "hip_ms": round(th, 3), "torch_ms": round(tt, 3), "speedup": round(tt / th, 1),
                      "max_dloss": float((oh["loss"] - ot["loss"]).abs().max()),
                      "max_dgrad": float((oh["grad"] - ot["grad"]).abs().max())}), flush=True)


if __name__ == "__main__":
    main()
