"""Timing of the MFMA engine's parameter-shift estimator (``HeaMfmaProgram.param_shift``, prefix reuse + pi identity)
at BASELINE config 5's circuit (24q x 3L, 2 classes, shot-sampled), for K clients x B samples.

python scripts/ps_kbench.py [--clients 16 --batch 8 --iters 2]
Prints one JSON line: ms per estimator call and ms per client (config 5 runs 256 clients x 8 samples per round).
"""
import argparse
import json
import os
import sys
import time

# QFX_PKG_ROOT: import the package from another built tree (scripts/gpu_ab.sh)
sys.path.insert(0, os.environ.get("QFX_PKG_ROOT") or os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--qubits", type=int, default=24)
    ap.add_argument("--layers", type=int, default=3)
    ap.add_argument("--clients", type=int, default=16)
    ap.add_argument("--batch", type=int, default=8)
    ap.add_argument("--iters", type=int, default=2)
    args, _ = ap.parse_known_args()
    import torch
    from qfedx_amd.models.vqc import VQCSpec
    from qfedx_amd.ops.hea_mfma import HeaMfmaProgram
    from qfedx_amd.quantum.noise import NoiseModel

    dev = torch.device("cuda", 0)
    spec = VQCSpec(args.qubits, args.layers, 2, readout_scale=3.0)
    prog = HeaMfmaProgram(spec, dev)
    K, B = args.clients, args.batch
    g = torch.Generator().manual_seed(0)
    x = spec.encode_features(torch.rand(K, B, args.qubits, generator=g)).to(dev)
    params = torch.stack([spec.init_params(k) for k in range(K)]).to(dev)[:, :spec.n_theta].contiguous()
    w = (torch.rand(K, B, 2, generator=g) - 0.5).to(dev)
    keys = torch.randint(0, 2 ** 31, (K, 2), generator=g).long().to(dev)
    nz = NoiseModel(shots=1024)
    out = prog.param_shift(x, params, w, noise=nz, keys=keys, step=0)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(args.iters):
        out = prog.param_shift(x, params, w, noise=nz, keys=keys, step=i + 1)
    torch.cuda.synchronize()
    ms = 1e3 * (time.perf_counter() - t0) / args.iters
    print(json.dumps({"ps_ms": round(ms, 2), "ms_per_client": round(ms / K, 3), "clients": K, "batch": B,
                      "passes": prog.shift_pass_counts(), "checksum": float(out.double().abs().sum())}), flush=True)


if __name__ == "__main__":
    main()
