"""Kernel micro-benchmark: time each statevector pass of one local step and report effective HBM
bandwidth (bytes of state streamed / time).  Used with rocprofv3 --pmc for counter collection.

python scripts/kbench.py --qubits 16 --layers 3 --samples 2048 --iters 5
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from qfedx_amd.models.vqc import VQCSpec  # noqa: E402
from qfedx_amd.ops._ext import ext  # noqa: E402
from qfedx_amd.ops.statevec_hip import HipProgram  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--qubits", type=int, default=16)
    ap.add_argument("--layers", type=int, default=3)
    ap.add_argument("--samples", type=int, default=2048)
    ap.add_argument("--clients", type=int, default=64)
    ap.add_argument("--iters", type=int, default=5)
    ap.add_argument("--kmax", type=int, default=12)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    spec = VQCSpec(a.qubits, a.layers, 3)
    ops, coef = spec.program()
    prog = HipProgram(ops, coef, a.qubits, spec.readout, dev, spec.n_theta, kmax=a.kmax)
    K = a.clients
    B = a.samples // K
    S = K * B
    x = spec.encode_features(torch.rand(K, B, a.qubits, device=dev))
    y = torch.randint(0, 3, (K, B), device=dev)
    w = torch.full((K, B), 1.0 / B, device=dev)
    params = torch.stack([spec.init_params(k) for k in range(K)]).to(dev)
    for _ in range(2):
        prog.loss_and_grads(x, y, w, params, spec)
    torch.cuda.synchronize()
    C = ext()
    xr = x.reshape(S, -1).contiguous()
    psi = prog._ws["psi"]
    lam = prog._ws["lam"]
    part = prog._ws["part"]
    slab = prog._ws["slab"]
    wread = prog._ws["wread"]
    res = {}
    state_bytes = S * (1 << a.qubits) * 8
    for name, plan, adj in (("fwd", prog.train_plan, False), ("adj", prog.adj_plan, True)):
        for i, (off, k, ngrad, nops) in enumerate(plan.passes):
            ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
            ev[0].record()
            for _ in range(a.iters):
                if plan.jit_handles is not None:
                    C.jit_launch(plan.jit_handles[i], plan.blob, off, psi, lam if adj else None, params, B, xr,
                                 wread if adj else None, None if adj else part, slab if adj else None, S, ngrad)
                else:
                    C.pass_launch(plan.R, adj, plan.blob, off, k, a.qubits, nops, plan.info['G'], psi,
                                  lam if adj else None, params, B, xr, wread if adj else None,
                                  None if adj else part, slab if adj else None, S, ngrad)
            ev[1].record()
            torch.cuda.synchronize()
            ms = ev[0].elapsed_time(ev[1]) / a.iters
            p = plan.info["passes"][i]
            nbytes = state_bytes * (2 if adj else 1) * (2 if p["INIT"] != 1 else 1)
            res[f"{name}{i}"] = {"ms": round(ms, 4), "GBps": round(nbytes / ms / 1e6, 1), "nops": nops,
                                 "remaps": sum(1 for o in p["ops"] if o["code"] == 5)}
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    ev[0].record()
    for _ in range(a.iters):
        prog.loss_and_grads(x, y, w, params, spec)
    ev[1].record()
    torch.cuda.synchronize()
    res["step_ms"] = round(ev[0].elapsed_time(ev[1]) / a.iters, 4)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
