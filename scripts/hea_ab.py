"""Interleaved A/B of MFMA-engine variants in ONE process (guide rule: perf deltas from interleaved rounds on one
device).  Variants are run-time environment switches (``env.NAME=value``, e.g. env.QFEDX_HEA_PAIR=0) and the state
storage (fp16 | bf16).  Each round times every variant's full local step (frags, forward, readout, adjoint, gradient
reduction) and its adjoint passes alone; prints per-variant median / min ms over the rounds as JSON.

python scripts/hea_ab.py [--qubits 16 --layers 3 --clients 64 --batch 32 --rounds 7 --iters 10]
                         [--variants "fp16:storage=fp16,bf16:storage=bf16"]
"""
import argparse
import json
import os
import statistics
import sys

sys.path.insert(0, os.environ.get("QFX_PKG_ROOT") or os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def parse_variants(spec: str):
    out = []
    for item in spec.split(","):
        name, _, kv = item.partition(":")
        knobs = {}
        for pair in filter(None, kv.split(";")):
            k, _, v = pair.partition("=")
            knobs[k] = v
        out.append((name, knobs))
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--qubits", type=int, default=16)
    ap.add_argument("--layers", type=int, default=3)
    ap.add_argument("--clients", type=int, default=64)
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--rounds", type=int, default=7)
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--variants", default="fp16:storage=fp16,bf16:storage=bf16")
    args = ap.parse_args()
    import torch
    from qfedx_amd.models.vqc import VQCSpec
    from qfedx_amd.ops._ext import ext
    from qfedx_amd.ops.hea_mfma import HeaMfmaProgram

    dev = torch.device("cuda", 0)
    spec = VQCSpec(args.qubits, args.layers, 3)
    K, B = args.clients, args.batch
    S = K * B
    g = torch.Generator().manual_seed(0)
    x = (torch.rand(K, B, args.qubits, generator=g) * 3).to(dev)
    y = torch.randint(0, 3, (K, B), generator=g).to(dev)
    w = torch.full((K, B), 1.0 / B, device=dev)
    params = torch.stack([spec.init_params(k) for k in range(K)]).to(dev)
    variants = parse_variants(args.variants)
    progs = {}

    def set_knobs(knobs):
        for k, v in knobs.items():
            if k.startswith("env."):           # environment switches, e.g. env.QFEDX_HEA_PAIR=0
                os.environ[k[4:]] = v

    for name, knobs in variants:
        set_knobs(knobs)                       # plan-level switches (QFEDX_HEA_PAIR) act when the program is built
        progs[name] = HeaMfmaProgram(spec, dev, storage=knobs.get("storage", "fp16"))
    ext()

    def prep(prog):
        xx = x.reshape(S, -1).float().contiguous()
        fr = prog._frags(params, K)
        part = prog._buf("part", S * prog.tiles_last * prog.C, torch.float32)
        stored = prog._forward(xx, params, fr, K, B, part, store_last=True)
        wread = torch.randn(S, prog.C, device=dev, generator=None) / B
        gslab = prog._buf("gslab", S * prog.slab_tiles * prog.n_gradops * 32, torch.int64)
        return xx, fr, stored, wread, gslab

    state = {}
    for name, knobs in variants:
        set_knobs(knobs)
        prog = progs[name]
        for _ in range(2):
            prog.loss_and_grads(x, y, w, params, spec)
        state[name] = prep(prog)
    torch.cuda.synchronize()
    res = {name: {"step": [], "adjoint": []} for name, _ in variants}

    def timed(fn):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        fn()
        a.record()
        for _ in range(args.iters):
            fn()
        b.record()
        torch.cuda.synchronize()
        return a.elapsed_time(b) / args.iters

    for _ in range(args.rounds):
        for name, knobs in variants:
            set_knobs(knobs)
            prog = progs[name]
            xx, fr, stored, wread, gslab = state[name]
            res[name]["step"].append(timed(lambda: prog.loss_and_grads(x, y, w, params, spec)))
            res[name]["adjoint"].append(timed(lambda: prog._adjoint(xx, params, fr, K, B, stored, wread, gslab)))
    out = {"qubits": args.qubits, "layers": args.layers, "clients": K, "batch": B, "rounds": args.rounds}
    for name, r in res.items():
        out[name] = {k: {"median_ms": round(statistics.median(v), 4), "min_ms": round(min(v), 4)} for k, v in r.items()}
    # bitwise agreement of the variants' gradients (same storage): the launch variants change scheduling only
    ref = None
    for name, knobs in variants:
        set_knobs(knobs)
        z, gr = progs[name].vjp(x, params[:, : spec.n_theta], w[..., None].expand(K, B, 3).contiguous() / 3)
        key = knobs.get("storage", "fp16")
        if ref is None or ref[0] != key:
            ref = (key, gr)
        else:
            out[name]["bitwise_vs_first_same_storage"] = bool(torch.equal(gr, ref[1]))
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
