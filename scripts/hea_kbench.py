"""Per-launch timing of the MFMA statevector engine (one local training step of K clients x B samples).

python scripts/hea_kbench.py [--qubits 16 --layers 3 --clients 64 --batch 32 --iters 20]
Prints one JSON line: per-kernel ms (frags, forward passes, readout_ce, adjoint passes, grad reduce),
the whole step, and effective HBM bandwidth of each pass (fp16 state bytes moved / time).
"""
import argparse
import json
import os
import sys

# QFX_PKG_ROOT: import the package from another built tree (scripts/ab_kbench.sh)
sys.path.insert(0, os.environ.get("QFX_PKG_ROOT") or os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--qubits", type=int, default=16)
    ap.add_argument("--layers", type=int, default=3)
    ap.add_argument("--clients", type=int, default=64)
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--precision", action="store_true", help="also report errors against the fp32 VALU engine")
    args = ap.parse_args()
    import torch
    from qfedx_amd.models.vqc import VQCSpec
    from qfedx_amd.ops._ext import ext
    from qfedx_amd.ops.hea_mfma import _NODBG, HeaMfmaProgram

    dev = torch.device("cuda", 0)
    spec = VQCSpec(args.qubits, args.layers, 3)
    prog = HeaMfmaProgram(spec, dev)
    K, B = args.clients, args.batch
    S = K * B
    g = torch.Generator().manual_seed(0)
    x = (torch.rand(K, B, args.qubits, generator=g) * 3).to(dev)
    y = torch.randint(0, 3, (K, B), generator=g).to(dev)
    w = torch.full((K, B), 1.0 / B, device=dev)
    params = torch.stack([spec.init_params(k) for k in range(K)]).to(dev)
    for _ in range(3):
        prog.loss_and_grads(x, y, w, params, spec)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(args.iters):
        prog.loss_and_grads(x, y, w, params, spec)
    e1.record()
    torch.cuda.synchronize()
    step_ms = e0.elapsed_time(e1) / args.iters

    # per-pass timing: replay the launches one at a time
    C = ext()
    xx = x.reshape(S, -1).float().contiguous()
    fr = prog._frags(params, K)
    part = prog._buf("part", S * prog.tiles_last * prog.C, torch.float32)
    stored = prog._forward(xx, params, fr, K, B, part, store_last=True)
    wread = torch.randn(S, prog.C, device=dev) / B
    gslab = prog._buf("gslab", S * prog.slab_tiles * prog.n_gradops * 32, torch.int64)
    empty = torch.empty(0, dtype=torch.int32, device=dev)
    fempty = torch.empty(0, dtype=torch.float32, device=dev)
    J = prog.n_passes
    N = S << prog.n
    res = {"step_ms": round(step_ms, 4), "n_passes": J, "samples": S}

    def timeit(fn, name, nbytes):
        fn()
        torch.cuda.synchronize()
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        for _ in range(args.iters):
            fn()
        b.record()
        torch.cuda.synchronize()
        ms = a.elapsed_time(b) / args.iters
        res[name] = {"ms": round(ms, 4), "GBps": round(nbytes / ms / 1e6, 1)}

    timeit(lambda: prog._frags(params, K), "frags", 0)
    R = getattr(prog, "fwd_last", J - 1)                # forward passes after R are identities (older trees: none)
    for j, ent in enumerate(prog.passes):
        if j > R:
            break
        p, fwd = ent[0], ent[1]
        out = prog._buf(f"psi{j}", N, torch.int32)
        psi_in = stored[j - 1] if j > 0 else empty
        geom = prog._geom(p, j == 0, False, True, False, B, params.shape[1], S, xx.shape[1], K)
        nb = 4 * N * ((j > 0) + 1)
        timeit(lambda: C.hea_pass(False, fwd[0], fwd[1], fwd[2], geom, prog.scale, psi_in, out, empty, empty, xx, params, fr, fempty,
                                  part if j == R else fempty, fempty, _NODBG), f"fwd{j}", nb)
    lam = [prog._buf("lam0", N, torch.int32), prog._buf("lam1", N, torch.int32)]
    for j in range(J - 1, -1, -1):
        ent = prog.passes[j]                          # (fwd pass, fwd prog, adj prog[, adj pass]) (older trees: 3)
        adj, p = ent[2], ent[-1] if len(ent) > 3 else ent[0]
        geom = prog._geom(p, False, j < J - 1, False, j > 0, B, params.shape[1], S, xx.shape[1], K,
                          n_regions=prog.n_regions[j])
        lin = lam[(j + 1) % 2] if j < J - 1 else empty
        lout = lam[j % 2] if j > 0 else empty
        nb = 4 * N * (1 + (j < J - 1) + (j > 0))
        timeit(lambda: C.hea_pass(True, adj[0], adj[1], adj[2], geom, prog.scale, stored[j], empty, lin, lout,
                                  xx, params, fr, wread, fempty, gslab, _NODBG), f"adj{j}", nb)
    grad = torch.zeros(K, params.shape[1], device=dev)
    timeit(lambda: C.hea_grad_reduce(gslab, prog.slab_tiles, prog.n_gradops, prog.gmeta, B, K, params, grad,
                                     params.shape[1]), "grad_reduce", 0)
    if args.precision:
        # max |error| of <Z> and of the gradient against the fp32 VALU engine (as bench.py's precision fields)
        from qfedx_amd.ops.engine import VQCEngine
        from qfedx_amd.ops.statevec_hip import HipProgram
        eng = VQCEngine(spec, dev, "hip", "mfma")
        kp = min(K, 16)
        xang = spec.encode_features(x[:kp].float())
        th = params[:kp, : spec.n_theta].float().contiguous()
        wp = (torch.randn(kp * B, spec.n_classes, generator=g) / B).to(dev)
        z_m, g_m = eng.hip.vjp(xang, th, wp)
        ref = HipProgram(eng.ops, eng.coef, spec.n_qubits, spec.readout, dev, n_theta=spec.n_theta,
                         state_dtype="fp32", jit=False, x_width=spec.x_width)
        z_r, g_r = ref.vjp(xang, th, wp)
        res["max_abs_err_expz"] = float((z_m - z_r).abs().max())
        res["max_abs_err_grad"] = float((g_m - g_r).abs().max())
        res["rms_err_expz"] = float((z_m - z_r).pow(2).mean().sqrt())
        res["rms_err_grad"] = float((g_m - g_r).pow(2).mean().sqrt())
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
