"""Ablation timing of the MFMA pass kernel: the same pass with its op list cut down, to attribute time to
tile load / generation, each group op, readout and store.  python scripts/hea_ablate.py"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch
    from qfedx_amd.models.vqc import VQCSpec
    from qfedx_amd.ops._ext import ext
    from qfedx_amd.ops.hea_mfma import HeaMfmaProgram

    dev = torch.device("cuda", 0)
    spec = VQCSpec(16, 3, 3)
    prog = HeaMfmaProgram(spec, dev)
    K, B = 64, 32
    S = K * B
    C = ext()
    x = (torch.rand(S, 16) * 3).to(dev)
    params = torch.stack([spec.init_params(k) for k in range(K)]).to(dev)
    fr = prog._frags(params, K)
    N = S << 16
    buf = torch.zeros(N, dtype=torch.int32, device=dev)
    buf2 = torch.zeros(N, dtype=torch.int32, device=dev)
    lam = torch.zeros(N, dtype=torch.int32, device=dev)
    part = torch.zeros(S * 64 * 3, device=dev)
    gslab = torch.zeros(S * prog.slab_tiles * prog.n_gradops * 32, dtype=torch.int64, device=dev)
    wread = torch.randn(S, 3, device=dev) / B
    empty = torch.empty(0, dtype=torch.int32, device=dev)
    fempty = torch.empty(0, dtype=torch.float32, device=dev)
    res = {}

    dbg = torch.zeros(8 * 64, dtype=torch.int64, device=dev)
    nodbg = torch.zeros(0, dtype=torch.int64)
    phases = {}

    def run(name, adj, p, ops, fidx, gen, load_lam, store_psi, store_lam):
        geom = prog._geom(p, gen, load_lam, store_psi, store_lam, B, params.shape[1], S, 16, K)
        dbg.zero_()
        C.hea_pass(adj, ops, fidx, geom, prog.scale, buf, buf2, lam, lam, x, params, fr, wread, part, gslab, dbg)
        torch.cuda.synchronize()
        d = dbg.view(8, 64).cpu()
        nz = int((d[0] != 0).sum())
        phases[name] = [int(v) for v in (d[:, 1:nz] - d[:, : nz - 1]).float().mean(0).round().tolist()]
        f = lambda: C.hea_pass(adj, ops, fidx, geom, prog.scale, buf, buf2, lam, lam, x, params, fr, wread, part, gslab,
                               nodbg)
        f()
        torch.cuda.synchronize()
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        for _ in range(10):
            f()
        b.record()
        torch.cuda.synchronize()
        res[name] = round(a.elapsed_time(b) / 10, 4)

    p0, (f0, fi0), (a0, ai0), pa0 = prog.passes[0]
    p1, (f1, fi1), (a1, ai1), pa1 = prog.passes[1]
    run("gen_only", False, p0, f0[:0], fi0[:0], True, False, False, False)
    run("gen_store", False, p0, f0[:0], fi0[:0], True, False, True, False)
    for k in (1, 3, 7):
        run(f"gen_{k}apply_store", False, p0, f0[:k].contiguous(), fi0[:k].contiguous(), True, False, True, False)
    run("load_only", False, p1, f1[:0], fi1[:0], False, False, False, False)
    run("load_readout", False, p1, f1[-1:].contiguous(), fi1[-1:].contiguous(), False, False, False, False)
    run("load_3apply_readout", False, p1, f1, fi1, False, False, False, False)
    nop = torch.zeros(64, 128, dtype=torch.int32, device=dev)
    nop[:, 0] = 9                                   # unknown code: the kernel only does the per-op bookkeeping
    nopf = torch.full((64,), -1, dtype=torch.int32, device=dev)
    run("gen_store_64nop", False, p0, nop, nopf, True, False, True, False)
    nopf2 = fi0[:1].repeat(64).contiguous()
    run("gen_store_64nop_frag", False, p0, nop, nopf2, True, False, True, False)
    run("adj1_full", True, pa1, a1, ai1, False, False, False, True)
    run("adj0_full", True, pa0, a0, ai0, False, True, False, False)
    run("adj0_load_only", True, pa0, a0[:0].contiguous(), ai0[:0].contiguous(), False, True, False, False)
    run("adj0_load_store", True, pa0, a0[:0].contiguous(), ai0[:0].contiguous(), False, True, False, True)
    run("adj0_1back", True, pa0, a0[:1].contiguous(), ai0[:1].contiguous(), False, True, False, False)
    run("adj0_4back", True, pa0, a0[:4].contiguous(), ai0[:4].contiguous(), False, True, False, False)
    run("adj0_5back", True, pa0, a0[:5].contiguous(), ai0[:5].contiguous(), False, True, False, False)
    run("adj0_5back_1grad", True, pa0, a0[:6].contiguous(), ai0[:6].contiguous(), False, True, False, False)
    run("adj0_load_64nop", True, pa0, nop, nopf, False, True, False, False)
    print(json.dumps(res), flush=True)
    for k, v in phases.items():
        print("phases", k, v, flush=True)
    print("adj0 ops:", [int(c) for c in a0[:, 0].tolist()], "adj1 ops:", [int(c) for c in a1[:, 0].tolist()])


if __name__ == "__main__":
    main()
