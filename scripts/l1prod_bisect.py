"""OP_L1PROD determinism bisection (round 4): for each program variant, three identical vjp calls on one fresh
program; prints, per gradient record, how many slab entries differ between calls (records of the last group op vs
the layer-1 product-state op), and the gradient differences against the GRAD_L1 program.
Variants: l1prod (last group op un-applies lambda only, fused cross at its output) and l1prod_psi
(QFEDX_HEA_L1PROD_PSI=1: the last group op keeps un-applying psi, transposed form as in the default program)."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch
    from tests.test_gpu_hea import _inputs
    from qfedx_amd.models.vqc import VQCSpec
    from qfedx_amd.ops.hea_mfma import HeaMfmaProgram
    dev = torch.device("cuda", 0)
    n, L, K, B = [int(v) for v in (sys.argv[1:5] if len(sys.argv) >= 5 else (16, 3, 16, 8))]
    spec = VQCSpec(n, L, 3)
    x, params, wr = _inputs(spec, K, B, seed=11)
    xx, th, ww = x.to(dev), params[:, : spec.n_theta].to(dev), wr.to(dev)
    os.environ["QFEDX_HEA_L1PROD"] = "0"
    ref = HeaMfmaProgram(spec, dev)
    _, g_ref = ref.vjp(xx, th, ww)
    from qfedx_amd.ops._ext import ext
    diags = [int(v) for v in os.environ.get("L1_DIAGS", "0").split(",")]
    variants = [(f"l1prod_d{d}", {"QFEDX_HEA_L1PROD": "1", "QFEDX_HEA_L1PROD_PSI": "0"}, d) for d in diags]
    variants += [("gradl1", {"QFEDX_HEA_L1PROD": "0", "QFEDX_HEA_L1PROD_PSI": "0"}, 0)]
    for name, env, diag in variants:
        os.environ.update(env)
        ext().hea_set_knob("diag", diag)
        prog = HeaMfmaProgram(spec, dev)
        import qfedx_amd.ops.hea_mfma as hm
        nwg = K * B * prog.slab_tiles
        dbg = torch.zeros(512 + nwg * 512 * 16, dtype=torch.int64, device=dev)
        dumps = []
        hm._NODBG = dbg if diag & 896 else torch.zeros(0, dtype=torch.int64, device=dev)
        gs, slabs = [], []
        for _ in range(3):
            _, g = prog.vjp(xx, th, ww)
            torch.cuda.synchronize()
            gs.append(g.clone())
            slabs.append(prog._ws["gslab"].clone().reshape(K * B, prog.slab_tiles, prog.n_gradops, 32))
            if diag & 256:
                dumps.append(dbg[512:].view(torch.float32).reshape(nwg, 512, 32).clone())
        per_rec = [int(((slabs[0] != slabs[1]) | (slabs[1] != slabs[2]))[:, :, r].sum()) for r in range(prog.n_gradops)]
        per_tile = [int(((slabs[0] != slabs[1]) | (slabs[1] != slabs[2]))[:, t].sum()) for t in range(prog.slab_tiles)]
        if dumps:
            names = ["c", "lamsum", "hbsum"] + [f"T{i}" for i in range(9)] + ["mu", "e_nsc", "w0", "w1"]
            first = {}
            for q, nm in enumerate(names):
                dq = (dumps[0][..., 2 * q:2 * q + 2] != dumps[1][..., 2 * q:2 * q + 2]).any(-1) | \
                     (dumps[1][..., 2 * q:2 * q + 2] != dumps[2][..., 2 * q:2 * q + 2]).any(-1)
                first[nm] = int(dq.sum())
            print(json.dumps({"variant": name, "dump_diff_counts": first}), flush=True)
            d01 = (slabs[0] != slabs[1])
            print(json.dumps({"slab_diff_rec_jq": {f"{r}.{j}": int(d01[:, :, r, 8 * j:8 * j + 8].sum())
                                                   for r in range(5, 9) for j in range(4)}}), flush=True)
            dq = (dumps[0] != dumps[1]).any(-1)
            idx = dq.nonzero()[:8].tolist()
            for wg, t in idx:
                print(json.dumps({"wg": wg, "tid": t, "call0": dumps[0][wg, t, 24:32].tolist(),
                                  "call1": dumps[1][wg, t, 24:32].tolist()}), flush=True)
            # thread 0 of workgroup 0 writes rec[gidx0] entries 0, 1 (bit 0, x = 0, y = 0): recompute on the host
            r = dumps[0][0, 0]
            mu, nsc, w0 = (float(r[24]), float(r[25])), float(r[27]), (float(r[28]), float(r[29]))
            re = w0[0] * mu[0] + w0[1] * mu[1]
            print(json.dumps({"host_expected_ent0": round(re * nsc), "w0": w0, "mu": mu, "nsc": nsc}), flush=True)
            # slab entries of the layer-1 records that differ between calls 0 and 1, with the writer's mu
            sd = (slabs[0] != slabs[1]).nonzero()[:12].tolist()
            for sm, tl, rec, ent in sd:
                print(json.dumps({"sample": sm, "tile": tl, "rec": rec, "ent": ent,
                                  "v": [int(slabs[c][sm, tl, rec, ent]) for c in range(3)]}), flush=True)
        print(json.dumps({"variant": name, "n": n, "K": K, "B": B, "n_gradops": prog.n_gradops,
                          "diff_per_record": per_rec, "diff_per_tile": per_tile,
                          "dbg": dbg[:5].tolist(),
                          "call0_vs_1": float((gs[0] - gs[1]).abs().max()),
                          "call1_vs_2": float((gs[1] - gs[2]).abs().max()),
                          "vs_gradl1": [float((g - g_ref).abs().max()) for g in gs]}), flush=True)


if __name__ == "__main__":
    main()
