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
    for name, env in (("l1prod", {"QFEDX_HEA_L1PROD": "1", "QFEDX_HEA_L1PROD_PSI": "0"}),
                      ("l1prod_psi", {"QFEDX_HEA_L1PROD": "1", "QFEDX_HEA_L1PROD_PSI": "1"}),
                      ("gradl1", {"QFEDX_HEA_L1PROD": "0", "QFEDX_HEA_L1PROD_PSI": "0"})):
        os.environ.update(env)
        prog = HeaMfmaProgram(spec, dev)
        gs, slabs = [], []
        for _ in range(3):
            _, g = prog.vjp(xx, th, ww)
            torch.cuda.synchronize()
            gs.append(g.clone())
            slabs.append(prog._ws["gslab"].clone().reshape(K * B, prog.slab_tiles, prog.n_gradops, 32))
        per_rec = [int(((slabs[0] != slabs[1]) | (slabs[1] != slabs[2]))[:, :, r].sum()) for r in range(prog.n_gradops)]
        per_tile = [int(((slabs[0] != slabs[1]) | (slabs[1] != slabs[2]))[:, t].sum()) for t in range(prog.slab_tiles)]
        print(json.dumps({"variant": name, "n": n, "K": K, "B": B, "n_gradops": prog.n_gradops,
                          "diff_per_record": per_rec, "diff_per_tile": per_tile,
                          "call0_vs_1": float((gs[0] - gs[1]).abs().max()),
                          "call1_vs_2": float((gs[1] - gs[2]).abs().max()),
                          "vs_gradl1": [float((g - g_ref).abs().max()) for g in gs]}), flush=True)


if __name__ == "__main__":
    main()
