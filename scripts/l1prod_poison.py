"""OP_L1PROD determinism diagnostics (round 4): one process per LDS poison word (QFEDX_HEA_POISON is read once per
process).  For each shape: three identical vjp calls of a fresh L1PROD program and one of a GRAD_L1 program; prints the
max gradient differences between calls and against GRAD_L1, and how many slab entries differ between calls."""
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
    shapes = [(16, 3, 64, 32), (20, 3, 3, 4), (16, 3, 16, 8)]
    for n, L, K, B in shapes:
        spec = VQCSpec(n, L, 3)
        x, params, wr = _inputs(spec, K, B, seed=11)
        xx, th, ww = x.to(dev), params[:, : spec.n_theta].to(dev), wr.to(dev)
        os.environ["QFEDX_HEA_L1PROD"] = "0"
        ref = HeaMfmaProgram(spec, dev)
        _, g_ref = ref.vjp(xx, th, ww)
        os.environ["QFEDX_HEA_L1PROD"] = "1"
        prog = HeaMfmaProgram(spec, dev)
        gs, slabs = [], []
        for _ in range(3):
            _, g = prog.vjp(xx, th, ww)
            torch.cuda.synchronize()
            gs.append(g.clone())
            slabs.append(prog._ws["gslab"].clone())
        d01 = float((gs[0] - gs[1]).abs().max())
        d12 = float((gs[1] - gs[2]).abs().max())
        ds = int((slabs[0] != slabs[1]).sum()) + int((slabs[1] != slabs[2]).sum())
        print(json.dumps({"n": n, "L": L, "K": K, "B": B, "poison": os.environ.get("QFEDX_HEA_POISON", "0"),
                          "wgs": K * B << (n - prog.adj_tile_bits),
                          "call0_vs_1": d01, "call1_vs_2": d12, "slab_diffs": ds,
                          "vs_gradl1": [float((g - g_ref).abs().max()) for g in gs],
                          "max_grad": float(g_ref.abs().max()),
                          "finite": bool(all(torch.isfinite(g).all() for g in gs))}), flush=True)


if __name__ == "__main__":
    main()
