"""OP_L1PROD accuracy check on the GPU: gradient errors of the MFMA engine (one-sample and paired forward) against
the dense float64 oracle, with QFEDX_HEA_L1PROD=1 (product-state layer-1 gradients) and =0 (per-group GRAD_L1)."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch
    from tests.test_gpu_hea import _dense, _inputs
    from qfedx_amd.models.vqc import VQCSpec
    from qfedx_amd.ops.hea_mfma import HeaMfmaProgram
    dev = torch.device("cuda", 0)
    for n, L in ((16, 3), (20, 2)):
        spec = VQCSpec(n, L, 3)
        K, B = 3, 4
        x, params, wr = _inputs(spec, K, B, seed=11)
        ez_ref, g_ref = _dense(spec, x.double(), params.double(), wr.double())
        xx, th, ww = x.to(dev), params[:, : spec.n_theta].to(dev), wr.to(dev)
        for l1p in ("1", "0"):
            os.environ["QFEDX_HEA_L1PROD"] = l1p
            os.environ["QFEDX_HEA_FWD_PAIR"] = "1"
            prog = HeaMfmaProgram(spec, dev)
            out = {}
            for pair in (True, False):
                prog.pair_kernel = pair
                z, g = prog.vjp(xx, th, ww)
                z2, g2 = prog.vjp(xx, th, ww)
                torch.cuda.synchronize()
                gc = g.cpu().double()
                err = (gc - g_ref).abs()
                out["pair" if pair else "single"] = {
                    "max_err": float(err.max()), "argmax": int(err.argmax()), "det": bool(torch.equal(g, g2)),
                    "zerr": float((z.cpu().reshape(K, B, -1).double() - ez_ref).abs().max())}
                out["g_" + ("pair" if pair else "single")] = gc
            d = (out.pop("g_pair") - out.pop("g_single")).abs()
            print(json.dumps({"n": n, "L": L, "l1prod": l1p, "pair_vs_single": float(d.max()),
                              "pair_vs_single_arg": int(d.argmax()), "max_grad": float(g_ref.abs().max()), **out}),
                  flush=True)


if __name__ == "__main__":
    main()
