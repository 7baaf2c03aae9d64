"""ab/v6 (poisoned scratch before OP_L1PROD): NaN / garbage in the gradients or the layer-1 slab rows would mean the op
reads LDS it never wrote; also repeats the first-call determinism check at 20q x 2L, K=3, B=4."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
if os.environ.get("QFX_PKG_ROOT"):
    sys.path.insert(0, os.environ["QFX_PKG_ROOT"])


def main():
    import torch
    from tests.test_gpu_hea import _dense, _inputs
    from qfedx_amd.models.vqc import VQCSpec
    from qfedx_amd.ops.hea_mfma import HeaMfmaProgram
    dev = torch.device("cuda", 0)
    for n, L, K, B in ((20, 2, 3, 4), (16, 3, 3, 4)):
        spec = VQCSpec(n, L, 3)
        x, params, wr = _inputs(spec, K, B, seed=11)
        xx, th, ww = x.to(dev), params[:, : spec.n_theta].to(dev), wr.to(dev)
        prog = HeaMfmaProgram(spec, dev)
        gs, slabs = [], []
        for _ in range(3):
            _, g = prog.vjp(xx, th, ww)
            torch.cuda.synchronize()
            gs.append(g.cpu().double())
            slabs.append(prog._ws["gslab"].clone().view(K * B, prog.slab_tiles, prog.n_gradops, 32).cpu())
        _, g_ref = _dense(spec, x.double(), params.double(), wr.double())
        print(json.dumps({"n": n, "nan": [bool(torch.isnan(g).any()) for g in gs],
                          "err": [float((g - g_ref).abs().max()) for g in gs],
                          "ndiff12": int((slabs[0] != slabs[1]).sum()), "ndiff23": int((slabs[1] != slabs[2]).sum())}),
              flush=True)


if __name__ == "__main__":
    main()
