"""OP_L1PROD debug build (ab/v3): per-workgroup intermediates written into unused slab slots; which differ between
the first and a later identical vjp call?"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
if os.environ.get("QFX_PKG_ROOT"):
    sys.path.insert(0, os.environ["QFX_PKG_ROOT"])


def main():
    import torch
    from tests.test_gpu_hea import _inputs
    from qfedx_amd.models.vqc import VQCSpec
    from qfedx_amd.ops.hea_mfma import HeaMfmaProgram
    dev = torch.device("cuda", 0)
    spec = VQCSpec(20, 2, 3)
    K, B = 3, 4
    x, params, wr = _inputs(spec, K, B, seed=11)
    xx, th, ww = x.to(dev), params[:, : spec.n_theta].to(dev), wr.to(dev)
    prog = HeaMfmaProgram(spec, dev)
    slabs = []
    for _ in range(2):
        prog.vjp(xx, th, ww)
        torch.cuda.synchronize()
        slabs.append(prog._ws["gslab"].clone().view(K * B, prog.slab_tiles, prog.n_gradops, 32).cpu())
    a, b = slabs
    real = (a[:, :, 3:6, :] != b[:, :, 3:6, :]).any(-1).any(-1)   # WGs whose real entries differ
    dbg = a[:, :, 6, 8:20] != b[:, :, 6, 8:20]
    names = ["outer", "hb5", "rj3", "fw12", "c0", "scr0", "scr_5_7", "rj12", "fw3b", "rho_scale", "c77", "scr2_77"]
    out = {"wg_bad": int(real.sum()), "wg_total": int(real.numel())}
    for i, nm in enumerate(names):
        out[nm] = [int(dbg[..., i][real].sum()), int(dbg[..., i][~real].sum())]
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
