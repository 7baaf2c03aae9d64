"""ab/v4: lambda read twice across a barrier (mismatch count per workgroup in slot 31 of the last layer-1 record),
P terms written only after every read: is the first-call difference gone, and does lambda change under the op?"""
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
    for _ in range(3):
        prog.vjp(xx, th, ww)
        torch.cuda.synchronize()
        slabs.append(prog._ws["gslab"].clone().view(K * B, prog.slab_tiles, prog.n_gradops, 32).cpu())
    a, b = slabs[0], slabs[1]
    real = (a[:, :, 3:6, :] != b[:, :, 3:6, :]).any(-1).any(-1)
    hdiff = a[:, :, 6, 30] != b[:, :, 6, 30]
    rdiff = a[:, :, 6, 29] != b[:, :, 6, 29]
    print(json.dumps({"lam_hash_diff_bad": int(hdiff[real].sum()), "lam_hash_diff_good": int(hdiff[~real].sum()),
                      "rj3_diff_bad": int(rdiff[real].sum()), "rj3_diff_good": int(rdiff[~real].sum()),
                      "first_bad": real.nonzero()[:5].tolist()}), flush=True)
    print(json.dumps({"p_mismatch_wgs": [int((s[:, :, 6, 28] > 0).sum()) for s in slabs],
                      "p_mismatch_max": [int(s[:, :, 6, 28].max()) for s in slabs]}), flush=True)
    print(json.dumps({"wg_bad": int(real.sum()), "mism_call": [int((s[:, :, 6, 31] > 0).sum()) for s in slabs],
                      "mism_max": [int(s[:, :, 6, 31].max()) for s in slabs]}), flush=True)


if __name__ == "__main__":
    main()
