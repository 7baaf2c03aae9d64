"""Stored forward pass outputs of the MFMA engine with and without chained APPLY2 pairs (QFEDX_HEA_PAIR=1 vs 0):
max difference per pass and where the differing amplitudes sit.  python scripts/pair_state_diff.py n L"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import numpy as np
    import torch
    from qfedx_amd.models.vqc import VQCSpec
    from qfedx_amd.ops.hea_mfma import HeaMfmaProgram
    from tests.test_gpu_hea import _inputs
    n, L = int(sys.argv[1]), int(sys.argv[2])
    K, B = 1, 2
    spec = VQCSpec(n, L, 3)
    x, params, _ = _inputs(spec, K, B, seed=5)
    dev = torch.device("cuda", 0)
    outs = {}
    for mask in (0, 1):
        os.environ["QFEDX_HEA_PAIR"] = str(mask)
        prog = HeaMfmaProgram(spec, dev)
        xx, th, K_, B_ = prog._prep(x.to(dev), params[:, : spec.n_theta].to(dev))
        th = torch.cat([th, th.new_zeros(K, spec.n_theta + 2 * spec.n_classes - th.shape[1])], 1)
        fr = prog._frags(th, K)
        part = prog._buf("part", K * B * prog.tiles_last * prog.C, torch.float32)
        st = prog._forward(xx, th, fr, K, B, part, store_last=True)
        torch.cuda.synchronize()
        outs[mask] = ([s.view(torch.float16).float().cpu().clone() for s in st],
                      [[int(c) for c in p[1][0][:, 0].cpu()] for p in prog.passes],
                      [(p[0].c, p[0].lo, p[0].hi) for p in prog.passes])
    for j, (a, b) in enumerate(zip(outs[0][0], outs[1][0])):
        d = (a - b).abs().view(B, -1, 2).amax(-1)      # per amplitude
        idx = torch.nonzero(d[0] > 1e-2).flatten()
        rec = {"pass": j, "max_diff": float(d.max()), "n_bad": int((d > 1e-2).sum()), "fwd_ops": outs[1][1][j],
               "tile": outs[1][2][j], "first_bad": [int(i) for i in idx[:12]],
               "bad_bit_or": int(np.bitwise_or.reduce(idx.numpy())) if len(idx) else 0,
               "bad_bit_and": int(np.bitwise_and.reduce(idx.numpy())) if len(idx) else 0}
        print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
