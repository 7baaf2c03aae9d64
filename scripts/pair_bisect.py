"""Which chained pair kind breaks a shape on the GPU: vjp of the MFMA engine against the dense oracle with pairing
restricted to one kind at a time (QFEDX_HEA_PAIR mask: 1 APPLY2, 2 BACK2, 4 GRAD2).  python scripts/pair_bisect.py n L"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import numpy as np
    import torch
    from qfedx_amd.models.vqc import VQCSpec
    from qfedx_amd.ops.hea_mfma import HeaMfmaProgram
    from tests.test_gpu_hea import _dense, _inputs
    n, L = int(sys.argv[1]), int(sys.argv[2])
    K, B = 1, 2
    spec = VQCSpec(n, L, 3)
    x, params, wr = _inputs(spec, K, B, seed=5)
    ez, gr = _dense(spec, x.double(), params.double(), wr.double())
    dev = torch.device("cuda", 0)
    for mask in [int(m) for m in (sys.argv[3] if len(sys.argv) > 3 else '0,1,2,4,7').split(',')]:
        os.environ["QFEDX_HEA_PAIR"] = str(mask)
        prog = HeaMfmaProgram(spec, dev)
        z, g = prog.vjp(x.to(dev), params[:, : spec.n_theta].to(dev), wr.to(dev))
        torch.cuda.synchronize()
        dg = (g.cpu().double() - gr).abs()[0]
        bad = [int(i) for i in torch.nonzero(dg > 4e-3 * max(1.0, float(gr.abs().max()))).flatten()]
        print(json.dumps({"mask": mask, "ops": [[int(c) for c in p[2][0][:, 0].cpu()] for p in prog.passes],
                          "max_dz": float((z.cpu().double().reshape(K, B, -1) - ez).abs().max()),
                          "max_dg": float(dg.max()), "bad_params": bad}), flush=True)


if __name__ == "__main__":
    main()
