"""Where does the 20q OP_L1PROD run differ between two identical vjp calls?  Dumps the differing gradient-slab
entries (sample, tile, gradient record, slot) of the MFMA engine's adjoint."""
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
    n, L = int(sys.argv[1]), int(sys.argv[2])
    spec = VQCSpec(n, L, 3)
    K, B = (int(sys.argv[3]), int(sys.argv[4])) if len(sys.argv) > 4 else (3, 4)
    x, params, wr = _inputs(spec, K, B, seed=11)
    xx, th, ww = x.to(dev), params[:, : spec.n_theta].to(dev), wr.to(dev)
    prog = HeaMfmaProgram(spec, dev)
    slabs = []
    for _ in range(3):
        prog.vjp(xx, th, ww)
        torch.cuda.synchronize()
        slabs.append(prog._ws["gslab"].clone().view(K * B, prog.slab_tiles, prog.n_gradops, 32).cpu())
    d = (slabs[0] != slabs[1]) | (slabs[0] != slabs[2])
    idx = d.nonzero()
    print(json.dumps({"K": K, "B": B, "wgs": K * B << (n - prog.adj_tile_bits), "n": n, "n_gradops": prog.n_gradops, "slab_tiles": prog.slab_tiles, "ndiff": int(d.sum()),
                      "by_record": torch.bincount(idx[:, 2], minlength=prog.n_gradops).tolist() if len(idx) else [],
                      "by_slot": torch.bincount(idx[:, 3], minlength=32).tolist() if len(idx) else [],
                      "by_tile": torch.bincount(idx[:, 1], minlength=prog.slab_tiles).tolist()[:16] if len(idx) else [],
                      "first": idx[:8].tolist(),
                      "vals": [[int(slabs[r][tuple(i)]) for r in range(3)] for i in idx[:8].tolist()]}), flush=True)


if __name__ == "__main__":
    main()
