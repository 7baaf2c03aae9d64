"""Measured error of the MFMA engine (fp16 / bf16 storage) against the float64 dense oracle, per test shape of
tests/test_gpu_hea.py, next to the tile-exact emulator's error (fp16 / bf16 rounding after every op).  The GPU
tests' tolerances are set from this table (about 3x the measured error), so a precision regression - a dropped
lo half of the gate split, an extra rounding - fails them.

    python scripts/hea_err_table.py > gpurun_out/hea_err_table.txt
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402

from qfedx_amd.models.vqc import VQCSpec  # noqa: E402
from qfedx_amd.ops import hea_plan as hp  # noqa: E402
from qfedx_amd.ops.hea_mfma import HeaMfmaProgram  # noqa: E402
from tests.test_gpu_hea import _dense, _inputs  # noqa: E402

CASES = [(8, 2, 14, True, "ry"), (10, 3, 14, True, "ry"), (10, 3, 8, True, "ry"), (11, 2, 8, False, "rx"),
         (12, 4, 9, True, "ry"), (9, 1, 8, True, "rz"), (13, 3, 10, True, "ry"), (16, 3, 14, True, "ry"),
         (12, 1, 9, True, "ry"), (20, 1, 14, True, "rx")]


def main():
    dev = torch.device("cuda", 0)
    print("n L tile chain feat storage | err_z err_g/scale | emu_z emu_g/scale")
    for n, L, tile, chain, feat in CASES:
        spec = VQCSpec(n, L, 3, feature_map=feat, entangler="chain" if chain else "none")
        K, B = 2, 3
        x, params, wr = _inputs(spec, K, B)
        ez_ref, g_ref = _dense(spec, x.double(), params.double(), wr.double())
        scale = max(1.0, float(g_ref.abs().max()))
        for st in ("fp16", "bf16"):
            prog = HeaMfmaProgram(spec, dev, tile_bits=tile, storage=st)
            z, g = prog.vjp(x.to(dev), params[:, : spec.n_theta].to(dev), wr.to(dev))
            torch.cuda.synchronize()
            ez = np.abs(z.cpu().reshape(K, B, -1).numpy() - ez_ref.numpy()).max()
            eg = np.abs(g.cpu().numpy() - g_ref.numpy()).max() / scale
            emu = ""
            if n <= 16:
                ze, ge = hp.emulate(prog.plan, x.double().numpy(), params.double().numpy(), wr.double().numpy(),
                                    storage=st)
                emu = f"{np.abs(ze - ez_ref.numpy()).max():.2e} {np.abs(ge - g_ref.numpy()).max() / scale:.2e}"
            print(f"{n} {L} {tile} {chain} {feat} {st} | {ez:.2e} {eg:.2e} | {emu}", flush=True)


if __name__ == "__main__":
    main()
