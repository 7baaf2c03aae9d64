"""Pre-build circuit-specialised kernels (hiprtc, gfx950) for the standard configs into build/jit so a
fresh GPU box starts with a warm code-object cache.  Runs on a CPU-only host."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from qfedx_amd.models.vqc import VQCSpec  # noqa: E402
from qfedx_amd.ops import statevec_hip as sh  # noqa: E402
from qfedx_amd.ops._ext import ext  # noqa: E402

CONFIGS = [  # (n, L, C, entangler)
    (16, 3, 3, "chain"), (20, 3, 3, "chain"), (24, 2, 3, "chain"), (4, 2, 3, "chain"), (4, 2, 2, "chain"),
    (2, 1, 2, "chain"), (3, 2, 3, "chain"), (6, 2, 3, "chain"), (6, 2, 3, "ring"), (8, 2, 3, "chain"),
    (8, 3, 3, "chain"), (10, 2, 3, "chain"), (12, 2, 3, "ring"), (13, 2, 3, "chain"), (14, 2, 3, "chain"),
    (16, 2, 3, "chain"),
]


def main():
    C = ext()
    t0 = time.time()
    for n, L, ncls, ent in CONFIGS:
        spec = VQCSpec(n, L, ncls, entangler=ent)
        ops, coef = spec.program()
        R = sh.choose_R(n)
        for mode, fin in ((0, 2), (0, 3), (2, 0)):
            blob = C.plan(torch.from_numpy(ops), torch.from_numpy(coef), n, R, sh.KMAX, spec.readout,
                          spec.n_theta, mode, fin)
            for p in range(int(blob[1])):
                C.jit_prepare(blob, p, mode == 2, sh.JIT_CACHE, sh.CSRC, sh.ARCH)
        print(f"n={n} L={L} C={ncls} {ent}: ok ({time.time() - t0:.1f}s)", flush=True)


if __name__ == "__main__":
    main()
