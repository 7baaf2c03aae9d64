"""Pre-build circuit-specialised kernels (hiprtc, gfx950) for the standard configs into build/jit so a
fresh GPU box starts with a warm code-object cache.  Runs on a CPU-only host (parallel workers)."""
import os
import sys
import time
from multiprocessing import Pool

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

CONFIGS = [  # (n, L, C, entangler, noisy)
    (16, 3, 3, "chain", False), (20, 3, 3, "chain", False), (20, 2, 3, "chain", False), (24, 2, 3, "chain", False),
    (24, 1, 2, "chain", False), (4, 2, 3, "chain", False), (4, 2, 2, "chain", False), (2, 1, 2, "chain", False),
    (3, 2, 3, "chain", False), (5, 2, 3, "chain", False), (6, 2, 3, "chain", False),
    (6, 2, 3, "ring", False), (8, 2, 3, "chain", False), (8, 3, 3, "chain", False), (10, 2, 3, "chain", False),
    (11, 2, 3, "chain", False), (11, 2, 3, "ring", False), (12, 2, 3, "ring", False), (13, 2, 3, "chain", False),
    (14, 2, 3, "chain", False), (16, 2, 3, "chain", False), (16, 3, 3, "chain", True),
    (4, 2, 3, "chain", True), (7, 2, 3, "chain", True), (12, 2, 3, "chain", True), (3, 1, 2, "chain", True),
    (16, 3, 3, "chain", False, True), (6, 2, 3, "chain", False, True), (13, 2, 3, "chain", False, True),
    (20, 2, 3, "chain", False, True),
]


def build(cfg):
    import torch
    from qfedx_amd.models.vqc import VQCSpec
    from qfedx_amd.ops import statevec_hip as sh
    from qfedx_amd.ops._ext import ext
    n, L, ncls, ent, noisy = cfg[:5]
    bf16 = bool(cfg[5]) if len(cfg) > 5 else False
    C = ext()
    t0 = time.time()
    spec = VQCSpec(n, L, ncls, entangler=ent, noisy=noisy)
    ops, coef = spec.program()
    R = sh.choose_R(n)
    for mode, fin in ((0, 2), (0, 3), (2, 0)):
        blob = C.plan(torch.from_numpy(ops), torch.from_numpy(coef), n, R, sh.KMAX, spec.readout,
                      spec.n_theta, mode, fin)
        for p in range(int(blob[1])):
            C.jit_prepare(blob, p, mode == 2, sh.JIT_CACHE, sh.CSRC, sh.ARCH, bf16)
    return f"n={n} L={L} C={ncls} {ent}{' noisy' if noisy else ''}{' bf16' if bf16 else ''}: ok ({time.time() - t0:.1f}s)"


def main():
    t0 = time.time()
    with Pool(min(6, os.cpu_count() or 1)) as pool:
        for line in pool.imap_unordered(build, CONFIGS):
            print(line, flush=True)
    print(f"done in {time.time() - t0:.1f}s")


if __name__ == "__main__":
    main()
