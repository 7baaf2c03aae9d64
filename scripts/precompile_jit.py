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
    (3, 1, 3, "chain", False, False, "amplitude"), (5, 2, 3, "ring", False, False, "amplitude"),
    (10, 2, 3, "chain", False, False, "amplitude"), (13, 2, 3, "ring", False, False, "amplitude"),
    (16, 2, 3, "chain", False, False, "amplitude"), (3, 3, 3, "chain", False, False, "amplitude"),
]


def build(cfg):
    import torch
    from qfedx_amd.models.vqc import VQCSpec
    from qfedx_amd.ops import statevec_hip as sh
    from qfedx_amd.ops._ext import ext
    n, L, ncls, ent, noisy = cfg[:5]
    bf16 = bool(cfg[5]) if len(cfg) > 5 else False
    fm = cfg[6] if len(cfg) > 6 else "ry"
    C = ext()
    t0 = time.time()
    spec = VQCSpec(n, L, ncls, feature_map=fm, entangler=ent, noisy=noisy)
    ops, coef = spec.program()
    R = sh.choose_R(n)
    modes = ((0, 2), (0, 3), (2, 0)) + (((1, 2), (1, 3)) if spec.amplitude else ())
    for mode, fin in modes:
        blob = C.plan(torch.from_numpy(ops), torch.from_numpy(coef), n, R, sh.KMAX, spec.readout,
                      spec.n_theta, mode, fin)
        for p in range(int(blob[1])):
            C.jit_prepare(blob, p, mode == 2, sh.JIT_CACHE, sh.CSRC, sh.ARCH, bf16)
    return (f"n={n} L={L} C={ncls} {ent}{' noisy' if noisy else ''}{' bf16' if bf16 else ''}"
            f"{' ' + fm if spec.amplitude else ''}: ok ({time.time() - t0:.1f}s)")


def from_config(path, overrides):
    """The kernel set one experiment config needs (``--config file.yaml key=value ...``)."""
    from qfedx_amd.config import load_config
    cfg = load_config(path, overrides)
    m, nz = cfg.model, cfg.noise
    if m.kind != "vqc":
        return []
    from qfedx_amd.quantum.noise import NoiseModel
    model = NoiseModel.from_config(nz, 0)
    noisy = model is not None and model.gate_noise
    return [(m.n_qubits, m.n_layers, m.n_classes, m.entangler, noisy, m.state_dtype == "bf16", m.feature_map)]


def main():
    t0 = time.time()
    todo = CONFIGS
    if len(sys.argv) > 2 and sys.argv[1] == "--config":
        todo = from_config(sys.argv[2], sys.argv[3:])
    with Pool(max(1, min(6, os.cpu_count() or 1, len(todo)))) as pool:
        for line in pool.imap_unordered(build, todo):
            print(line, flush=True)
    print(f"done in {time.time() - t0:.1f}s")


if __name__ == "__main__":
    main()
