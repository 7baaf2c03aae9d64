"""cProfile of the host side of a bench_suite config's timed rounds (which Python work a round's enqueue costs).

python scripts/host_profile.py cfed128 [--rounds 50]   -> top functions by own time, then by cumulative time
"""
import cProfile
import os
import pstats
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    name = sys.argv[1]
    rounds = int(sys.argv[sys.argv.index("--rounds") + 1]) if "--rounds" in sys.argv else 50
    import bench_suite
    from bench import timed_rounds
    from qfedx_amd.api import setup
    from qfedx_amd.config import load_config
    path, ov, _, _ = bench_suite.SUITE[name]
    cfg = load_config(os.path.join(ROOT, path), ov)
    device, backend, world = setup(cfg)
    runner, _ = timed_rounds(cfg, device, backend, world, 3, 3)
    import torch
    torch.cuda.synchronize()
    pr = cProfile.Profile()
    pr.enable()
    for r in range(6, 6 + rounds):
        runner.run_round(r, sync=False)
    pr.disable()
    torch.cuda.synchronize()
    st = pstats.Stats(pr)
    st.sort_stats("tottime").print_stats(25)
    st.sort_stats("cumulative").print_stats(25)


if __name__ == "__main__":
    main()
