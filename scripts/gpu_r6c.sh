#!/bin/bash
# GPU suite with the round-6 tests (CC4 side-stream gather, small-batch tiling, tightened MFMA tolerances), the error
# table on the final kernel, and the config-2 per-GPU point (1 client, bf16) with the auto tiling.
source "$(dirname "$0")/gpu_step.sh"
step gpu_tests 1000 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider
step err_table 300 python scripts/hea_err_table.py
step bench_c1 300 python bench.py --clients 1 --engine mfma_bf16 --steps 100 --warmup 10
step bench_c1_fp16 300 python bench.py --clients 1 --steps 100 --warmup 10
TAILN=1 QFEDX_HEA_TILE=13 step c8_t13 200 python scripts/hea_kbench.py --clients 8 --iters 100
TAILN=1 step c8_t14 200 python scripts/hea_kbench.py --clients 8 --iters 100
step bench 300 python bench.py --steps 20 --warmup 3
