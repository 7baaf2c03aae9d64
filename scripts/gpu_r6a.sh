#!/bin/bash
# Round 6, first measurement: HEA numerics of the new pair-back kernel, error table, interleaved A/B (ab/base vs ab/new),
# headline bench.
source "$(dirname "$0")/gpu_step.sh"
step hea_tests 400 python -u -m pytest tests/test_gpu_hea.py tests/test_gpu_paramshift.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider
step err_table 300 python scripts/hea_err_table.py
for r in 1 2; do for v in base new; do
  QFX_PKG_ROOT=$PWD/ab/$v step ab_${v}$r 200 python scripts/hea_kbench.py --iters 30
done; done
step bench 300 python bench.py --steps 20 --warmup 3
step bench_c8 300 python bench.py --clients 8 --steps 50 --warmup 5
step bench_c1 300 python bench.py --clients 1 --engine mfma_bf16 --steps 50 --warmup 5
