#!/bin/bash
# CC4 cost/benefit at one rank with an RCCL group (the driver's N > 1 runs have CC4 on): bench.py --dist-backend nccl,
# QFEDX_CC4=0 vs 1 interleaved, at the 8-client share and the 64-client headline; then the NT-store build's headline
# bench and the 1-client bf16 round timeline (rocprofv3) for profiles/.
source "$(dirname "$0")/gpu_step.sh"
for r in 1 2 3; do for c in 0 1; do
  TAILN=1 QFEDX_CC4=$c step cc4_c8_${c}_$r 200 python bench.py --dist-backend nccl --clients 8 --steps 200 --warmup 10 --precision-check 0
done; done
for r in 1 2; do for c in 0 1; do
  TAILN=1 QFEDX_CC4=$c step cc4_c64_${c}_$r 200 python bench.py --dist-backend nccl --steps 30 --warmup 3 --precision-check 0
done; done
step bench 300 python bench.py --steps 20 --warmup 3
step bench_c8 300 python bench.py --clients 8 --steps 100 --warmup 5
step prof_c1 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/prof_c1 -o c1 -- \
  python3 bench.py --clients 1 --engine mfma_bf16 --steps 50 --warmup 5 --precision-check 0
