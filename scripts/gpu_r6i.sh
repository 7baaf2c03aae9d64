#!/bin/bash
# Round 6: adjoint tile size at the 8-client share (2^13: two 8-wave workgroups per CU; 2^14: one 16-wave workgroup),
# interleaved bench.py runs, plus the 64-client step for reference.
source "$(dirname "$0")/gpu_step.sh"
for r in 1 2 3; do
  for t in 13 14; do
    TAILN=1 QFEDX_HEA_ADJ_TILE=$t step adjt${t}_c8_$r 200 python bench.py --clients 8 --steps 50 --warmup 5
  done
done
for r in 1 2; do
  for t in 13 14; do
    TAILN=1 QFEDX_HEA_ADJ_TILE=$t step adjt${t}_c64_$r 200 python bench.py --steps 20 --warmup 3
  done
done
