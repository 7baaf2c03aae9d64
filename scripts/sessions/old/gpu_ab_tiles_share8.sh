#!/bin/bash
# Tile-size A/B at the 8-client per-rank share (strong-scaling floor at 8 GPUs) and at 64 clients:
# forward tile 2^14 (default) vs 2^13, adjoint tile 2^13 (default) vs 2^12; interleaved bench.py runs.
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for r in 1 2; do
  for v in "14 13" "13 13" "14 12" "13 12"; do
    set -- $v
    for cl in 8 64; do
      QFEDX_HEA_TILE=$1 QFEDX_HEA_ADJ_TILE=$2 timeout -k 10 300 python bench.py --steps 40 --warmup 5 --clients $cl \
        > gpurun_out/abt_$1_$2_${cl}_$r.log 2>&1 || exit 1
      echo "fwd=$1 adj=$2 clients=$cl r=$r $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/abt_$1_$2_${cl}_$r.log)"
    done
  done
done
