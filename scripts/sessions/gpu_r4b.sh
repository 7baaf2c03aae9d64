#!/bin/bash
# Round 4, call 2: OP_L1PROD bisection (which gradient records differ between identical calls; last group op in
# the transposed form vs the fused-output form), at two shapes.
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u scripts/l1prod_bisect.py 16 3 16 8 > gpurun_out/r4b_bisect_16x8.log 2>&1 || { tail -20 gpurun_out/r4b_bisect_16x8.log; exit 1; }
cat gpurun_out/r4b_bisect_16x8.log | grep variant
timeout -k 10 300 python -u scripts/l1prod_bisect.py 16 3 64 32 > gpurun_out/r4b_bisect_64x32.log 2>&1 || { tail -20 gpurun_out/r4b_bisect_64x32.log; exit 1; }
cat gpurun_out/r4b_bisect_64x32.log | grep variant
