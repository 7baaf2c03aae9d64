#!/bin/bash
# Round 4, call 21: OP_L1PROD repeatability re-checked after the fragment-DMA M0 wait-state fix (the earlier bisection
# runs predate it): three identical vjp calls per program at 8 x 32 and at the headline 64 x 32.
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
timeout -k 10 300 python -u scripts/l1prod_bisect.py 16 3 8 32 > gpurun_out/r4t_bisect_8x32.log 2>&1 || { tail -20 gpurun_out/r4t_bisect_8x32.log; exit 1; }
grep variant gpurun_out/r4t_bisect_8x32.log | cut -c1-330
timeout -k 10 300 python -u scripts/l1prod_bisect.py 16 3 64 32 > gpurun_out/r4t_bisect_64x32.log 2>&1 || { tail -20 gpurun_out/r4t_bisect_64x32.log; exit 1; }
grep variant gpurun_out/r4t_bisect_64x32.log | cut -c1-330
