#!/bin/bash
# Round 4, call 5: OP_L1PROD without mixed-precision FMAs on the lambda words: determinism at three shapes (three
# identical calls each), then the step / adjoint A/B against the per-group GRAD_L1 ops.
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for shp in "16 3 16 8" "16 3 64 32" "20 3 3 4" "16 3 8 32"; do
  timeout -k 10 300 python -u scripts/l1prod_bisect.py $shp > gpurun_out/r4e_bisect.log 2>&1 || { tail -20 gpurun_out/r4e_bisect.log; exit 1; }
  grep variant gpurun_out/r4e_bisect.log | cut -c1-400
done
timeout -k 10 300 python -u scripts/hea_ab.py --rounds 5 --variants "g1:l1prod=0,lp:l1prod=1" > gpurun_out/r4e_ab.log 2>&1 || { tail -20 gpurun_out/r4e_ab.log; exit 1; }
tail -1 gpurun_out/r4e_ab.log
