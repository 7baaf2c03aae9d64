#!/bin/bash
# Round 6: vectorised SecAgg host tables (sparse neighbour circle, live counts, cached seed rows) - interleaved
# CFed SecAgg suite lines of the old and new trees.
source "$(dirname "$0")/gpu_step.sh"
for r in 1 2; do for v in base new; do for c in cfed128_secagg_sparse cfed128_secagg; do
  (cd ab/$v && timeout -k 10 300 python bench_suite.py --config $c --steps 30 --warmup 3 > ../../gpurun_out/sa_${c}_${v}$r.log 2>&1) || { echo "sa_${c}_${v}$r failed"; exit 1; }
  echo "$c $v $r $(grep '"metric"' gpurun_out/sa_${c}_${v}$r.log | python -c "import json,sys; print(json.loads(sys.stdin.read())['ms_per_step'])")"
done; done; done
