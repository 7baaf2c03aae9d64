#!/bin/bash
# Round 6: where the CFed SecAgg rounds' time goes - kernel traces of the full-graph and sparse-graph suite lines.
source "$(dirname "$0")/gpu_step.sh"
for c in cfed128_secagg cfed128_secagg_sparse; do
  mkdir -p gpurun_out/sa_$c
  step sa_$c 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/sa_$c -o sa -- python3 bench_suite.py --config $c --steps 10 --warmup 2
done
