#!/bin/bash
# Round 6: kernel traces of the DP (config 3) and MPS 48q suite lines
source "$(dirname "$0")/gpu_step.sh"
for c in vqc20q_dp64_mfma vqc48q_mps64; do
  mkdir -p gpurun_out/kt_$c
  step kt_$c 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/kt_$c -o kt -- python3 bench_suite.py --config $c --steps 10 --warmup 2
done
