#!/bin/bash
# Round 6: where config 5's parameter-shift time goes (kernel stats of scripts/ps_kbench.py, 16 clients x 8 samples).
source "$(dirname "$0")/gpu_step.sh"
step ps_prof 400 rocprofv3 --kernel-trace --stats -d gpurun_out/ps_prof -o ps -- python3 scripts/ps_kbench.py --clients 16 --batch 8 --iters 1
find gpurun_out/ps_prof -name "*kernel_stats.csv" | head -3
