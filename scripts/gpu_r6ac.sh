#!/bin/bash
# Round 6: 8-client share round timeline (rocprofv3 kernel trace of bench.py --clients 8).
source "$(dirname "$0")/gpu_step.sh"
step prof8 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/prof8 -o k -- python3 bench.py --clients 8 --steps 40 --warmup 20
python3 scripts/round_timeline.py --marker qfx_round_prologue_kernel gpurun_out/prof8/k_kernel_trace.csv > gpurun_out/prof8/timeline.txt
python3 scripts/round_periods.py gpurun_out/prof8/k_kernel_trace.csv > gpurun_out/prof8/periods.txt
