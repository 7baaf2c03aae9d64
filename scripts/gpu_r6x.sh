#!/bin/bash
# Round 6: kernel stats of the config-3 DP suite lines (20q x 64 clients, local and distributed DP).
source "$(dirname "$0")/gpu_step.sh"
step prof_dp 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_dp -o dp -- python3 bench_suite.py --config vqc20q_dp64_mfma --steps 5 --warmup 2
step prof_ddp 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_ddp -o ddp -- python3 bench_suite.py --config vqc20q_ddp64_mfma --steps 5 --warmup 2
