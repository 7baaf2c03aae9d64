#!/bin/bash
# CFed TinyCNN x 128 clients: suite entries and kernel-trace round timeline.
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out/profc
STEPS=10 WARMUP=3 bash scripts/gpu_suite.sh cfed128 cfed128_epoch || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/profc -o cfed -- python3 bench_suite.py --config cfed128 --steps 10 --warmup 3 > gpurun_out/profc.log 2>&1 || exit 1
python3 scripts/prof_summary.py gpurun_out/profc/cfed_kernel_trace.csv > gpurun_out/profc/summary.txt
python3 scripts/round_timeline.py gpurun_out/profc/cfed_kernel_trace.csv > gpurun_out/profc/timeline.txt; cat gpurun_out/profc/timeline.txt
