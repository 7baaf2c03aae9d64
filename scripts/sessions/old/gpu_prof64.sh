#!/bin/bash
# Headline bench + kernel-trace round timeline (64 clients) and the host/device round timing.
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out/prof64
timeout -k 10 300 python bench.py --steps 20 --warmup 3 > gpurun_out/bench.log 2>&1 || exit 1
grep metric gpurun_out/bench.log | cut -c1-200
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/prof64 -o full64 -- python3 bench.py --steps 10 --warmup 3 > gpurun_out/prof64.log 2>&1 || exit 1
python3 scripts/round_timeline.py gpurun_out/prof64/full64_kernel_trace.csv
timeout -k 10 300 python scripts/host_round_time.py --clients 64 > gpurun_out/host64.log 2>&1 || exit 1
tail -1 gpurun_out/host64.log
