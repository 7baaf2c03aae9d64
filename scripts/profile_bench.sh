#!/bin/bash
# rocprofv3 kernel-trace + stats of the headline bench (no PMC counters in this run).
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out/prof
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o bench -- python3 bench.py --steps 3 --warmup 1 "$@" > gpurun_out/prof_bench.log 2>&1
rc=$?; echo "rc=$rc"; tail -3 gpurun_out/prof_bench.log
find gpurun_out/prof -name "*stats*" | head
exit $rc
