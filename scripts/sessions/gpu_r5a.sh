#!/bin/bash
# Round 5, call 1: baseline on a fresh box -- headline bench, 8-client share, kernel stats.
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r5a
timeout -k 10 300 python bench.py --steps 20 --warmup 3 > gpurun_out/r5a/bench.log 2>&1; rc=$?
echo "bench rc=$rc"; grep '"metric"' gpurun_out/r5a/bench.log | cut -c1-400; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --steps 30 --warmup 5 --clients 8 > gpurun_out/r5a/share8.log 2>&1; rc=$?
echo "share8 rc=$rc"; grep '"metric"' gpurun_out/r5a/share8.log | cut -c1-400; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r5a/prof -o bench -- python3 bench.py --steps 10 --warmup 2 > gpurun_out/r5a/prof.log 2>&1; rc=$?
echo "prof rc=$rc"; exit $rc
