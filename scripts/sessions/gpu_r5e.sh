#!/bin/bash
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r5e
timeout -k 10 300 python -u scripts/pair_bisect.py 20 2 1,3,5,6,7 > gpurun_out/r5e/b20.log 2>&1; rc=$?; echo "b20 rc=$rc"; grep mask gpurun_out/r5e/b20.log | cut -c1-300; [ $rc -eq 0 ] || { tail -5 gpurun_out/r5e/b20.log; exit $rc; }
timeout -k 10 300 python -u scripts/pair_bisect.py 16 2 1,7 > gpurun_out/r5e/b162.log 2>&1; rc=$?; echo "b16x2 rc=$rc"; grep mask gpurun_out/r5e/b162.log | cut -c1-300
timeout -k 10 300 python -u scripts/pair_bisect.py 18 2 1,7 > gpurun_out/r5e/b182.log 2>&1; rc=$?; echo "b18x2 rc=$rc"; grep mask gpurun_out/r5e/b182.log | cut -c1-300
