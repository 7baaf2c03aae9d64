#!/bin/bash
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r5f
timeout -k 10 300 python -u scripts/pair_state_diff.py 20 2 > gpurun_out/r5f/d20.log 2>&1; rc=$?; echo "d20 rc=$rc"; grep pass gpurun_out/r5f/d20.log | cut -c1-600; [ $rc -eq 0 ] || { tail -5 gpurun_out/r5f/d20.log; exit $rc; }
timeout -k 10 300 python -u scripts/pair_state_diff.py 16 3 > gpurun_out/r5f/d16.log 2>&1; rc=$?; echo "d16 rc=$rc"; grep pass gpurun_out/r5f/d16.log | cut -c1-600
