#!/bin/bash
# Round 5, call 4: which pair kind breaks 20q x 2L gradients (release + device-check build), 16q for comparison.
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r5d
timeout -k 10 200 python -u scripts/pair_bisect.py 20 2 > gpurun_out/r5d/b20.log 2>&1; rc=$?; echo "b20 rc=$rc"; grep mask gpurun_out/r5d/b20.log; [ $rc -eq 0 ] || { tail -5 gpurun_out/r5d/b20.log; exit $rc; }
timeout -k 10 200 python -u scripts/pair_bisect.py 16 3 > gpurun_out/r5d/b16.log 2>&1; rc=$?; echo "b16 rc=$rc"; grep mask gpurun_out/r5d/b16.log; [ $rc -eq 0 ] || exit $rc
QFEDX_DEBUG=1 timeout -k 10 300 python -u scripts/pair_bisect.py 20 2 > gpurun_out/r5d/b20d.log 2>&1; rc=$?; echo "b20 debug rc=$rc"; grep -E "mask|check" gpurun_out/r5d/b20d.log | head; tail -3 gpurun_out/r5d/b20d.log
