#!/bin/bash
# per-pass timings for JIT occupancy targets
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
for w in 0 4; do
  QFEDX_JIT_WAVES_ADJ=$w timeout -k 10 300 python scripts/kbench.py > gpurun_out/kbench_w$w.log 2>&1
  rc=$?; echo "adj waves=$w rc=$rc $(tail -1 gpurun_out/kbench_w$w.log)"
  [ $rc -eq 0 ] || exit $rc
done
