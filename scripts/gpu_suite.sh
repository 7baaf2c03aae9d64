#!/bin/bash
# BASELINE-config benchmark suite on one GPU (each step with its own time limit, stop on failure)
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
for c in "$@"; do
  timeout -k 10 600 python bench_suite.py --config $c --steps ${STEPS:-5} --warmup ${WARMUP:-2} > gpurun_out/suite_$c.log 2>&1
  rc=$?; echo "$c rc=$rc"; grep '"metric"' gpurun_out/suite_$c.log || tail -5 gpurun_out/suite_$c.log
  [ $rc -eq 0 ] || exit $rc
done
