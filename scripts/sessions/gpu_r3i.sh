#!/bin/bash
# Host enqueue cost per round (bench host_ms_per_round excludes waits for the GPU) and the paired-forward tests.
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
step() {
  local name=$1 secs=$2; shift 2
  timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc"; tail -2 "gpurun_out/$name.log"
  if [ $rc -ne 0 ]; then
    if { [ "$name" = gpu_tests ] || [ "${name#t_}" != "$name" ]; } && [ $rc -eq 1 ]; then return 0; fi
    exit $rc
  fi
}
step t_pair 400 python -u -m pytest tests/test_gpu_hea.py tests/test_gpu_paramshift.py -q -k "paired or shift" --timeout 120 --timeout-method thread -p no:cacheprovider
step bench 300 python bench.py --steps 30 --warmup 5
step share8 300 python bench.py --steps 60 --warmup 5 --clients 8
grep -o '"host_ms_per_round": [0-9.]*\|"ms_per_step": [0-9.]*' gpurun_out/bench.log gpurun_out/share8.log
