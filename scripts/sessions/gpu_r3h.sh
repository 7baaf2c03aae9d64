#!/bin/bash
# Paired two-sample forward A/B (kernel step), GPU suite, headline bench + 8-client share (+ host enqueue time).
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
step() {  # step <name> <seconds> <cmd...>; pytest rc 1 (failed tests) continues, any other failure ends the run
  local name=$1 secs=$2; shift 2
  timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc"; tail -2 "gpurun_out/$name.log"
  if [ $rc -ne 0 ]; then
    if { [ "$name" = gpu_tests ] || [ "${name#t_}" != "$name" ]; } && [ $rc -eq 1 ]; then return 0; fi
    exit $rc
  fi
}
step t_pair 400 python -u -m pytest tests/test_gpu_hea.py tests/test_gpu_paramshift.py -q -k "paired or train_step or vjp_matches or shift" --timeout 120 --timeout-method thread -p no:cacheprovider
for v in 1 0 1 0; do
  QFEDX_HEA_FWD_PAIR=$v step kb_pair$v 300 python scripts/hea_kbench.py --iters 10
done
step gpu_tests 900 python -u -m pytest tests -m gpu -q --maxfail=8 --timeout 120 --timeout-method thread -p no:cacheprovider
grep -E "^(FAILED|ERROR)" gpurun_out/gpu_tests.log | head -20
step bench 300 python bench.py --steps 20 --warmup 5
step share8 300 python bench.py --steps 30 --warmup 5 --clients 8
QFEDX_HEA_FWD_PAIR=0 step bench_nopair 300 python bench.py --steps 20 --warmup 5
