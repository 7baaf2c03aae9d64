#!/bin/bash
# Adjoint LDS layout / last-pass recompute A/B (kernel step on one box), GPU suite, headline bench, CFed profile.
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out/profc
step() {  # step <name> <seconds> <cmd...>; pytest rc 1 (failed tests) continues, any other failure ends the run
  local name=$1 secs=$2; shift 2
  timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc"; tail -2 "gpurun_out/$name.log"
  if [ $rc -ne 0 ]; then
    if [ "$name" = gpu_tests ] && [ $rc -eq 1 ]; then return 0; fi
    exit $rc
  fi
}
for v in "0 0" "1 0" "0 1" "1 1" "0 0"; do
  set -- $v
  QFEDX_HEA_PLANES=$1 QFEDX_HEA_RECOMPUTE=$2 step kb_p$1_r$2 300 python scripts/hea_kbench.py --iters 10
done
step gpu_tests 900 python -u -m pytest tests -m gpu -q --maxfail=8 --timeout 120 --timeout-method thread -p no:cacheprovider
grep -E "^(FAILED|ERROR)" gpurun_out/gpu_tests.log | head -20
step bench 300 python bench.py --steps 20 --warmup 5
step prof_cfed 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/profc -o cfed -- python3 bench_suite.py --config cfed128 --steps 10 --warmup 3
python3 scripts/prof_summary.py gpurun_out/profc/cfed_kernel_trace.csv > gpurun_out/profc/summary.txt
python3 scripts/round_timeline.py gpurun_out/profc/cfed_kernel_trace.csv > gpurun_out/profc/timeline.txt
head -14 gpurun_out/profc/summary.txt
