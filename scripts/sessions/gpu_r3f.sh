#!/bin/bash
# Fused BACK cross-matrix A/B (kernel step on one box), GPU suite, headline bench + 8-client share, CFed suite with
# the 16-byte-load fc1 kernels, inter-graph launch gap microbenchmark.
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out/profc gpurun_out/profg
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
for v in "1 0" "0 0" "0 1" "1 0" "0 0"; do
  set -- $v
  QFEDX_HEA_FUSE=$1 QFEDX_HEA_PLANES=$2 step kb_f$1_p$2 300 python scripts/hea_kbench.py --iters 10
done
step gpu_tests 900 python -u -m pytest tests -m gpu -q --maxfail=8 --timeout 120 --timeout-method thread -p no:cacheprovider
grep -E "^(FAILED|ERROR)" gpurun_out/gpu_tests.log | head -20
step bench 300 python bench.py --steps 20 --warmup 5
step share8 300 python bench.py --steps 30 --warmup 5 --clients 8
STEPS=10 WARMUP=8 bash scripts/gpu_suite.sh cfed128 || exit 1
step prof_cfed 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/profc -o cfed -- python3 bench_suite.py --config cfed128 --steps 10 --warmup 3
python3 scripts/round_timeline.py gpurun_out/profc/cfed_kernel_trace.csv > gpurun_out/profc/timeline.txt
head -8 gpurun_out/profc/timeline.txt
for g in 1 2; do for e in 0 2; do step gap_g${g}_e$e 120 python scripts/graph_gap.py --graphs $g --events $e; done; done
step prof_gap 120 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/profg -o gap -- python3 scripts/graph_gap.py --graphs 2 --reps 50
