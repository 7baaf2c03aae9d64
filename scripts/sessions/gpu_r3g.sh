#!/bin/bash
# Event-free round graphs (device round counter instead of HIP events; phases timed after the timed rounds):
# GPU suite, headline / RCCL / 8-client share benches, kernel-trace timelines of the headline and the share.
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out/prof gpurun_out/prof8
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
step gpu_tests 900 python -u -m pytest tests -m gpu -q --maxfail=8 --timeout 120 --timeout-method thread -p no:cacheprovider
grep -E "^(FAILED|ERROR)" gpurun_out/gpu_tests.log | head -20
step bench 300 python bench.py --steps 20 --warmup 5
step bench_rccl 300 python bench.py --steps 20 --warmup 5 --dist-backend nccl
step share8 300 python bench.py --steps 30 --warmup 5 --clients 8
step prof_bench 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/prof -o bench -- python3 bench.py --steps 10 --warmup 3 --precision-check 0
python3 scripts/round_timeline.py gpurun_out/prof/bench_kernel_trace.csv > gpurun_out/prof/bench_timeline.txt
step prof_share8 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/prof8 -o share8 -- python3 bench.py --steps 20 --warmup 3 --clients 8 --precision-check 0
python3 scripts/round_timeline.py gpurun_out/prof8/share8_kernel_trace.csv > gpurun_out/prof8/share8_timeline.txt
head -3 gpurun_out/prof/bench_timeline.txt gpurun_out/prof8/share8_timeline.txt
STEPS=10 WARMUP=8 bash scripts/gpu_suite.sh vqc16q_64_mfma_secagg vqc16q_bf16_8_mfma || exit 1
