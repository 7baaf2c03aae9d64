#!/bin/bash
# Round 5, call 9: HIP column-contraction MPS kernel (tests vs oracle and vs the torch MPS backend, the 48-qubit suite
# line), then the privacy suite lines (20q DP local / distributed: accuracy, mode, epsilon) and config 5.
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r5i
step() {  # step <name> <seconds> <cmd...>
  local name=$1 secs=$2; shift 2
  timeout -k 10 "$secs" "$@" > "gpurun_out/r5i/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc"; tail -3 "gpurun_out/r5i/$name.log" | cut -c1-700
  [ $rc -eq 0 ] || exit $rc
}
step mps_tests 300 python -u -m pytest tests/test_gpu_mps_chain.py -x -v --timeout 200 --timeout-method thread -p no:cacheprovider
step suite_mps 400 python bench_suite.py --config vqc48q_mps64 --steps 10 --warmup 2
step prof_mps 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r5i/profm -o mps -- python3 bench_suite.py --config vqc48q_mps64 --steps 5 --warmup 1
step suite_dp 400 python bench_suite.py --config vqc20q_dp64_mfma --steps 10 --warmup 2
step suite_ddp 400 python bench_suite.py --config vqc20q_ddp64_mfma --steps 10 --warmup 2
step suite_ps 600 python bench_suite.py --config vqc24q_ps256_mfma --steps 3 --warmup 1
