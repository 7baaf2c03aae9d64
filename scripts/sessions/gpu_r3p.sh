#!/bin/bash
# FedAvg weight sum lane-parallel: kernel + trainer GPU tests, headline bench, 64-client round timeline.
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out/prof10
step() {
  local name=$1 secs=$2; shift 2
  timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc"; grep -E '"metric"|passed|failed' "gpurun_out/$name.log" | cut -c1-220
  [ $rc -eq 0 ] || exit $rc
}
step tests 600 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_multirank.py tests/test_gpu_rccl.py tests/test_gpu_cnn.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider
step bench 300 python bench.py --steps 20 --warmup 3
step prof64 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/prof10 -o f64 -- python3 bench.py --steps 10 --warmup 3
python3 scripts/round_timeline.py gpurun_out/prof10/f64_kernel_trace.csv
