#!/bin/bash
# Round 5, call 13: CFed fc1 kernels (forward loads 5 steps ahead, input gradient 2 steps ahead, weight gradient as the
# transposed product with 16-byte sink accesses; 16-byte image gather in the prologue): the CNN GPU tests, the cfed128 suite line and its round timeline.
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r5m
step() {  # step <name> <seconds> <cmd...>
  local name=$1 secs=$2; shift 2
  timeout -k 10 "$secs" "$@" > "gpurun_out/r5m/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc"; tail -3 "gpurun_out/r5m/$name.log" | cut -c1-600
  [ $rc -eq 0 ] || exit $rc
}
step cnn_tests 400 python -u -m pytest tests/test_gpu_cnn.py -x -q --timeout 200 --timeout-method thread -p no:cacheprovider
step cfed 300 python bench_suite.py --config cfed128 --steps 50 --warmup 5
step profcfed 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r5m/profcfed -o bench -- python3 bench_suite.py --config cfed128 --steps 20 --warmup 3
python3 scripts/round_timeline.py gpurun_out/r5m/profcfed/bench_kernel_trace.csv --marker qfx_host_upload_kernel > gpurun_out/r5m/timelinecfed.txt 2>&1
cat gpurun_out/r5m/timelinecfed.txt
