#!/bin/bash
# Round 5, call 23: cnn_head loads the fc1 partials of four elements per thread before summing (one round trip per
# element before): CNN GPU tests, the cfed128 50-round line and its round timeline.
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r5w
step() {  # step <name> <seconds> <cmd...>
  local name=$1 secs=$2; shift 2
  timeout -k 10 "$secs" "$@" > "gpurun_out/r5w/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc"; tail -2 "gpurun_out/r5w/$name.log" | cut -c1-300
  [ $rc -eq 0 ] || exit $rc
}
step tests 400 python -u -m pytest tests/test_gpu_cnn.py tests/test_gpu_multirank.py -x -q --timeout 200 --timeout-method thread -p no:cacheprovider
step cfed 300 python bench_suite.py --config cfed128 --steps 50 --warmup 5
step profcfed 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r5w/profcfed -o bench -- python3 bench_suite.py --config cfed128 --steps 20 --warmup 3
python3 scripts/round_timeline.py gpurun_out/r5w/profcfed/bench_kernel_trace.csv --marker qfx_host_upload_kernel > gpurun_out/r5w/timelinecfed.txt 2>&1
cat gpurun_out/r5w/timelinecfed.txt
