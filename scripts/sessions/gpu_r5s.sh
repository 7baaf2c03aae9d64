#!/bin/bash
# Round 5, call 19: the plain FedAvg reduce (no DP / SecAgg) as its own 40-VGPR instantiation (the general one holds
# 123 VGPRs: one 1024-thread block per CU): kernel + CNN tests, CFed 50-round line and round timeline, headline bench.
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r5s
step() {  # step <name> <seconds> <cmd...>
  local name=$1 secs=$2; shift 2
  timeout -k 10 "$secs" "$@" > "gpurun_out/r5s/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc"; tail -2 "gpurun_out/r5s/$name.log" | cut -c1-400
  [ $rc -eq 0 ] || exit $rc
}
step tests 600 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_cnn.py -x -q --timeout 200 --timeout-method thread -p no:cacheprovider
step cfed 300 python bench_suite.py --config cfed128 --steps 50 --warmup 5
step profcfed 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r5s/profcfed -o bench -- python3 bench_suite.py --config cfed128 --steps 20 --warmup 3
python3 scripts/round_timeline.py gpurun_out/r5s/profcfed/bench_kernel_trace.csv --marker qfx_host_upload_kernel > gpurun_out/r5s/timelinecfed.txt 2>&1
cat gpurun_out/r5s/timelinecfed.txt
step bench64 300 python bench.py --steps 20 --warmup 3
step prof64 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r5s/prof64 -o bench -- python3 bench.py --steps 10 --warmup 3
python3 scripts/round_timeline.py gpurun_out/r5s/prof64/bench_kernel_trace.csv --marker qfx_round_prologue_kernel > gpurun_out/r5s/timeline64.txt 2>&1
cat gpurun_out/r5s/timeline64.txt
