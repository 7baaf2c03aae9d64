#!/bin/bash
# Round 5, call 14: owned fused Adam with per-client FedAvg term rows (summed by the pack launch) instead of atomics;
# fc1 forward / input-gradient changes reverted.  Kernel tests, then owned on / off interleaved three times at 64
# clients, the 8-client share, the 64-client timeline and the CFed line.
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r5n
step() {  # step <name> <seconds> <cmd...>
  local name=$1 secs=$2; shift 2
  timeout -k 10 "$secs" "$@" > "gpurun_out/r5n/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc"; tail -3 "gpurun_out/r5n/$name.log" | cut -c1-400
  [ $rc -eq 0 ] || exit $rc
}
step tests 600 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_cnn.py tests/test_gpu_hea.py -x -q --timeout 200 --timeout-method thread -p no:cacheprovider
for i in a b c; do
  step bench64_on_$i 300 python bench.py --steps 20 --warmup 3
  step bench64_off_$i 300 env QFEDX_OWNED_ADAM=0 python bench.py --steps 20 --warmup 3
done
step share8 300 python bench.py --steps 40 --warmup 5 --clients 8
step prof64 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r5n/prof64 -o bench -- python3 bench.py --steps 10 --warmup 3
python3 scripts/round_timeline.py gpurun_out/r5n/prof64/bench_kernel_trace.csv --marker qfx_round_prologue_kernel > gpurun_out/r5n/timeline64.txt 2>&1
cat gpurun_out/r5n/timeline64.txt
step cfed 300 python bench_suite.py --config cfed128 --steps 50 --warmup 5
