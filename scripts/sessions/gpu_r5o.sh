#!/bin/bash
# Round 5, call 15: owned fused Adam with its operands prefetched before the reduction and a 1024-thread pack sum:
# kernel tests, owned on / off interleaved three times at 64 clients, the 64-client timeline.
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r5o
step() {  # step <name> <seconds> <cmd...>
  local name=$1 secs=$2; shift 2
  timeout -k 10 "$secs" "$@" > "gpurun_out/r5o/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc"; tail -3 "gpurun_out/r5o/$name.log" | cut -c1-400
  [ $rc -eq 0 ] || exit $rc
}
step tests 600 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 200 --timeout-method thread -p no:cacheprovider
for i in a b c; do
  step bench64_on_$i 300 python bench.py --steps 20 --warmup 3
  step bench64_off_$i 300 env QFEDX_OWNED_ADAM=0 python bench.py --steps 20 --warmup 3
done
step prof64 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r5o/prof64 -o bench -- python3 bench.py --steps 10 --warmup 3
python3 scripts/round_timeline.py gpurun_out/r5o/prof64/bench_kernel_trace.csv --marker qfx_round_prologue_kernel > gpurun_out/r5o/timeline64.txt 2>&1
cat gpurun_out/r5o/timeline64.txt
