#!/bin/bash
# Round 5, call 22: short rows gathered 256 / tps to a prologue block (64 clients: 128 gather blocks instead of 2,048),
# which lets the host upload fold into the prologue at 64 clients too: the GPU suite, then fold on / off interleaved
# at 64 and 8 clients, both round timelines.
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r5v
step() {  # step <name> <seconds> <cmd...>
  local name=$1 secs=$2; shift 2
  timeout -k 10 "$secs" "$@" > "gpurun_out/r5v/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc"; tail -2 "gpurun_out/r5v/$name.log" | cut -c1-300
  [ $rc -eq 0 ] || exit $rc
}
step gpu_tests 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider
for i in a b; do
  step bench64_on_$i 300 python bench.py --steps 20 --warmup 3
  step bench64_off_$i 300 env QFEDX_FOLD_UPLOAD=0 python bench.py --steps 20 --warmup 3
  step share8_on_$i 300 python bench.py --steps 40 --warmup 5 --clients 8
  step share8_off_$i 300 env QFEDX_FOLD_UPLOAD=0 python bench.py --steps 40 --warmup 5 --clients 8
done
step prof64 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r5v/prof64 -o bench -- python3 bench.py --steps 10 --warmup 3
python3 scripts/round_timeline.py gpurun_out/r5v/prof64/bench_kernel_trace.csv --marker qfx_round_prologue_kernel > gpurun_out/r5v/timeline64.txt 2>&1
step prof8 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r5v/prof8 -o bench -- python3 bench.py --steps 20 --warmup 3 --clients 8
python3 scripts/round_timeline.py gpurun_out/r5v/prof8/bench_kernel_trace.csv --marker qfx_round_prologue_kernel > gpurun_out/r5v/timeline8.txt 2>&1
cat gpurun_out/r5v/timeline64.txt gpurun_out/r5v/timeline8.txt
