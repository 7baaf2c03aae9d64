#!/bin/bash
# Round 5, call 12: host upload folded into the round prologue only while its gather is small (<= 512 rows), and the
# owned fused-Adam mode of hea_grad_reduce past one block per CU (64 clients: Adam + FedAvg tail without the separate
# Adam and FedAvg launches): the GPU suite, the 8- and 64-client benches (owned on / off interleaved) and both round
# timelines.
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r5l
step() {  # step <name> <seconds> <cmd...>
  local name=$1 secs=$2; shift 2
  timeout -k 10 "$secs" "$@" > "gpurun_out/r5l/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc"; tail -3 "gpurun_out/r5l/$name.log" | cut -c1-600
  [ $rc -eq 0 ] || exit $rc
}
step gpu_tests 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider
step share8a 300 python bench.py --steps 40 --warmup 5 --clients 8
step bench64a 300 python bench.py --steps 20 --warmup 3
step bench64_off_a 300 env QFEDX_OWNED_ADAM=0 python bench.py --steps 20 --warmup 3
step share8b 300 python bench.py --steps 40 --warmup 5 --clients 8
step bench64b 300 python bench.py --steps 20 --warmup 3
step bench64_off_b 300 env QFEDX_OWNED_ADAM=0 python bench.py --steps 20 --warmup 3
step prof8 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r5l/prof8 -o bench -- python3 bench.py --steps 20 --warmup 3 --clients 8
python3 scripts/round_timeline.py gpurun_out/r5l/prof8/bench_kernel_trace.csv --marker qfx_round_prologue_kernel > gpurun_out/r5l/timeline8.txt 2>&1
step prof64 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r5l/prof64 -o bench -- python3 bench.py --steps 10 --warmup 3
python3 scripts/round_timeline.py gpurun_out/r5l/prof64/bench_kernel_trace.csv --marker qfx_round_prologue_kernel > gpurun_out/r5l/timeline64.txt 2>&1
cat gpurun_out/r5l/timeline64.txt gpurun_out/r5l/timeline8.txt
