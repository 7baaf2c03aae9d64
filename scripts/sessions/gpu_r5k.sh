#!/bin/bash
# Round 5, call 11: host upload folded into the round prologue + 4-wide FedAvg reduce (CNN rows) + FedAvg folded into the MFMA engine's Adam epilogue (QfxFedTail): the bitwise tail tests first,
# then the full GPU suite, benches, the 8- and 64-client timelines and the config-5 suite line.
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r5k
step() {  # step <name> <seconds> <cmd...>
  local name=$1 secs=$2; shift 2
  timeout -k 10 "$secs" "$@" > "gpurun_out/r5k/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc"; tail -3 "gpurun_out/r5k/$name.log" | cut -c1-600
  [ $rc -eq 0 ] || exit $rc
}
step tail_tests 300 python -u -m pytest tests/test_gpu_kernels.py -x -v -k "fedavg_tail or prologue_fragments" --timeout 120 --timeout-method thread -p no:cacheprovider
step gpu_tests 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider
step share8 300 python bench.py --steps 30 --warmup 5 --clients 8
step bench64 300 python bench.py --steps 20 --warmup 3
step prof8 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r5k/prof8 -o bench -- python3 bench.py --steps 20 --warmup 3 --clients 8
python3 scripts/round_timeline.py gpurun_out/r5k/prof8/bench_kernel_trace.csv --marker qfx_round_prologue_kernel > gpurun_out/r5k/timeline8.txt 2>&1
step prof64 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r5k/prof64 -o bench -- python3 bench.py --steps 10 --warmup 3
python3 scripts/round_timeline.py gpurun_out/r5k/prof64/bench_kernel_trace.csv --marker qfx_round_prologue_kernel > gpurun_out/r5k/timeline64.txt 2>&1
cat gpurun_out/r5k/timeline64.txt gpurun_out/r5k/timeline8.txt
step cfed 300 python bench_suite.py --config cfed128 --steps 50 --warmup 5
step profcfed 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r5k/profcfed -o bench -- python3 bench_suite.py --config cfed128 --steps 20 --warmup 3
python3 scripts/round_timeline.py gpurun_out/r5k/profcfed/bench_kernel_trace.csv --marker qfx_host_upload_kernel > gpurun_out/r5k/timelinecfed.txt 2>&1
cat gpurun_out/r5k/timelinecfed.txt
step suite_c5 400 python bench_suite.py --config vqc24q_ps256_mfma --steps 5 --warmup 1
