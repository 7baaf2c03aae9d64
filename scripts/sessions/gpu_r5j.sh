#!/bin/bash
# Round 5, call 10: host fo table + first-barrier + direct regions + short layer-1 gradient pairs + prologue-built
# fragments + the MPS column kernel: MFMA tests, the full GPU suite, benches, timelines, stall table, suite lines.
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r5j
step() {  # step <name> <seconds> <cmd...>
  local name=$1 secs=$2; shift 2
  timeout -k 10 "$secs" "$@" > "gpurun_out/r5j/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc"; tail -3 "gpurun_out/r5j/$name.log" | cut -c1-600
  [ $rc -eq 0 ] || exit $rc
}
#step hea_tests 400 python -u -m pytest tests/test_gpu_hea.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider
step gpu_tests 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider
step bench64 300 python bench.py --steps 20 --warmup 3
step share8 300 python bench.py --steps 30 --warmup 5 --clients 8
step prof8 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r5j/prof8 -o bench -- python3 bench.py --steps 20 --warmup 3 --clients 8
python3 scripts/round_timeline.py gpurun_out/r5j/prof8/bench_kernel_trace.csv --marker qfx_host_upload_kernel > gpurun_out/r5j/timeline8.txt 2>&1
step stamps64 300 python -u scripts/hea_stamps.py --clients 64 --out gpurun_out/r5j/stamps64.jsonl
step suite_mps 400 python bench_suite.py --config vqc48q_mps64 --steps 10 --warmup 2
step prof64 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r5j/prof64 -o bench -- python3 bench.py --steps 10 --warmup 3
python3 scripts/round_timeline.py gpurun_out/r5j/prof64/bench_kernel_trace.csv --marker qfx_host_upload_kernel > gpurun_out/r5j/timeline64.txt 2>&1
cat gpurun_out/r5j/timeline64.txt gpurun_out/r5j/timeline8.txt
step suite_dp 300 python bench_suite.py --config vqc20q_dp64_mfma --steps 10 --warmup 2
step suite_ddp 300 python bench_suite.py --config vqc20q_ddp64_mfma --steps 10 --warmup 2
