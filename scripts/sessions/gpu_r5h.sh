#!/bin/bash
# Round 5, call 8: prologue off wave 0's critical path (host fo table), first barrier without the readout wave's store
# drain, direct gradient regions (no ring flush) - MFMA tests, full GPU suite, benches, per-wave stall table, timelines.
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r5h
step() {  # step <name> <seconds> <cmd...>
  local name=$1 secs=$2; shift 2
  timeout -k 10 "$secs" "$@" > "gpurun_out/r5h/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc"; tail -3 "gpurun_out/r5h/$name.log" | cut -c1-600
  [ $rc -eq 0 ] || exit $rc
}
step hea_tests 400 python -u -m pytest tests/test_gpu_hea.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider
step gpu_tests 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider
step bench64 300 python bench.py --steps 20 --warmup 3
step share8 300 python bench.py --steps 30 --warmup 5 --clients 8
step stamps64 300 python -u scripts/hea_stamps.py --clients 64 --out gpurun_out/r5h/stamps64.jsonl
step prof64 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r5h/prof64 -o bench -- python3 bench.py --steps 10 --warmup 3
step prof8 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r5h/prof8 -o bench -- python3 bench.py --steps 20 --warmup 3 --clients 8
python3 scripts/round_timeline.py gpurun_out/r5h/prof64/bench_kernel_trace.csv --marker qfx_host_upload_kernel > gpurun_out/r5h/timeline64.txt 2>&1
python3 scripts/round_timeline.py gpurun_out/r5h/prof8/bench_kernel_trace.csv --marker qfx_host_upload_kernel > gpurun_out/r5h/timeline8.txt 2>&1
cat gpurun_out/r5h/timeline64.txt gpurun_out/r5h/timeline8.txt
