#!/bin/bash
# Relaxed round-signal store (no L2 writeback at each round's end): benches + share8 timeline under the profiler.
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out/prof8
step() {
  local name=$1 secs=$2; shift 2
  timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc"; tail -1 "gpurun_out/$name.log" | cut -c1-250
  [ $rc -eq 0 ] || exit $rc
}
step bench 300 python bench.py --steps 30 --warmup 5
step share8 300 python bench.py --steps 60 --warmup 5 --clients 8
step prof_share8 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/prof8 -o share8 -- python3 bench.py --steps 20 --warmup 3 --clients 8 --precision-check 0
python3 scripts/round_timeline.py gpurun_out/prof8/share8_kernel_trace.csv > gpurun_out/prof8/share8_timeline.txt
head -2 gpurun_out/prof8/share8_timeline.txt
grep -o '"host_ms_per_round": [0-9.]*\|"ms_per_step": [0-9.]*' gpurun_out/bench.log gpurun_out/share8.log
