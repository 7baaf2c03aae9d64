#!/bin/bash
# Kernel-trace timeline of the per-rank share at 8 GPUs (8 of the 64 headline clients on one GPU) and of the
# full 64-client headline round.
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out/prof8
step() {
  local name=$1 secs=$2; shift 2
  timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc"; grep '"metric"' "gpurun_out/$name.log" | cut -c1-220
  [ $rc -eq 0 ] || exit $rc
}
step share8 300 python bench.py --steps 30 --warmup 5 --clients 8
step bench64 300 python bench.py --steps 20 --warmup 3
step prof8 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/prof8 -o share8 -- python3 bench.py --steps 20 --warmup 3 --clients 8
step prof64 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/prof8 -o full64 -- python3 bench.py --steps 10 --warmup 3
python3 scripts/round_timeline.py gpurun_out/prof8/share8_kernel_trace.csv
python3 scripts/round_timeline.py gpurun_out/prof8/full64_kernel_trace.csv
