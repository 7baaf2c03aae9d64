#!/bin/bash
# Full GPU test suite, then the headline / per-rank-share benches and the share's kernel timeline.
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out/prof8
step() {
  local name=$1 secs=$2; shift 2
  timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc"; tail -${TAILN:-3} "gpurun_out/$name.log" | cut -c1-250
  [ $rc -eq 0 ] || exit $rc
}
step gpu_tests 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider
TAILN=1 step bench64 300 python bench.py --steps 20 --warmup 3
TAILN=1 step share8 300 python bench.py --steps 30 --warmup 5 --clients 8
TAILN=1 step prof8 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/prof8 -o share8 -- python3 bench.py --steps 20 --warmup 3 --clients 8
python3 scripts/round_timeline.py gpurun_out/prof8/share8_kernel_trace.csv
