#!/bin/bash
# Round 4, call 10: per-client int64 gradient accumulators (adjoint atomics, one-block-per-client reduction with the
# Adam step always fused): full GPU suite, headline + share-8 benches, timelines, chunked share-8 A/B.
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out/prof7
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider -m gpu tests/ > gpurun_out/r4j_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r4j_tests.log; [ $rc -eq 0 ] || exit $rc
step() {
  local name=$1 secs=$2; shift 2
  timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc"; grep '"metric"' "gpurun_out/$name.log" | cut -c1-260
  [ $rc -eq 0 ] || exit $rc
}
step r4j_bench64 300 python bench.py --steps 30 --warmup 5
step r4j_share8 300 python bench.py --steps 40 --warmup 5 --clients 8
QFEDX_HEA_CHUNKS=2 step r4j_share8_ch2 300 python bench.py --steps 40 --warmup 5 --clients 8
step r4j_prof8 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/prof7 -o share8 -- python3 bench.py --steps 20 --warmup 3 --clients 8
step r4j_prof64 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/prof7 -o full64 -- python3 bench.py --steps 10 --warmup 3
python3 scripts/round_timeline.py gpurun_out/prof7/share8_kernel_trace.csv | tee gpurun_out/r4j_share8_timeline.txt
python3 scripts/round_timeline.py gpurun_out/prof7/full64_kernel_trace.csv | tee gpurun_out/r4j_full64_timeline.txt
