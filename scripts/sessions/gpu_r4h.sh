#!/bin/bash
# Round 4, call 8: fused readout (first adjoint pass + grad-reduce readout block): HEA + kernel GPU tests, headline
# and 8-client share benches with kernel-trace timelines, SecAgg suite lines with the cached SecAgg+ tables.
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out/prof5
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider -m gpu tests/ > gpurun_out/r4h_tests.log 2>&1
rc=$?; tail -4 gpurun_out/r4h_tests.log; [ $rc -eq 0 ] || exit $rc
step() {
  local name=$1 secs=$2; shift 2
  timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc"; grep '"metric"' "gpurun_out/$name.log" | cut -c1-300
  [ $rc -eq 0 ] || exit $rc
}
step r4h_bench64 300 python bench.py --steps 30 --warmup 5
step r4h_share8 300 python bench.py --steps 40 --warmup 5 --clients 8
step r4h_prof8 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/prof5 -o share8 -- python3 bench.py --steps 20 --warmup 3 --clients 8
python3 scripts/round_timeline.py gpurun_out/prof5/share8_kernel_trace.csv | tee gpurun_out/r4h_share8_timeline.txt
STEPS=20 WARMUP=3 bash scripts/gpu_suite.sh cfed128 cfed128_secagg_sparse vqc16q_64_mfma_secagg_sparse vqc16q_64_mfma_secagg || exit 1
