#!/bin/bash
# Round 4, call 11: step-0 fragments on a parallel graph branch (QFEDX_FRAG_BRANCH), the single-rank FedAvg
# reduce that applies the round itself (QFEDX_FUSED_APPLY) and the upload merged into the prologue launch
# (QFEDX_ROUND_START): GPU tests, interleaved share-8 A/B, headline A/B, CFed A/B, share-8 timeline.
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out/prof8
timeout -k 10 700 python -u -m pytest -x -q --timeout 200 --timeout-method thread -p no:cacheprovider -m gpu tests/test_gpu_kernels.py tests/test_gpu_hea.py tests/test_gpu_amplitude.py tests/test_gpu_rccl.py > gpurun_out/r4k_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r4k_tests.log; [ $rc -eq 0 ] || exit $rc
step() {
  local name=$1 secs=$2; shift 2
  timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc"; grep '"metric"' "gpurun_out/$name.log" | cut -c1-200
  [ $rc -eq 0 ] || exit $rc
}
for rep in 1 2; do
  QFEDX_FRAG_BRANCH=0 QFEDX_FUSED_APPLY=0 QFEDX_ROUND_START=0 step r4k_share8_base$rep 200 python bench.py --steps 40 --warmup 5 --clients 8
  QFEDX_FRAG_BRANCH=1 QFEDX_FUSED_APPLY=0 QFEDX_ROUND_START=0 step r4k_share8_br$rep 200 python bench.py --steps 40 --warmup 5 --clients 8
  QFEDX_FRAG_BRANCH=0 QFEDX_FUSED_APPLY=1 QFEDX_ROUND_START=0 step r4k_share8_fa$rep 200 python bench.py --steps 40 --warmup 5 --clients 8
  QFEDX_FRAG_BRANCH=0 QFEDX_FUSED_APPLY=0 QFEDX_ROUND_START=1 step r4k_share8_rs$rep 200 python bench.py --steps 40 --warmup 5 --clients 8
  step r4k_share8_all$rep 200 python bench.py --steps 40 --warmup 5 --clients 8
done
QFEDX_FRAG_BRANCH=0 QFEDX_FUSED_APPLY=0 QFEDX_ROUND_START=0 step r4k_bench64_base 300 python bench.py --steps 30 --warmup 5
step r4k_bench64_all 300 python bench.py --steps 30 --warmup 5
QFEDX_FUSED_APPLY=0 step r4k_cfed_base 300 python bench_suite.py --config cfed128 --steps 30 --warmup 5
step r4k_cfed_fa 300 python bench_suite.py --config cfed128 --steps 30 --warmup 5
step r4k_prof8 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/prof8 -o share8 -- python3 bench.py --steps 20 --warmup 3 --clients 8
python3 scripts/round_timeline.py gpurun_out/prof8/share8_kernel_trace.csv | tee gpurun_out/r4k_share8_timeline.txt
