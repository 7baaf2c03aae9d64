#!/bin/bash
# Round 4, call 13: fused single-rank apply without per-block releases: kernel tests, interleaved CFed and share-8
# A/B (QFEDX_FUSED_APPLY=0/1), headline bench.
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -p no:cacheprovider -m gpu tests/test_gpu_kernels.py > gpurun_out/r4m_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r4m_tests.log; [ $rc -eq 0 ] || exit $rc
step() {
  local name=$1 secs=$2; shift 2
  timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc"; grep '"metric"' "gpurun_out/$name.log" | grep -o '"ms_per_step": [0-9.]*'
  [ $rc -eq 0 ] || exit $rc
}
for rep in 1 2 3; do
  QFEDX_FUSED_APPLY=0 step r4m_cfed_off$rep 200 python bench_suite.py --config cfed128 --steps 30 --warmup 5
  QFEDX_FUSED_APPLY=1 step r4m_cfed_on$rep 200 python bench_suite.py --config cfed128 --steps 30 --warmup 5
  QFEDX_FUSED_APPLY=0 step r4m_share8_off$rep 200 python bench.py --steps 40 --warmup 5 --clients 8
  QFEDX_FUSED_APPLY=1 step r4m_share8_on$rep 200 python bench.py --steps 40 --warmup 5 --clients 8
done
step r4m_bench64 300 python bench.py --steps 30 --warmup 5
