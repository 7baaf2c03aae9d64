#!/bin/bash
# Round 4, call 20: FusedApply counter allocated outside the round-graph capture (no captured fill node): graph /
# fused-apply GPU tests, share-8 and headline benches, share-8 timeline.
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out/prof12
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -p no:cacheprovider -m gpu tests/test_gpu_kernels.py tests/test_gpu_rccl.py > gpurun_out/r4s_tests.log 2>&1
rc=$?; tail -2 gpurun_out/r4s_tests.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  timeout -k 10 200 python bench.py --steps 40 --warmup 5 --clients 8 > gpurun_out/r4s_share8_$r.log 2>&1 || exit 1
  grep -o '"ms_per_step": [0-9.]*' gpurun_out/r4s_share8_$r.log
  timeout -k 10 200 python bench.py --steps 40 --warmup 5 > gpurun_out/r4s_bench64_$r.log 2>&1 || exit 1
  grep -o '"ms_per_step": [0-9.]*' gpurun_out/r4s_bench64_$r.log
done
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/prof12 -o share8 -- python3 bench.py --steps 20 --warmup 3 --clients 8 > gpurun_out/r4s_prof8.log 2>&1 || exit 1
python3 scripts/round_timeline.py gpurun_out/prof12/share8_kernel_trace.csv --marker qfx_fedavg_reduce_kernel | tee gpurun_out/r4s_share8_timeline.txt
