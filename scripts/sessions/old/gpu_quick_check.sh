#!/bin/bash
# Quick GPU check of a change: the kernel/round tests, then the headline and 8-client-share benches.
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest ${TESTS:-tests/test_gpu_kernels.py tests/test_gpu_hea.py tests/test_gpu_multirank.py tests/test_gpu_debug_build.py} \
  -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/quick_tests.log 2>&1
rc=$?; tail -3 gpurun_out/quick_tests.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do for cl in 64 8; do
  timeout -k 10 300 python bench.py --steps 40 --warmup 5 --clients $cl > gpurun_out/qb_${cl}_$r.log 2>&1 || exit 1
  echo "clients=$cl r=$r $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/qb_${cl}_$r.log)"
done; done
