#!/bin/bash
# Iteration run: kernel numerics tests, then a rocprofv3 kernel-trace profile of the bench.
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out/prof
timeout -k 10 900 python -m pytest tests/test_gpu_kernels.py -x -q -p no:cacheprovider > gpurun_out/gpu_tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -15 gpurun_out/gpu_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o bench -- python3 bench.py --steps 3 --warmup 1 "$@" > gpurun_out/prof_bench.log 2>&1
rc=$?; echo "prof rc=$rc"; grep '"metric"' gpurun_out/prof_bench.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python bench.py --steps 5 --warmup 2 "$@" > gpurun_out/bench.log 2>&1
rc=$?; echo "bench rc=$rc"; cat gpurun_out/bench.log | grep metric
exit $rc
