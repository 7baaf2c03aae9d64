#!/bin/bash
# CFed CNN kernels: numerics tests, then the cfed128 suite timing and per-kernel stats.
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out/profc
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_cnn.py > gpurun_out/cnn_tests.log 2>&1 || { tail -40 gpurun_out/cnn_tests.log; exit 1; }
tail -3 gpurun_out/cnn_tests.log
STEPS=10 WARMUP=3 bash scripts/gpu_suite.sh cfed128 cfed128_epoch || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/profc -o cfed -- python3 bench_suite.py --config cfed128 --steps 10 --warmup 3 > gpurun_out/profc.log 2>&1 || exit 1
python3 scripts/prof_summary.py gpurun_out/profc/cfed_kernel_trace.csv | head -12
