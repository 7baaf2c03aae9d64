#!/bin/bash
# Train-kernel numerics + CNN numerics, then the CFed suite and kernel stats.
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kernels.py > gpurun_out/kern_tests.log 2>&1 || { tail -40 gpurun_out/kern_tests.log; exit 1; }
tail -2 gpurun_out/kern_tests.log
bash scripts/gpu_cnn_iter.sh
