#!/bin/bash
# GPU tests of the training runtime (round graphs, gathers, noise trajectories, multi-rank, CFed).
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_noise.py tests/test_gpu_multirank.py \
  tests/test_gpu_qlayer.py tests/test_gpu_cnn.py -x -v --timeout 120 --timeout-method thread -p no:cacheprovider \
  > gpurun_out/trainer_tests.log 2>&1
rc=$?; tail -3 gpurun_out/trainer_tests.log; exit $rc
