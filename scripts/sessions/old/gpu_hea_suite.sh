#!/bin/bash
# MFMA engine tests, then the MFMA suite entries (24q param-shift, 20q DP with a longer warm-up for the Poisson
# client-count graph buckets, headline).
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_hea.py tests/test_gpu_kernels.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/hea_tests.log 2>&1; rc=$?; tail -2 gpurun_out/hea_tests.log; [ $rc -eq 0 ] || exit $rc
STEPS=3 WARMUP=1 bash scripts/gpu_suite.sh vqc24q_ps256_mfma || exit 1
STEPS=10 WARMUP=8 bash scripts/gpu_suite.sh vqc20q_dp64_mfma || exit 1
