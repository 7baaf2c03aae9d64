#!/bin/bash
# Round 6: CNN GPU tests with the split-fp16 conv2 forward (float64 autograd reference)
source "$(dirname "$0")/gpu_step.sh"
step cnn_tests 500 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_cnn.py tests/test_gpu_kernels.py
