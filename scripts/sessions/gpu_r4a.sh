#!/bin/bash
# Round 4, call 1: headline bench, OP_L1PROD poison diagnostics, the new GPU tests (bf16 MFMA engine, SecAgg 32-bit
# and sparse graph, captured-collective self-check), config-2 suite lines.
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/r4a_bench.log 2>&1 || { tail -20 gpurun_out/r4a_bench.log; exit 1; }
grep '"metric"' gpurun_out/r4a_bench.log | cut -c1-600
timeout -k 10 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_hea.py::test_hea_vjp_matches_dense_bf16 tests/test_gpu_rccl.py tests/test_gpu_cnn.py \
  "tests/test_gpu_kernels.py::test_secagg_sparse_graph_in_fused_reduce_match_host_protocol" \
  "tests/test_gpu_kernels.py::test_secagg_masks_in_fused_reduce_match_host_protocol" > gpurun_out/r4a_tests.log 2>&1
rc=$?; grep -E "PASS|FAIL|Error|passed|failed" gpurun_out/r4a_tests.log | tail -20; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u scripts/hea_ab.py --variants "w8:adj_waves=8,w8f:adj_waves=8;full13=1,w4:adj_waves=4;full13=0,bf16w8:storage=bf16;adj_waves=8;full13=0" > gpurun_out/r4a_ab.log 2>&1 || { tail -20 gpurun_out/r4a_ab.log; exit 1; }
tail -1 gpurun_out/r4a_ab.log
STEPS=10 WARMUP=3 bash scripts/gpu_suite.sh vqc16q_bf16_8 vqc16q_fp16_8_mfma cfed128 || exit 1
for p in 0 0x7e007e00 0x3c003c00; do
  QFEDX_HEA_POISON=$p timeout -k 10 300 python -u scripts/l1prod_poison.py > gpurun_out/r4a_poison_$p.log 2>&1 || { tail -20 gpurun_out/r4a_poison_$p.log; exit 1; }
  grep '"n"' gpurun_out/r4a_poison_$p.log
done
