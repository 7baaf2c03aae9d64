#!/bin/bash
# GPU suite (fc1 kernels, RCCL single rank, CFed rank invariance) + HEA per-op ablation timings + CFed bench.
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_rccl.py tests/test_gpu_simulator.py tests/test_gpu_kernels.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -k "rccl or simulator or norms_ride" > gpurun_out/gpu_tests.log 2>&1
rc=$?; echo "gpu_tests rc=$rc"; tail -3 gpurun_out/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  for m in 0 1 2 4 8 3 12; do
    QFEDX_HEA_ABLATE=$m QFX_PKG_ROOT=$PWD/ab/abl timeout -k 10 200 python scripts/hea_kbench.py --iters 20 --clients 64 > gpurun_out/abl_${m}_$r.log 2>&1 || exit 1
    echo "abl=$m r$r $(tail -1 gpurun_out/abl_${m}_$r.log)"
  done
done
STEPS=10 WARMUP=8 bash scripts/gpu_suite.sh cfed128 cfed128_epoch vqc16q_64_mfma vqc16q_64_mfma_secagg cfed128_secagg
