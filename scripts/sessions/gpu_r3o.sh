#!/bin/bash
# OP_L1PROD (layer-1 gradients of the last adjoint pass from the closed-form product state): MFMA-engine GPU tests,
# then the kernel-step A/B QFEDX_HEA_L1PROD=1 vs 0, interleaved on one box, with errors vs the fp32 VALU engine.
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
step() {
  local name=$1 secs=$2; shift 2
  timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc"; tail -2 "gpurun_out/$name.log"
  [ $rc -eq 0 ] || exit $rc
}
step hea_tests 600 python -u -m pytest tests/test_gpu_hea.py tests/test_gpu_paramshift.py tests/test_gpu_kernels.py -q -x --timeout 120 --timeout-method thread -p no:cacheprovider
for v in 1 0 1 0; do
  QFEDX_HEA_L1PROD=$v step kb_l1p$v 300 python scripts/hea_kbench.py --iters 20 --precision
done
