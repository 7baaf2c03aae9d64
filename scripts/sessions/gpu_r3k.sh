#!/bin/bash
# Transposed BACK ops (cross matrix at the op input): MFMA-engine GPU tests, then kernel-step A/B
# QFEDX_HEA_TRANS=1 (default) vs 0 (output-side fused cross), interleaved on one box.
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
step() {  # step <name> <seconds> <cmd...>; pytest rc 1 (failed tests) continues, any other failure ends the run
  local name=$1 secs=$2; shift 2
  timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc"; tail -2 "gpurun_out/$name.log"
  if [ $rc -ne 0 ]; then
    if [ "$name" = hea_tests ] && [ $rc -eq 1 ]; then return 0; fi
    exit $rc
  fi
}
mkdir -p gpurun_out
step hea_tests 600 python -u -m pytest tests/test_gpu_hea.py tests/test_gpu_paramshift.py -q -x --timeout 120 --timeout-method thread -p no:cacheprovider
grep -E "^(FAILED|ERROR)" gpurun_out/hea_tests.log | head -20
for v in 1 0 1 0; do
  QFEDX_HEA_TRANS=$v step kb_t$v 300 python scripts/hea_kbench.py --iters 10
done
