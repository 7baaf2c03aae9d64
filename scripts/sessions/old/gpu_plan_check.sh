#!/bin/bash
# Planner change check: MFMA numerics tests, kernel timing at 16q x 3L and 20q x 2L, then the 20q DP suite entry.
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_hea.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/hea_tests.log 2>&1
rc=$?; echo "hea_tests rc=$rc"; tail -2 gpurun_out/hea_tests.log; [ $rc -eq 0 ] || exit $rc
for cfg in "16 3 64 32" "20 2 64 8"; do
  set -- $cfg
  for T in 0 auto; do
    out=$(QFEDX_HEA_TRIM=$T timeout -k 10 300 python scripts/hea_kbench.py --qubits $1 --layers $2 --clients $3 --batch $4 --iters 10 2>/dev/null | grep step_ms)
    rc=$?; [ $rc -eq 0 ] || { echo "kbench q=$1 rc=$rc"; exit $rc; }
    echo "q=$1 L=$2 trim=$T $out" | tee -a gpurun_out/plan_check.log
  done
done
bash scripts/gpu_suite.sh vqc20q_dp64_mfma
