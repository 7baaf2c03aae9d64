#!/bin/bash
# A/B of the MFMA pass planner: greedy (QFEDX_HEA_TRIM=0) vs trimmed (=1) plans at 20 and 24 qubits, interleaved.
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
for rep in 1 2; do
  for cfg in "20 16 32" "24 16 8"; do
    set -- $cfg
    for T in 0 1; do
      out=$(QFEDX_HEA_TRIM=$T timeout -k 10 300 python scripts/hea_kbench.py --qubits $1 --clients $2 --batch $3 --iters 10 2>/dev/null | grep step_ms)
      rc=$?; [ $rc -eq 0 ] || { echo "q=$1 trim=$T rc=$rc"; exit $rc; }
      echo "q=$1 trim=$T $out" | tee -a gpurun_out/ab_trim.log
    done
  done
done
