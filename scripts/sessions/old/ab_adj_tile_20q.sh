#!/bin/bash
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
for r in 1 2; do for at in 13 14; do
  QFEDX_HEA_ADJ_TILE=$at timeout -k 10 200 python scripts/hea_kbench.py --iters 10 --qubits 20 --layers 2 --clients 32 --batch 32 > gpurun_out/adjt_$at$r.log 2>&1 || exit 1
  echo "adj$at r$r $(tail -1 gpurun_out/adjt_$at$r.log | cut -c1-400)"
done; done
