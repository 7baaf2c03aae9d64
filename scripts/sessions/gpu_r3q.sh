#!/bin/bash
# FedAvg reduce with 16 client groups per block: full GPU suite + smoke + headline bench, then CFed suite lines.
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
bash scripts/gpu_round.sh || exit $?
timeout -k 10 300 python bench.py --steps 30 --warmup 5 --clients 8 > gpurun_out/share8.log 2>&1 || exit 1
grep '"metric"' gpurun_out/share8.log | cut -c1-200
STEPS=10 WARMUP=5 bash scripts/gpu_suite.sh cfed128 vqc20q_dp64_mfma
