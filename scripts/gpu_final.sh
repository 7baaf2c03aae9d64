#!/bin/bash
# Round-end validation: full GPU suite + smoke + headline bench + kernel stats, then the per-rank 8-client share
# and the MFMA suite entries (every step time-limited; stop at the first failure).
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
bash scripts/gpu_round.sh || exit $?
timeout -k 10 300 python bench.py --steps 30 --warmup 5 --clients 8 > gpurun_out/share8.log 2>&1
rc=$?; echo "share8 rc=$rc"; grep '"metric"' gpurun_out/share8.log; [ $rc -eq 0 ] || exit $rc
STEPS=10 WARMUP=8 bash scripts/gpu_suite.sh vqc16q_64_mfma vqc20q_dp64_mfma vqc24q_ps256_mfma cfed128 cfed128_epoch
