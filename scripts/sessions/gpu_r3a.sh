#!/bin/bash
# Round-3 first validation: GPU suite, smoke, headline bench (+ profile), 8-client share, CFed 128.
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
bash scripts/gpu_round.sh || exit $?
timeout -k 10 300 python bench.py --steps 30 --warmup 5 --clients 8 > gpurun_out/share8.log 2>&1
rc=$?; echo "share8 rc=$rc"; grep '"metric"' gpurun_out/share8.log; [ $rc -eq 0 ] || exit $rc
STEPS=10 WARMUP=8 bash scripts/gpu_suite.sh cfed128
