#!/bin/bash
# Round 5, call 17: stall table with the first forward pass's layer-1 generation split into sub-phases (GEN1, GEN2).
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r5q
timeout -k 10 300 python -u scripts/hea_stamps.py --clients 64 --out gpurun_out/r5q/stamps64.jsonl > gpurun_out/r5q/stamps64.log 2>&1
rc=$?; echo "stamps64 rc=$rc"; tail -45 gpurun_out/r5q/stamps64.log
