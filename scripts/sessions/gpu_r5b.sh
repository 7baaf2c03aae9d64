#!/bin/bash
# Round 5, call 2: after deleting the rejected variants -- GPU suite, headline + 8-client bench, stall attribution
# (stamps build), fused-readout A/B at 64 and 8 clients.  Every GPU step time-limited; stop at the first failure.
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r5b
step() {  # step <name> <seconds> <cmd...>
  local name=$1 secs=$2; shift 2
  timeout -k 10 "$secs" "$@" > "gpurun_out/r5b/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc"; tail -3 "gpurun_out/r5b/$name.log" | cut -c1-600
  [ $rc -eq 0 ] || exit $rc
}
step gpu_tests 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider
step bench64 300 python bench.py --steps 20 --warmup 3
step share8 300 python bench.py --steps 30 --warmup 5 --clients 8
step stamps64 300 python -u scripts/hea_stamps.py --clients 64 --out gpurun_out/r5b/stamps64.jsonl
step stamps8 300 python -u scripts/hea_stamps.py --clients 8 --out gpurun_out/r5b/stamps8.jsonl
step ab_ro64 300 python -u scripts/hea_ab.py --rounds 7 --variants "sep:env.QFEDX_FUSED_READOUT=0,fused:env.QFEDX_FUSED_READOUT=1"
step ab_ro8 300 python -u scripts/hea_ab.py --rounds 7 --clients 8 --iters 30 --variants "sep:env.QFEDX_FUSED_READOUT=0,fused:env.QFEDX_FUSED_READOUT=1"
