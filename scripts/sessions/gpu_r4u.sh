#!/bin/bash
# Round 4, call 22: end-of-round bench_suite lines (every GPU config short of the 30 s param-shift one): JSON lines
# collected into gpurun_out/r4u_suite.jsonl.
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
: > gpurun_out/r4u_suite.jsonl
for c in cfed128 cfed128_epoch cfed128_secagg cfed128_secagg_sparse vqc16q_64_mfma vqc16q_64_mfma_secagg \
         vqc16q_64_mfma_secagg_sparse vqc16q_bf16_8 vqc16q_fp16_8_mfma vqc20q_dp64_mfma vqc48q_mps64; do
  timeout -k 10 240 python bench_suite.py --config $c --steps 10 --warmup 3 > gpurun_out/r4u_$c.log 2>&1
  rc=$?; echo "$c rc=$rc"
  [ $rc -eq 0 ] || { tail -5 gpurun_out/r4u_$c.log; exit $rc; }
  grep '"metric"' gpurun_out/r4u_$c.log >> gpurun_out/r4u_suite.jsonl
  grep '"metric"' gpurun_out/r4u_$c.log | grep -o '"ms_per_step": [0-9.]*'
done
