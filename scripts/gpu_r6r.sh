#!/bin/bash
# Round 6: host time per round of every suite line (is any config host-bound?)
source "$(dirname "$0")/gpu_step.sh"
for c in cfed128 cfed128_secagg_sparse vqc16q_64_mfma vqc16q_64_mfma_secagg_sparse vqc16q_bf16_8_mfma vqc20q_dp64_mfma vqc20q_ddp64_mfma vqc48q_mps64; do
  TAILN=0 step hm_$c 300 python bench_suite.py --config $c --steps 20 --warmup 3
  echo "$c $(grep '"metric"' gpurun_out/hm_$c.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], 'ms/round, host', d['host_ms_per_round'], 'ms')")"
done
