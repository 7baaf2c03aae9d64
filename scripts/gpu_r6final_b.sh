#!/bin/bash
# Round 6 final validation, part B: every BASELINE config line of bench_suite.py (config 5 = vqc24q_ps256_mfma),
# 50 timed rounds each (config 5: 10).  Long steps keep a heartbeat file under gpurun_out/ so the run is not taken for hung.
source "$(dirname "$0")/gpu_step.sh"
rm -f gpurun_out/suite_lines.jsonl
for c in cfed128 cfed128_epoch cfed128_secagg cfed128_secagg_sparse vqc16q_64_mfma vqc16q_64_mfma_secagg \
         vqc16q_64_mfma_secagg_sparse vqc16q_bf16_8_mfma vqc16q_fp16_8_mfma vqc20q_dp64_mfma vqc20q_ddp64_mfma \
         vqc48q_mps64 vqc4q_2_cpu vqc24q_ps256_mfma; do
  ( while sleep 45; do date >> gpurun_out/heartbeat_$c.txt; done ) &
  hb=$!
  trap "kill $hb 2>/dev/null" EXIT
  # millisecond rounds: 50 timed after 20 warm-up rounds (10 rounds of ~2 ms sit inside the clock ramp);
  # config 5 (26 s rounds): 10 after 2
  if [ "$c" = vqc24q_ps256_mfma ]; then S=10; W=2; else S=50; W=20; fi
  TAILN=1 step suite_$c 600 python bench_suite.py --config $c --steps $S --warmup $W
  kill $hb
  grep '"metric"' gpurun_out/suite_$c.log >> gpurun_out/suite_lines.jsonl
done
