#!/bin/bash
# Round 6: host-side key derivation change - GPU tests that draw per-client keys (DP, dropout, noise), then the CFed
# lines with their host time
source "$(dirname "$0")/gpu_step.sh"
step keys_tests 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_cnn.py tests/test_gpu_kernels.py tests/test_gpu_noise.py
for c in cfed128 cfed128_secagg_sparse vqc20q_dp64_mfma; do
  TAILN=0 step hk_$c 300 python bench_suite.py --config $c --steps 30 --warmup 3
  echo "$c $(grep '"metric"' gpurun_out/hk_$c.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], 'ms/round, host', d['host_ms_per_round'], 'ms')")"
done
