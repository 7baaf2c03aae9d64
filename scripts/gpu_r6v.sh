#!/bin/bash
# Round 6: fused-readout MPS chain training launch - MPS GPU tests, then interleaved vqc48q_mps64 suite lines.
source "$(dirname "$0")/gpu_step.sh"
step mps_tests 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_mps_chain.py tests/test_gpu_mps.py
for r in 1 2 3; do for v in base new; do
  (cd ab/$v && timeout -k 10 300 python bench_suite.py --config vqc48q_mps64 --steps 30 --warmup 3 > ../../gpurun_out/mpsab_${v}$r.log 2>&1) || { echo "mpsab_${v}$r failed"; tail -5 gpurun_out/mpsab_${v}$r.log; exit 1; }
  echo "$v $r $(grep '"metric"' gpurun_out/mpsab_${v}$r.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], 'ms, host', d.get('host_ms_per_round'), 'acc', d['test_acc_after'])")"
done; done
