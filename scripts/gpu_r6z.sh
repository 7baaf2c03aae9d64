#!/bin/bash
# Round 6: XCD-contiguous pass workgroups (QFX_HEA_XCD) - interleaved headline and 8-client bench.py runs of the
# ab/base and ab/new trees (50 timed rounds after 20 warm-up).
source "$(dirname "$0")/gpu_step.sh"
for r in 1 2 3; do for v in base new; do
  (cd ab/$v && timeout -k 10 300 python bench.py --steps 50 --warmup 20 > ../../gpurun_out/xcd_${v}$r.log 2>&1) || { echo "xcd_${v}$r failed"; tail -5 gpurun_out/xcd_${v}$r.log; exit 1; }
  (cd ab/$v && timeout -k 10 300 python bench.py --steps 50 --warmup 20 --clients 8 > ../../gpurun_out/xcd8_${v}$r.log 2>&1) || { echo "xcd8_${v}$r failed"; exit 1; }
  echo "$v $r $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/xcd_${v}$r.log) | 8 clients $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/xcd8_${v}$r.log) $(grep -o '"max_abs_err_grad": [0-9.e-]*' gpurun_out/xcd_${v}$r.log)"
done; done
