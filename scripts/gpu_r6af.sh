#!/bin/bash
# Round 6: fused Adam epilogue as per-block owned updates - the whole GPU suite on the new tree, interleaved
# bench.py runs (8 and 64 clients, 50 timed rounds after 20 warm-up) of ab/base and ab/new, kernel traces at 8 clients.
source "$(dirname "$0")/gpu_step.sh"
step t_all 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider
for r in 1 2 3; do for v in base new; do
  (cd ab/$v && timeout -k 10 300 python bench.py --clients 8 --steps 50 --warmup 20 > ../../gpurun_out/ad8_${v}$r.log 2>&1) || { echo "ad8_${v}$r failed"; exit 1; }
  (cd ab/$v && timeout -k 10 300 python bench.py --steps 50 --warmup 20 > ../../gpurun_out/ad64_${v}$r.log 2>&1) || { echo "ad64_${v}$r failed"; exit 1; }
  echo "$v $r 8c $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/ad8_${v}$r.log) 64c $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/ad64_${v}$r.log) $(grep -o '"max_abs_err_grad": [0-9.e-]*' gpurun_out/ad64_${v}$r.log)"
done; done
for v in base new; do
  (cd ab/$v && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d ../../gpurun_out/ad_prof_$v -o k -- python3 bench.py --clients 8 --steps 20 --warmup 5 > ../../gpurun_out/ad_prof_$v.log 2>&1) || exit 1
done
