#!/bin/bash
# Round 6: FedAvg reduce with 8 client rows in flight per thread (FA_U) - interleaved cfed128 suite lines of the
# ab/base and ab/new trees (50 timed rounds after 20 warm-up), then a kernel trace of each.
source "$(dirname "$0")/gpu_step.sh"
for r in 1 2 3; do for v in base new; do
  (cd ab/$v && timeout -k 10 300 python bench_suite.py --config cfed128 --steps 50 --warmup 20 > ../../gpurun_out/fau_${v}$r.log 2>&1) || { echo "fau_${v}$r failed"; tail -5 gpurun_out/fau_${v}$r.log; exit 1; }
  echo "$v $r $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/fau_${v}$r.log)"
done; done
for v in base new; do
  (cd ab/$v && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d ../../gpurun_out/fau_prof_$v -o k -- python3 bench_suite.py --config cfed128 --steps 10 --warmup 3 > ../../gpurun_out/fau_prof_$v.log 2>&1) || exit 1
  grep -h "fedavg_reduce" gpurun_out/fau_prof_$v/k_kernel_stats.csv | cut -c1-60,200-260
done
