#!/bin/bash
# Round 6: FedAvg reduce with 4 parameters per thread (FA_X) at two blocks per CU - interleaved cfed128 suite lines of the
# ab/base and ab/new trees (50 timed rounds after 20 warm-up), then a kernel trace of each.
source "$(dirname "$0")/gpu_step.sh"
step t_fa 400 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_cnn.py -m gpu -x -v --timeout 120 --timeout-method thread -p no:cacheprovider -k "fedavg or secagg or reduce or round or cfed or cnn"
for r in 1 2 3; do for v in base new; do
  (cd ab/$v && timeout -k 10 300 python bench_suite.py --config cfed128 --steps 50 --warmup 20 > ../../gpurun_out/fax_${v}$r.log 2>&1) || { echo "fax_${v}$r failed"; tail -5 gpurun_out/fax_${v}$r.log; exit 1; }
  echo "$v $r $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/fax_${v}$r.log)"
done; done
for v in base new; do
  (cd ab/$v && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d ../../gpurun_out/fax_prof_$v -o k -- python3 bench_suite.py --config cfed128 --steps 10 --warmup 3 > ../../gpurun_out/fax_prof_$v.log 2>&1) || exit 1
  grep -h "fedavg_reduce" gpurun_out/fax_prof_$v/k_kernel_stats.csv | cut -c1-60,200-260
done
