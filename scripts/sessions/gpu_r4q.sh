#!/bin/bash
# Round 4, call 17: FedAvg reduce with 4 parameters per thread (16-byte row loads) for large P: kernel tests (exact
# fixed-point sums on both layouts), CFed bench + kernel trace, CFed SecAgg, headline bench.
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out/prof11
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -p no:cacheprovider -m gpu tests/test_gpu_kernels.py tests/test_gpu_cnn.py > gpurun_out/r4q_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r4q_tests.log; [ $rc -eq 0 ] || exit $rc
step() {
  local name=$1 secs=$2; shift 2
  timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc"; grep '"metric"' "gpurun_out/$name.log" | grep -o '"ms_per_step": [0-9.]*'
  [ $rc -eq 0 ] || exit $rc
}
step r4q_cfed1 200 python bench_suite.py --config cfed128 --steps 30 --warmup 5
step r4q_cfed2 200 python bench_suite.py --config cfed128 --steps 30 --warmup 5
step r4q_cfed_sa 200 python bench_suite.py --config cfed128_secagg --steps 20 --warmup 3
step r4q_cfed_sas 200 python bench_suite.py --config cfed128_secagg_sparse --steps 20 --warmup 3
step r4q_bench64 200 python bench.py --steps 30 --warmup 5
step r4q_cfedprof 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/prof11 -o cfed -- python3 bench_suite.py --config cfed128 --steps 10 --warmup 3
python3 scripts/round_timeline.py gpurun_out/prof11/cfed_kernel_trace.csv
grep -h "fedavg_reduce" gpurun_out/prof11/cfed_kernel_trace.csv | head -1 | tr ',' '\n' | sed -n '12,20p'
