#!/bin/bash
# Round 4, call 16: FedAvg reduce with 8 client rows in flight per thread (128 clients: one batch): kernel tests,
# CFed bench + kernel trace, headline bench.
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out/prof10
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -p no:cacheprovider -m gpu tests/test_gpu_kernels.py -k "fedavg or secagg or graph_round or dp_client" > gpurun_out/r4p_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r4p_tests.log; [ $rc -eq 0 ] || exit $rc
step() {
  local name=$1 secs=$2; shift 2
  timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc"; grep '"metric"' "gpurun_out/$name.log" | grep -o '"ms_per_step": [0-9.]*'
  [ $rc -eq 0 ] || exit $rc
}
step r4p_cfed1 200 python bench_suite.py --config cfed128 --steps 30 --warmup 5
step r4p_cfed2 200 python bench_suite.py --config cfed128 --steps 30 --warmup 5
step r4p_bench64 200 python bench.py --steps 30 --warmup 5
step r4p_cfedprof 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/prof10 -o cfed -- python3 bench_suite.py --config cfed128 --steps 10 --warmup 3
python3 scripts/round_timeline.py gpurun_out/prof10/cfed_kernel_trace.csv
