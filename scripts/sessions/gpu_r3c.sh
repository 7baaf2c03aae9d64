#!/bin/bash
# Full GPU suite + smoke + headline bench (RCCL single rank) + SecAgg/CFed suite + CFed kernel profile.
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out/profc gpurun_out/prof
step() {  # step <name> <seconds> <cmd...>
  local name=$1 secs=$2; shift 2
  timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc"; tail -3 "gpurun_out/$name.log"
  [ $rc -eq 0 ] || exit $rc
}
step gpu_tests 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
step bench 300 python bench.py --steps 20 --warmup 5
step bench_rccl 300 python bench.py --steps 20 --warmup 5 --dist-backend nccl
step share8 300 python bench.py --steps 30 --warmup 5 --clients 8
STEPS=10 WARMUP=8 bash scripts/gpu_suite.sh vqc16q_64_mfma_secagg cfed128 cfed128_secagg || exit 1
step prof_cfed 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/profc -o cfed -- python3 bench_suite.py --config cfed128 --steps 10 --warmup 3
python3 scripts/prof_summary.py gpurun_out/profc/cfed_kernel_trace.csv > gpurun_out/profc/summary.txt
python3 scripts/round_timeline.py gpurun_out/profc/cfed_kernel_trace.csv > gpurun_out/profc/timeline.txt; cat gpurun_out/profc/timeline.txt
bash scripts/gpu_abl2.sh
