#!/bin/bash
# Round-3 validation + measurement in one call: GPU suite (test failures do not stop the run; faults, aborts and
# time limits do), smoke, kernel A/B (adjoint compile-time block counts), headline bench (+ RCCL, 8-client share),
# rocprof kernel trace of the headline, SecAgg / CFed / 24q param-shift suite lines, PMC counters of the passes.
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out/prof gpurun_out/pmcn
step() {  # step <name> <seconds> <cmd...>; pytest rc 1 (failed tests) continues, any other failure ends the run
  local name=$1 secs=$2; shift 2
  timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc"; tail -3 "gpurun_out/$name.log"
  if [ $rc -ne 0 ]; then
    if [ "$name" = gpu_tests ] && [ $rc -eq 1 ]; then return 0; fi
    exit $rc
  fi
}
step gpu_tests 900 python -u -m pytest tests -m gpu -q --maxfail=8 --timeout 120 --timeout-method thread -p no:cacheprovider
grep -E "^(FAILED|ERROR)" gpurun_out/gpu_tests.log | head -20
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
step kbench 300 python scripts/hea_kbench.py --iters 10
QFEDX_HEA_ADJ_FULL=1 step kbench_full 300 python scripts/hea_kbench.py --iters 10
step bench 300 python bench.py --steps 20 --warmup 5
QFEDX_HEA_ADJ_FULL=1 step bench_full 300 python bench.py --steps 20 --warmup 5
step bench_rccl 300 python bench.py --steps 20 --warmup 5 --dist-backend nccl
step share8 300 python bench.py --steps 30 --warmup 5 --clients 8
step prof_bench 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o bench -- python3 bench.py --steps 10 --warmup 3
python3 scripts/prof_summary.py gpurun_out/prof/bench_kernel_trace.csv > gpurun_out/prof/bench_summary.txt
python3 scripts/round_timeline.py gpurun_out/prof/bench_kernel_trace.csv > gpurun_out/prof/bench_timeline.txt
head -12 gpurun_out/prof/bench_summary.txt
i=0
for set in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_MFMA SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_WAVE_CYCLES" \
           "SQ_WAVES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_ANY SQ_INSTS_VMEM_RD SQ_INSTS_SALU" \
           "FETCH_SIZE GRBM_GUI_ACTIVE" "WRITE_SIZE GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  step pmc$i 90 rocprofv3 --kernel-trace --pmc $set --output-format csv -d gpurun_out/pmcn -o set$i -- python3 scripts/hea_kbench.py --iters 2
done
for i in 1 2 3 4; do python3 scripts/pmc_summary.py gpurun_out/pmcn/set${i}_counter_collection.csv | grep -E "hea_(adj|fwd)"; done > gpurun_out/pmcn/summary.txt
STEPS=10 WARMUP=8 bash scripts/gpu_suite.sh vqc16q_64_mfma_secagg cfed128 cfed128_secagg || exit 1
STEPS=1 WARMUP=1 bash scripts/gpu_suite.sh vqc24q_ps256_mfma || exit 1
