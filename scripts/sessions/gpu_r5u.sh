#!/bin/bash
# Round 5, call 21: the last local Adam step deferred into the plain FedAvg reduce when the gradient reduction cannot
# fuse it (64 clients): kernel tests (bitwise vs the separate launches), then the headline bench and timeline with the
# deferral on / off (QFEDX_FED_TAIL=0 turns the plain-round folds off), and PMC of the CFed round's kernels.
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r5u
step() {  # step <name> <seconds> <cmd...>
  local name=$1 secs=$2; shift 2
  timeout -k 10 "$secs" "$@" > "gpurun_out/r5u/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc"; tail -2 "gpurun_out/r5u/$name.log" | cut -c1-300
  [ $rc -eq 0 ] || exit $rc
}
step tests 600 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_multirank.py -x -q --timeout 200 --timeout-method thread -p no:cacheprovider
for i in a b c; do
  step bench64_on_$i 300 python bench.py --steps 20 --warmup 3
  step bench64_off_$i 300 env QFEDX_FED_TAIL=0 python bench.py --steps 20 --warmup 3
done
step prof64 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r5u/prof64 -o bench -- python3 bench.py --steps 10 --warmup 3
python3 scripts/round_timeline.py gpurun_out/r5u/prof64/bench_kernel_trace.csv --marker qfx_round_prologue_kernel > gpurun_out/r5u/timeline64.txt 2>&1
cat gpurun_out/r5u/timeline64.txt
timeout -s KILL 150 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_MFMA SQ_ACTIVE_INST_LDS --output-format csv -d gpurun_out/r5u -o seta -- python3 bench_suite.py --config cfed128 --steps 2 --warmup 1 > gpurun_out/r5u/seta.log 2>&1
rc=$?; echo "pmc rc=$rc"; [ $rc -eq 0 ] || exit $rc
python3 scripts/pmc_summary.py gpurun_out/r5u/seta_counter_collection.csv > gpurun_out/r5u/seta_summary.txt 2>&1
cut -c1-300 gpurun_out/r5u/seta_summary.txt
