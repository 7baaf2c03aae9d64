#!/bin/bash
# Round validation on one MI355X: GPU test suite -> smoke -> headline bench -> rocprofv3 kernel stats.
# Every GPU step has its own time limit; the script stops at the first failure.
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out/prof
step() {  # step <name> <seconds> <cmd...>
  local name=$1 secs=$2; shift 2
  timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc"; tail -4 "gpurun_out/$name.log"
  [ $rc -eq 0 ] || exit $rc
}
step gpu_tests 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -p no:cacheprovider
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
step bench 600 python bench.py --steps 20 --warmup 3
step prof_bench 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o bench -- python3 bench.py --steps 10 --warmup 2
# end-of-round suite: every BASELINE config line (config 5 = vqc24q_ps256_mfma), 10 timed rounds each
for c in cfed128 cfed128_epoch cfed128_secagg cfed128_secagg_sparse vqc16q_64_mfma vqc16q_64_mfma_secagg \
         vqc16q_64_mfma_secagg_sparse vqc16q_bf16_8_mfma vqc16q_fp16_8_mfma vqc20q_dp64_mfma vqc20q_ddp64_mfma \
         vqc24q_ps256_mfma vqc48q_mps64; do
  step suite_$c 600 python bench_suite.py --config $c --steps 10 --warmup 2
  grep '"metric"' gpurun_out/suite_$c.log >> gpurun_out/suite_lines.jsonl
done
